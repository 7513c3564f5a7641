#!/bin/bash
# Alternating A/B runs on the GPU box (through gpurun): the one parameterised driver for every A/B.
#   bash tools/ab.sh TAG REPS KIND VARIANT...
# KIND: dense  -> bench.py encode only (--steps 100, no extras)
#       sparse -> tools/bench_sparse.py --reps 10 --aggregate 8 (8 distinct C3 payloads)
#       dsum   -> tools/bench_decode_sum.py
#       gap    -> tools/leaf_gap.py --steps 20 --reps 2 (gap26 / gap24: at 2^26 / 2^24 floats)
#       restore -> tools/bench_sparse.py --only-decode (restore of one C3 payload)
#       batch  -> tools/batch_probe.py (skml_dense_encode_batch_f32, 8 x 2^26 floats)
#       sparse_enc -> tools/bench_sparse.py --only-e2e (C3 dense -> payload)
# VARIANT: name=SETTINGS, SETTINGS a comma list of
#       lib:DIR          another in-tree build (SKML_LIB=sketchml_amd/DIR/libskml.so)
#       form:NAME:VALUE  a skml_debug_form setting, applied by the tool (tools/forms.py)
#       VAR:VALUE        any other environment variable
# Each run's JSON goes to gpurun_out/ab_TAG/NAME_REP.json; one summary line per run on stdout.
set -e
TAG=$1; REPS=$2; KIND=$3; shift 3
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/ab_$TAG
mkdir -p "$OUT"
case $KIND in
  dense)  CMD="python bench.py --steps 100 --warmup 10 --no-cpu-baseline --no-extras --no-configs" ;;
  sparse) CMD="python tools/bench_sparse.py --reps 10 --aggregate 8" ;;
  dsum)   CMD="python tools/bench_decode_sum.py" ;;
  gap)    CMD="python tools/leaf_gap.py --steps 20 --reps 2" ;;
  gap26)  CMD="python tools/leaf_gap.py --steps 40 --reps 2 --n 67108864" ;;
  gap24)  CMD="python tools/leaf_gap.py --steps 80 --reps 2 --n 16777216" ;;
  restore) CMD="python tools/bench_sparse.py --reps 20 --only-decode" ;;
  sparse_enc) CMD="python tools/bench_sparse.py --reps 20 --only-e2e" ;;
  batch)  CMD="python tools/batch_probe.py --reps 7" ;;
  *) echo "unknown kind $KIND"; exit 2 ;;
esac
for i in $(seq 1 "$REPS"); do
  for V in "$@"; do
    NAME=${V%%=*}; SET=${V#*=}
    ENVS=(); FORMS=""
    IFS=',' read -ra ITEMS <<< "$SET"
    for IT in "${ITEMS[@]}"; do
      case $IT in
        lib:*)  ENVS+=("SKML_LIB=sketchml_amd/${IT#lib:}/libskml.so") ;;
        form:*) FORMS="${FORMS:+$FORMS,}${IT#form:}" ;;
        "")     ;;
        *)      ENVS+=("${IT%%:*}=${IT#*:}") ;;
      esac
    done
    env "${ENVS[@]}" SKML_TOOL_FORMS="$FORMS" timeout -k 10 300 $CMD > "$OUT/${NAME}_$i.json" 2> "$OUT/${NAME}_$i.err"
    python3 tools/ab_summary.py "$KIND" "$NAME" "$i" "$OUT/${NAME}_$i.json" | tee -a "$OUT/summary.txt"
  done
done
