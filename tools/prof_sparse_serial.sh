#!/bin/bash
# Timeline of one C3 sparse encode with every kernel alone on one stream (SKML_SERIAL=1), so
# each duration is the kernel's own.  usage (GPU box): bash tools/prof_sparse_serial.sh TAG [ENV=VAL ...]
set -e
TAG=${1:-serial}
shift || true
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
D=gpurun_out/prof_sp_$TAG
rm -rf "$D"
env SKML_SERIAL=1 "$@" true
export SKML_SERIAL=1
for kv in "$@"; do export "$kv"; done
timeout -k 10 300 rocprofv3 --kernel-trace -d "$D" -o run -- python3 tools/bench_sparse.py --reps 2 > "$D.json"
DB=$(find "$D" -name "*.db" | head -1)
python3 tools/rocpd_timeline.py "$DB" --from k_compact --nth 3 --count 45 > "$D.txt"
python3 tools/rocpd_timeline.py "$DB" --stats >> "$D.txt"
rm -rf "$D"
