# r04s: k_dec_keys with nontemporal streams (SKML_DEC_NT) and k_rs_merge's per-word emission (SKML_RS_EMIT_BITS) A/B, and its L2 hit / miss counters
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r04s
set -e
for i in 1 2 3; do
  for V in base:SKML_AB_DEFAULT=1 nt:SKML_DEC_NT=1 bits:SKML_RS_EMIT_BITS=1; do
    env "${V#*:}" timeout -k 10 200 python tools/bench_sparse.py --reps 5 --aggregate 8 > gpurun_out/r04s/${V%%:*}_$i.json 2>&1
    python3 -c "
import json
d = json.loads(open('gpurun_out/r04s/${V%%:*}_$i.json').read().strip().splitlines()[-1])
print('${V%%:*}', $i, {k: d['ms'][k] for k in ('decode', 'decode_sum')})"
  done
done
for V in base:SKML_AB_DEFAULT=1 nt:SKML_DEC_NT=1; do
  env "${V#*:}" SKML_AGG_ONE_LANE=1 timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --kernel-trace -d gpurun_out/r04s/pmc_${V%%:*} -o run --output-format csv -- python3 tools/bench_sparse.py --reps 1 --aggregate 8 > gpurun_out/r04s/pmc_${V%%:*}.log 2>&1
done
python3 - <<'PY'
import csv, glob, re, statistics
for v in ("base", "nt"):
    res = {}
    for p in glob.glob(f"gpurun_out/r04s/pmc_{v}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(p)):
            m = re.search(r"(k_[A-Za-z0-9_]+)", r["Kernel_Name"])
            if m and m.group(1) in ("k_dec_keys", "k_agg_vtiles", "k_dec_deltas"):
                res.setdefault(m.group(1), {}).setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
    for k, d in res.items():
        h, ms = statistics.mean(d.get("TCC_HIT_sum", [0])), statistics.mean(d.get("TCC_MISS_sum", [0]))
        print(v, k, "hit", int(h), "miss", int(ms), "hit rate %.3f" % (h / max(h + ms, 1)))
PY
find gpurun_out/r04s -name "*counter_collection.csv" -size +20M -delete
