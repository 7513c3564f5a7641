#!/bin/bash
# Timeline of one sparse writeObject (skml_sparse_serialize, first call: the device stream build)
# and one readObject at C3.  usage (GPU box): bash tools/prof_wire.sh TAG
set -e
TAG=${1:-wire}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
D=gpurun_out/prof_wire_$TAG
rm -rf "$D"
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace -d "$D" -o run -- python3 tools/bench_sparse.py --reps 1 > "$D.json"
DB=$(find "$D" -name "*.db" | head -1)
python3 tools/rocpd_timeline.py "$DB" --from k_huff_hist --nth 1 --count 60 > "$D.txt"
echo "---- read" >> "$D.txt"
python3 tools/rocpd_timeline.py "$DB" --from k_rd_fixed_sum --nth 1 --count 60 >> "$D.txt"
rm -rf "$D"
