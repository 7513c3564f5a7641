# r04r + r04s in one call
set -e
bash tools/gpu_r04r.sh
bash tools/gpu_r04s.sh
