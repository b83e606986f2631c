# r05au: PMC passes + kernel trace of the C2 launch shape with the staged rows (r05as), for
# bench.py's roofline.traffic (r05ap measured the gather form).
set -o pipefail
export TMPDIR=/tmp
TRAFFIC="k_eval16_stream C2 16777216 4 16 24 872415232" bash scripts/leases/gpu_profile_w.sh r05au c2 || exit 1
ls gpurun_out/r05au
