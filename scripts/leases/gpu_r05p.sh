# r05p: PMC passes (FETCH_SIZE / WRITE_SIZE / SQ, separate runs) + kernel traces of the C1, C2 and
# C5 launch shapes on the final round-5 tree, for bench.py's roofline.traffic (round 4's files
# were the last for these three).
set -o pipefail
export TMPDIR=/tmp
TRAFFIC="k_eval16_pair C1 100000 16 16 0 3200000" bash scripts/leases/gpu_profile_w.sh r05p c1 || exit 1
TRAFFIC="k_eval16_stream C2 16777216 4 16 24 872415232" bash scripts/leases/gpu_profile_w.sh r05p c2 || exit 1
TRAFFIC="k_gen16+2*k_mk_prefix16+2*k_cw_keymajor+2*k_eval16_stream C5 67108864 16 16 0 35416702976" bash scripts/leases/gpu_profile_w.sh r05p c5 || exit 1
ls gpurun_out/r05p
