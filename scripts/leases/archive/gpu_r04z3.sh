# r04z3: PMC traffic of the round-4 C2 and C4 launch shapes (FETCH_SIZE / WRITE_SIZE in separate passes,
# kernel trace, SQ counters), recorded per launch shape for bench.py's roofline.traffic.
set -o pipefail
export TMPDIR=/tmp
# PMC traffic (FETCH_SIZE / WRITE_SIZE in separate passes) of the C2 and C4 launch shapes on this tree
TRAFFIC="k_eval16_stream C2 16777216 4 16 24 872415232" bash scripts/leases/gpu_profile_w.sh r04z c2 || exit 1
TRAFFIC="k_eval_wide_head_stream+k_eval_wide_tail C4 4194304 16 16384 21 68786585600" bash scripts/leases/gpu_profile_w.sh r04z c4 || exit 1
