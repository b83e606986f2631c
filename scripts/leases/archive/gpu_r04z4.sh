# r04z4: PMC traffic of the C1 and C5 launch shapes on the round-4 tree (FETCH_SIZE / WRITE_SIZE in
# separate passes, kernel trace, SQ counters).
set -o pipefail
export TMPDIR=/tmp
TRAFFIC="k_eval16_pair C1 100000 16 16 0 3200000" bash scripts/leases/gpu_profile_w.sh r04z4 c1 || exit 1
TRAFFIC="k_gen16+2*k_mk_prefix16+2*k_cw_keymajor+2*k_eval16_stream C5 67108864 16 16 0 35416702976" bash scripts/leases/gpu_profile_w.sh r04z4 c5 || exit 1
