# r05ap: PMC passes (FETCH_SIZE / WRITE_SIZE / SQ, separate runs) + kernel traces of every bench
# launch shape on the final round-5 tree (wave priority on; C3 at its auto prefix depth 27), for
# bench.py's roofline.traffic and the LDS-busy / VALU figures in DESIGN.md.
set -o pipefail
export TMPDIR=/tmp
TRAFFIC="k_eval16_stream C3 268435456 16 16 27 17179869184" bash scripts/leases/gpu_profile_w.sh r05ap c3 || exit 1
TRAFFIC="k_eval_wide_head_stream+k_eval_wide_tail C4 4194304 16 16384 21 68786585600" bash scripts/leases/gpu_profile_w.sh r05ap c4 || exit 1
TRAFFIC="k_eval16_stream C2 16777216 4 16 24 872415232" bash scripts/leases/gpu_profile_w.sh r05ap c2 || exit 1
TRAFFIC="k_gen16+2*k_mk_prefix16+2*k_cw_keymajor+2*k_eval16_stream C5 67108864 16 16 0 35416702976" bash scripts/leases/gpu_profile_w.sh r05ap c5 || exit 1
TRAFFIC="k_eval16_pair C1 100000 16 16 0 3200000" bash scripts/leases/gpu_profile_w.sh r05ap c1 || exit 1
ls gpurun_out/r05ap
