# PMC + trace summaries for C2, C4, C5 (bench defaults), with per-step traffic entries.
set -o pipefail
T=${1:-r02e}
TRAFFIC="k_eval16_stream C2 16777216 4 16 23 872415232" bash scripts/leases/gpu_profile_w.sh $T c2 &&
TRAFFIC="k_eval_wide_head_stream+k_eval_wide_tail C4 4194304 16 16384 21 68786585600" bash scripts/leases/gpu_profile_w.sh $T c4 &&
TRAFFIC="k_gen16+2*k_cw_keymajor+2*k_eval16_stream C5 67108864 16 16 0 35416702976" bash scripts/leases/gpu_profile_w.sh $T c5
