# rocprof kernel-trace + PMC summaries of the default C3 bench and C2 (auto depths 26 / 24).
set -o pipefail
T=${1:-r02r}
TRAFFIC="k_eval16_stream C3 268435456 16 16 26 17179869184" bash scripts/leases/gpu_profile_w.sh $T c3 &&
TRAFFIC="k_eval16_stream C2 16777216 4 16 24 872415232" bash scripts/leases/gpu_profile_w.sh $T c2
