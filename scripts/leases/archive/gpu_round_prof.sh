# Round evidence in one call: GPU tests + bench lines (gpu_round.sh), smoke, rocprof kernel traces and
# PMC passes of C3, C2 and C4 with their traffic entries.   bash scripts/leases/gpu_round_prof.sh <tag>
set -o pipefail
T=$1
bash scripts/leases/gpu_round.sh $T c1 c2 c4 c5 fd || exit 1
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/$T/smoke.log 2>&1 || { tail -20 gpurun_out/$T/smoke.log; exit 1; }
tail -1 gpurun_out/$T/smoke.log
bash scripts/leases/gpu_prof_r02.sh $T || exit 1
TRAFFIC="k_eval_wide_head_stream+k_eval_wide_tail C4 4194304 16 16384 21 68786585600" bash scripts/leases/gpu_profile_w.sh $T c4 || exit 1
