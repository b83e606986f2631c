# C3 bench line + rocprofv3 kernel trace of the same workload in one lease.
#   bash scripts/leases/gpu_c3_lease.sh <tag>
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/$1; mkdir -p $O
timeout -k 10 600 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_c3.json 2> $O/bench_c3.err || { tail -20 $O/bench_c3.err; exit 1; }
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/trace -o trace -- python3 bench.py --steps 5 --warmup 2 --no-cpu --no-compare > $O/bench_trace.log 2>&1 || { tail -20 $O/bench_trace.log; exit 1; }
python scripts/lease_c3.py $O > $O/prof_c3.md && cat $O/prof_c3.md
