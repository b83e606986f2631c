# GPU parity + rocprofv3 kernel stats + HBM PMC passes for the default bench workload.
# Usage (from repo root, on the GPU box): bash scripts/leases/gpu_profile.sh [tag]
set -o pipefail
TAG=${1:-r01}
export TMPDIR=/tmp
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/trace -o trace -- python bench.py --steps 3 --warmup 1 --no-cpu --no-compare > $OUT/bench_trace.log 2>&1 || exit 1
[ -n "$NO_PMC" ] || {
timeout -k 10 120 rocprofv3 --pmc FETCH_SIZE -d $OUT/pmc_fetch -o pmc -- python bench.py --steps 2 --warmup 1 --no-cpu --no-compare > $OUT/pmc_fetch.log 2>&1 || exit 1
timeout -k 10 120 rocprofv3 --pmc WRITE_SIZE -d $OUT/pmc_write -o pmc -- python bench.py --steps 2 --warmup 1 --no-cpu --no-compare > $OUT/pmc_write.log 2>&1 || exit 1
timeout -k 10 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_LDS -d $OUT/pmc_sq -o pmc -- python bench.py --steps 2 --warmup 1 --no-cpu --no-compare > $OUT/pmc_sq.log 2>&1 || exit 1
}
timeout -k 10 600 python bench.py --steps 5 --warmup 2 > $OUT/bench.log 2>&1 || exit 1
tail -1 $OUT/bench.log
for w in ${EXTRA:-}; do
  timeout -k 10 300 python bench.py --workload $w --steps 3 --warmup 1 --no-cpu > $OUT/bench_$w.log 2>&1 || exit 1
  tail -1 $OUT/bench_$w.log
done
