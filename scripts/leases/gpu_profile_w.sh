# rocprofv3 kernel trace + PMC passes for one bench workload (run on the GPU box).
#   bash scripts/leases/gpu_profile_w.sh <tag> <workload> [extra bench args...]
# Writes gpurun_out/<tag>/{trace,pmc_fetch,pmc_write,pmc_sq}_<workload>/ (one pass each,
# MI355X_MICROARCH.md: FETCH_SIZE and WRITE_SIZE in separate passes).
set -o pipefail
TAG=$1; W=$2; shift 2
export TMPDIR=/tmp
OUT=gpurun_out/$TAG
mkdir -p $OUT
B="bench.py --workload $W --steps 2 --warmup 1 --no-cpu --no-compare $*"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace_$W -o trace -- python $B > $OUT/trace_$W.log 2>&1 || { tail -5 $OUT/trace_$W.log; exit 1; }
grep "^{\"metric" $OUT/trace_$W.log > $OUT/bench_prof_$W.json || true
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE -d $OUT/pmc_fetch_$W -o pmc -- python $B > $OUT/pmc_fetch_$W.log 2>&1 || { tail -5 $OUT/pmc_fetch_$W.log; exit 1; }
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE -d $OUT/pmc_write_$W -o pmc -- python $B > $OUT/pmc_write_$W.log 2>&1 || { tail -5 $OUT/pmc_write_$W.log; exit 1; }
timeout -s KILL 240 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_INSTS_SALU GRBM_GUI_ACTIVE -d $OUT/pmc_sq_$W -o pmc -- python $B > $OUT/pmc_sq_$W.log 2>&1 || { tail -5 $OUT/pmc_sq_$W.log; exit 1; }

# summarise on the box (the rocpd databases are too large to bring back), then drop them
python scripts/prof_summary.py $OUT --suffix _$W > $OUT/prof_$W.md || exit 1
if [ -n "$TRAFFIC" ]; then  # TRAFFIC="<kernel prefix(es)> <workload> <points> <n_bytes> <lambda> <prefix> <alg bytes>"
  python scripts/prof_summary.py $OUT --suffix _$W --traffic $OUT/pmc_traffic_$W.json $TRAFFIC > /dev/null || exit 1
fi
rm -rf $OUT/trace_$W $OUT/pmc_fetch_$W $OUT/pmc_write_$W $OUT/pmc_sq_$W
echo "profiled $W"
