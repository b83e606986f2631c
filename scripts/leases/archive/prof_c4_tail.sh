# Kernel trace + LDS/VALU PMC of C4 for the default lib and variants:
#   bash scripts/leases/prof_c4_tail.sh <tag> [variant...]   (variant v = dcf_amd/libdcf_hip_<v>.so)
set -o pipefail
export TMPDIR=/tmp
T=$1; shift
O=gpurun_out/$T; mkdir -p $O
for v in default "$@"; do
  if [ $v = default ]; then export DCF_HIP_LIB=$PWD/dcf_amd/libdcf_hip.so; else export DCF_HIP_LIB=$PWD/dcf_amd/libdcf_hip_$v.so; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace_$v -o trace -- python bench.py --workload c4 --steps 3 --warmup 1 --no-cpu > $O/trace_$v.log 2>&1 || exit 1
  timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -d $O/pmc_sq_$v -o pmc -- python bench.py --workload c4 --steps 1 --warmup 1 --no-cpu > $O/pmc_$v.log 2>&1 || exit 1
  python scripts/prof_summary.py $O --suffix _$v > $O/summary_$v.md 2>&1
done
