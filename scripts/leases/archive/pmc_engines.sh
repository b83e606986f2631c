# PMC comparison of eval engines (LDS/VALU/clock counters), one rocprofv3 pass per engine and counter set.
# Usage (GPU box): bash scripts/leases/pmc_engines.sh <tag> "<modes>" [points] [set]
set -o pipefail
export TMPDIR=/tmp
TAG=${1:-pmc}; MODES=${2:-"1 4"}; PTS=${3:-67108864}; SET=${4:-a}
OUT=gpurun_out/$TAG
mkdir -p $OUT
case $SET in
  a) C="SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_INSTS_VALU SQ_WAIT_INST_LDS SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_SALU SQ_WAIT_ANY GRBM_GUI_ACTIVE GRBM_COUNT";;
  b) C="SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_VMEM SQ_WAIT_INST_ANY SQ_INST_LEVEL_LDS SQ_LDS_CMD_FIFO_FULL SQ_IFETCH GRBM_GUI_ACTIVE";;
esac
WL=${WORKLOAD:-c3}
for m in $MODES; do
  timeout -s KILL 120 rocprofv3 --pmc $C -d $OUT/m$m$SET -o pmc -- python bench.py --workload $WL --steps 2 --warmup 1 --no-cpu --eval-mode $m --points $PTS > $OUT/m$m$SET.log 2>&1 || exit 1
done
