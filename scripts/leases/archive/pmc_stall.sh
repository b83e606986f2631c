# Wave-state PMC pass (where the waves' cycles go) for the given workloads, one rocprofv3 pass each.
# Usage (GPU box): bash scripts/leases/pmc_stall.sh <tag> "<workload[:points]>..."
set -o pipefail
export TMPDIR=/tmp
TAG=$1; WS=$2
OUT=gpurun_out/$TAG
mkdir -p $OUT
C="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE"
for wp in $WS; do
  w=${wp%%:*}; p=${wp#*:}; PA=""; [ "$p" != "$wp" ] && PA="--points $p"
  timeout -s KILL 120 rocprofv3 --pmc $C -d $OUT/$w -o pmc -- python bench.py --workload $w $PA --steps 2 --warmup 1 --no-cpu --no-compare > $OUT/$w.log 2>&1 || { tail -5 $OUT/$w.log; exit 1; }
done
PMC_KERNELS="${PMC_KERNELS:-k_}" python scripts/pmc_print.py $OUT
rm -rf $OUT/*/
