# PMC set a (LDS/VALU/clock counters) for the default library and each A/B library given.
# Usage (GPU box): bash scripts/leases/pmc_ab.sh <tag> "<lib paths>" [points]
set -o pipefail
export TMPDIR=/tmp
TAG=$1; LIBS=$2; PTS=${3:-67108864}
OUT=gpurun_out/$TAG
mkdir -p $OUT
C="SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_INSTS_VALU SQ_WAIT_INST_LDS SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_SALU SQ_WAIT_ANY GRBM_GUI_ACTIVE GRBM_COUNT"
i=0
for lib in dcf_amd/libdcf_hip.so $LIBS; do
  DCF_HIP_LIB=$PWD/$lib timeout -s KILL 120 rocprofv3 --pmc $C -d $OUT/l$i -o pmc -- python bench.py --steps 2 --warmup 1 --no-cpu --no-compare --points $PTS > $OUT/l$i.log 2>&1 || exit 1
  i=$((i+1))
done
python scripts/pmc_print.py $OUT
