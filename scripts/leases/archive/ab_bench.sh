# A/B kernel variants: bench.py against each in-tree library build given (default build first).
# Usage (GPU box): bash scripts/leases/ab_bench.sh <tag> "<lib paths>" [bench args...]
set -o pipefail
TAG=$1; LIBS=$2; shift 2
OUT=gpurun_out/$TAG
mkdir -p $OUT
i=0
for lib in dcf_amd/libdcf_hip.so $LIBS; do
  DCF_HIP_LIB=$PWD/$lib timeout -k 10 200 python bench.py --no-cpu "$@" > $OUT/ab$i.log 2>&1 || { tail -5 $OUT/ab$i.log; exit 1; }
  python -c "import json,sys;d=json.loads(open('$OUT/ab$i.log').read().splitlines()[-1]);print('$lib', d['value'], d.get('roofline',{}).get('kernel_ms'), d['ms_per_step'])"
  i=$((i+1))
done
