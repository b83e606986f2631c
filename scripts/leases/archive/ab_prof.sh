# Kernel-trace A/B of library builds: rocprofv3 --kernel-trace --stats of bench.py per build.
# Usage (GPU box): bash scripts/leases/ab_prof.sh <tag> "<lib paths>" [bench args...]
# Summaries: python scripts/prof_summary.py gpurun_out/<tag>/<i> (one directory per build, 0 = default).
set -o pipefail
export TMPDIR=/tmp
TAG=$1; LIBS=$2; shift 2
OUT=gpurun_out/$TAG
i=0
for lib in dcf_amd/libdcf_hip.so $LIBS; do
  mkdir -p $OUT/$i/trace
  echo "$lib" > $OUT/$i/lib.txt
  DCF_HIP_LIB=$PWD/$lib timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT/$i/trace -o trace -- \
    python3 bench.py --no-cpu "$@" > $OUT/$i/log 2>&1 || { tail -5 $OUT/$i/log; exit 1; }
  i=$((i+1))
done
