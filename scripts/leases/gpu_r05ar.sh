# r05ar: C2 latency probe — every refill's prefix row from one L2-resident 32 KiB span (probe build,
# wrong results by construction, no parity) vs the default: the upper bound of hiding the row
# gather under wave priority.  C2 and C3, 3 alternating runs (bench's own parity check off: --no-compare).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05ar; mkdir -p $O
for rep in 1 2 3; do
for v in default probe; do
  if [ $v = default ]; then L=dcf_amd/libdcf_hip.so; else L=dcf_amd/libdcf_hip_$v.so; fi
  for w in c2 c3; do
    case $w in c2) SW="--steps 60 --warmup 10";; c3) SW="--steps 5 --warmup 2";; esac
    DCF_HIP_LIB=$PWD/$L timeout -k 10 300 python bench.py --workload $w $SW --no-cpu --no-compare > $O/${w}_${v}_$rep.json 2> $O/${w}_${v}_$rep.err || { tail -20 $O/${w}_${v}_$rep.err; exit 1; }
    python -c "import json; d=json.load(open('$O/${w}_${v}_$rep.json')); r=d['roofline']; print('$w', '$v', $rep, round(d['ms_per_step'],4), round(r['frac'],4), d['phases']['walk_ms'])" | tee -a $O/ab.txt
  done
done
done
