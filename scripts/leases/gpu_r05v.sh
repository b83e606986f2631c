# r05v: single-key N = 16 / N = 4 stream instances compiled for "every start below the shared-prefix
# table" (PFX; the fresh-x-word selects are compiled out, 87 -> 74 SGPRs) when the call has a table
# (default) vs the general instances (libdcf_hip_skpfx0.so, -DDCF_SK_PFX=0): the GPU suite with the
# default build, then C3 / C2 A/B, 3 alternating runs.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05v; mkdir -p $O
timeout -k 10 800 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -60 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
for rep in 1 2 3; do
for v in default skpfx0; do
  if [ $v = default ]; then L=dcf_amd/libdcf_hip.so; else L=dcf_amd/libdcf_hip_$v.so; fi
  for w in c3 c2; do
    case $w in c3) SW="--steps 10 --warmup 3";; c2) SW="--steps 60 --warmup 10";; esac
    DCF_HIP_LIB=$PWD/$L timeout -k 10 300 python bench.py --workload $w $SW --no-cpu --no-compare > $O/${w}_${v}_$rep.json 2> $O/${w}_${v}_$rep.err || { tail -20 $O/${w}_${v}_$rep.err; exit 1; }
    python -c "import json; d=json.load(open('$O/${w}_${v}_$rep.json')); r=d['roofline']; print('$w', '$v', $rep, round(d['ms_per_step'],3), round(r['frac'],4))" | tee -a $O/ab.txt
  done
done
done
