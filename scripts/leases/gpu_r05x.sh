# r05x: x in one word (N <= 4, C2): the stream step skips the x-word queue (its only 32-level
# crossing ends the point) — default vs the committed library (libdcf_hip_head.so): N = 4 parity
# tests, then C2 (and C3 as a control), 3 alternating runs.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05x; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fuzz.py tests/test_configs.py -x -q --timeout 300 --timeout-method thread -k "not wide and not large_lambda and not c4 and not c5" > $O/pytest.log 2>&1 || { tail -60 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for rep in 1 2 3; do
for v in default head; do
  if [ $v = default ]; then L=dcf_amd/libdcf_hip.so; else L=dcf_amd/libdcf_hip_$v.so; fi
  for w in c2 c3; do
    case $w in c3) SW="--steps 10 --warmup 3";; c2) SW="--steps 60 --warmup 10";; esac
    DCF_HIP_LIB=$PWD/$L timeout -k 10 300 python bench.py --workload $w $SW --no-cpu --no-compare > $O/${w}_${v}_$rep.json 2> $O/${w}_${v}_$rep.err || { tail -20 $O/${w}_${v}_$rep.err; exit 1; }
    python -c "import json; d=json.load(open('$O/${w}_${v}_$rep.json')); r=d['roofline']; print('$w', '$v', $rep, round(d['ms_per_step'],4), round(r['frac'],4))" | tee -a $O/ab.txt
  done
done
done
