# r05ac: single-key stream instances with the round keys read by v_readlane from one VGPR holding
# the schedule (libdcf_hip_rl.so, -DDCF_RL_KEYS=1) vs per-round device-copy loads (default):
# eval parity with the variant, then C3 / C2 A/B, 3 alternating runs.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05ac; mkdir -p $O
DCF_HIP_LIB=$PWD/dcf_amd/libdcf_hip_rl.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fuzz.py -x -q --timeout 300 --timeout-method thread -k "not wide and not large_lambda" > $O/pytest_rl.log 2>&1 || { tail -60 $O/pytest_rl.log; exit 1; }
tail -1 $O/pytest_rl.log
for rep in 1 2 3; do
for v in default rl; do
  if [ $v = default ]; then L=dcf_amd/libdcf_hip.so; else L=dcf_amd/libdcf_hip_$v.so; fi
  for w in c3 c2; do
    case $w in c3) SW="--steps 10 --warmup 3";; c2) SW="--steps 60 --warmup 10";; esac
    DCF_HIP_LIB=$PWD/$L timeout -k 10 300 python bench.py --workload $w $SW --no-cpu --no-compare > $O/${w}_${v}_$rep.json 2> $O/${w}_${v}_$rep.err || { tail -20 $O/${w}_${v}_$rep.err; exit 1; }
    python -c "import json; d=json.load(open('$O/${w}_${v}_$rep.json')); r=d['roofline']; print('$w', '$v', $rep, round(d['ms_per_step'],4), round(r['frac'],4))" | tee -a $O/ab.txt
  done
done
done
