# r05ax: C2 staging in 4 slots of 16 points (q4) vs 2 slots of 32 (default, the generalized code):
# parity with both, then C2, 4 alternating runs.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05ax; mkdir -p $O
for pv in default q4; do
  if [ $pv = default ]; then L=dcf_amd/libdcf_hip.so; else L=dcf_amd/libdcf_hip_$pv.so; fi
  DCF_HIP_LIB=$PWD/$L timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fuzz.py tests/test_configs.py -x -q --timeout 300 --timeout-method thread -k "prefix or device_large or eval_random or fuzz_single or c2" > $O/pytest_$pv.log 2>&1 || { tail -60 $O/pytest_$pv.log; exit 1; }
  echo "$pv $(tail -1 $O/pytest_$pv.log)"
done
for rep in 1 2 3 4; do
for v in default q4; do
  if [ $v = default ]; then L=dcf_amd/libdcf_hip.so; else L=dcf_amd/libdcf_hip_$v.so; fi
  DCF_HIP_LIB=$PWD/$L timeout -k 10 300 python bench.py --workload c2 --steps 60 --warmup 10 --no-cpu --no-compare > $O/c2_${v}_$rep.json 2> $O/c2_${v}_$rep.err || { tail -20 $O/c2_${v}_$rep.err; exit 1; }
  python -c "import json; d=json.load(open('$O/c2_${v}_$rep.json')); r=d['roofline']; print('c2', '$v', $rep, round(d['ms_per_step'],4), round(r['frac'],4), round(d['phases']['walk_ms'],3))" | tee -a $O/ab.txt
done
done
