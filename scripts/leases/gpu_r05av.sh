# r05av: the staged C2 instance (device-copy keys, DMA after the CW wait) with round keys 0..KS-1
# held in registers so the next pass first waits on the VM counter KS-1 rounds later: KS = 3 (ks3)
# and 5 (ks5) vs 0 (default): parity with each, then C2, 4 alternating runs.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05av; mkdir -p $O
for pv in ks3 ks5; do
DCF_HIP_LIB=$PWD/dcf_amd/libdcf_hip_$pv.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fuzz.py tests/test_configs.py -x -q --timeout 300 --timeout-method thread -k "prefix or device_large or eval_random or fuzz_single or c2" > $O/pytest_$pv.log 2>&1 || { tail -60 $O/pytest_$pv.log; exit 1; }
echo "$pv $(tail -1 $O/pytest_$pv.log)"
done
for rep in 1 2 3 4; do
for v in default ks3 ks5; do
  if [ $v = default ]; then L=dcf_amd/libdcf_hip.so; else L=dcf_amd/libdcf_hip_$v.so; fi
  DCF_HIP_LIB=$PWD/$L timeout -k 10 300 python bench.py --workload c2 --steps 60 --warmup 10 --no-cpu --no-compare > $O/c2_${v}_$rep.json 2> $O/c2_${v}_$rep.err || { tail -20 $O/c2_${v}_$rep.err; exit 1; }
  python -c "import json; d=json.load(open('$O/c2_${v}_$rep.json')); r=d['roofline']; print('c2', '$v', $rep, round(d['ms_per_step'],4), round(r['frac'],4), round(d['phases']['walk_ms'],3))" | tee -a $O/ab.txt
done
done
