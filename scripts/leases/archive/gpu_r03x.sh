# r03x: k_gen16_row (one wave per key, 16-lane-row AES) and a spin-wait for tiny calls — latency tests, then sweep + lat bench A/B (new, old = before the row kernels, spin = new + DCF_TINY_SPIN)
set -o pipefail
O=gpurun_out/r03x; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_lat_threads.py tests/test_gpu_parity.py tests/test_configs.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log

for rep in 1 2; do for v in "" old spin; do
  L=$PWD/dcf_amd/libdcf_hip.so; [ -n "$v" ] && L=$PWD/dcf_amd/libdcf_hip_$v.so
  DCF_HIP_LIB=$L timeout -k 10 300 python scripts/lat_sweep.py > $O/sweep_$v$rep.json 2> $O/sweep_$v$rep.err || { tail -5 $O/sweep_$v$rep.err; exit 1; }
  DCF_HIP_LIB=$L timeout -k 10 300 python bench.py --workload lat --steps 300 --warmup 30 > $O/lat_$v$rep.json 2> $O/lat_$v$rep.err || { tail -5 $O/lat_$v$rep.err; exit 1; }
  python -c "
import json; s=json.load(open('$O/sweep_$v$rep.json')); d=json.load(open('$O/lat_$v$rep.json'))
print('${v:-new}', 'lat eval/gen us', round(d['eval_us'],1), round(d['gen_us'],1), 'sweep gen', {k: round(x,1) for k,x in s['gen_us'].items()})"
done; done
