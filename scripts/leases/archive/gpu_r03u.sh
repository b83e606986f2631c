# r03u: k_eval16_oct slot schedule v2 (plan a slot ahead) — oct / host tests, in-kernel walk time (clock probes), latency sweep + lat bench A/B
set -o pipefail
O=gpurun_out/r03u; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_lat_threads.py tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
for v in clk clkold; do DCF_HIP_LIB=$PWD/dcf_amd/libdcf_hip_$v.so timeout -k 10 120 python scripts/lat_probe.py > $O/probe_$v.json 2>$O/probe_$v.err || { tail -5 $O/probe_$v.err; exit 1; }; echo $v; cat $O/probe_$v.json; done
for rep in 1 2; do for v in "" old; do
  L=$PWD/dcf_amd/libdcf_hip.so; [ -n "$v" ] && L=$PWD/dcf_amd/libdcf_hip_$v.so
  DCF_HIP_LIB=$L timeout -k 10 300 python scripts/lat_sweep.py > $O/sweep_$v$rep.json 2> $O/sweep_$v$rep.err || { tail -5 $O/sweep_$v$rep.err; exit 1; }
  DCF_HIP_LIB=$L timeout -k 10 300 python bench.py --workload lat --steps 300 --warmup 30 > $O/lat_$v$rep.json 2> $O/lat_$v$rep.err || { tail -5 $O/lat_$v$rep.err; exit 1; }
  python -c "
import json; s=json.load(open('$O/sweep_$v$rep.json')); d=json.load(open('$O/lat_$v$rep.json'))
print('${v:-new}', 'lat eval/gen us', round(d['eval_us'],1), round(d['gen_us'],1), 'sweep eval', {k: round(x,1) for k,x in s['eval_us'].items()})"
done; done
