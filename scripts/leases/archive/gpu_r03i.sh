# r03i: small-batch lane pair with per-pair block scheduling (k_eval16_pair2, default) — GPU suite, C1 A/B vs nop2
set -o pipefail
O=gpurun_out/r03i; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
for rep in 1 2 3; do for v in "" nop2; do
  L=$PWD/dcf_amd/libdcf_hip.so; [ -n "$v" ] && L=$PWD/dcf_amd/libdcf_hip_$v.so
  DCF_HIP_LIB=$L timeout -k 10 300 python bench.py --workload c1 --steps 300 --warmup 100 --no-cpu --no-compare > $O/c1_$v$rep.json 2> $O/c1_$v$rep.err || { tail -5 $O/c1_$v$rep.err; exit 1; }
  python -c "import json; d=json.load(open('$O/c1_$v$rep.json')); r=d['roofline']; print('c1', '${v:-default}', round(d['value']/1e6,2), round(r['frac'],4), round(r['kernel_ms'],4), round(r.get('executed_blocks_per_eval',0),1))"
done; done
timeout -k 10 300 python bench.py --workload c1 --steps 300 --warmup 100 > $O/bench_c1.json 2> $O/bench_c1.err || { tail -5 $O/bench_c1.err; exit 1; }
python -c "import json; d=json.load(open('$O/bench_c1.json')); r=d['roofline']; print('c1 full', d['value'], r['frac'], d['cpu_baseline']['matches_gpu'], d['host_path']['value'])"
timeout -k 10 300 python bench.py --workload lat > $O/bench_lat.json 2> $O/bench_lat.err || { tail -5 $O/bench_lat.err; exit 1; }
python -c "import json; d=json.load(open('$O/bench_lat.json')); print('lat', d['gen_us'], d['eval_us'])"
