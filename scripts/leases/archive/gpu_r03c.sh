# Round-3 A/B: latency-kernel round form (late vs early DPP) and the multi-key top-tree instance (C5).
set -o pipefail
O=gpurun_out/r03c; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -60 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
DCF_HIP_LIB=$PWD/dcf_amd/libdcf_hip_mkpf.so timeout -k 10 600 python -u -m pytest tests/test_configs.py tests/test_gpu_parity.py -m gpu -x -q -k "multikey or c5" --timeout 300 --timeout-method thread > $O/pytest_mkpf.log 2>&1 || { tail -30 $O/pytest_mkpf.log; exit 1; }
tail -1 $O/pytest_mkpf.log
for rep in 1 2; do for v in "" _early; do
  DCF_HIP_LIB=$PWD/dcf_amd/libdcf_hip$v.so timeout -k 10 300 python bench.py --workload lat > $O/lat$v.$rep.json 2>/dev/null || exit 1
  python -c "import json; d=json.load(open('$O/lat$v.$rep.json')); print('lat${v:-default}', round(d['gen_us'],1), round(d['eval_us'],1))"
done; done
for rep in 1 2; do for v in "" _mkpf; do
  DCF_HIP_LIB=$PWD/dcf_amd/libdcf_hip$v.so timeout -k 10 400 python bench.py --workload c5 --steps 3 --warmup 1 --no-cpu > $O/c5$v.$rep.json 2>/dev/null || exit 1
  python -c "import json; d=json.load(open('$O/c5$v.$rep.json')); r=d['roofline']; print('c5${v:-default}', round(d['value']/1e6,2), round(r['eval_only']['frac'],4), d['phases_ms']['eval_party0'])"
done; done
