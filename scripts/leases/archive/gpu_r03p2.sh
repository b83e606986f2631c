# r03p2: single-key CWs staged in LDS for the small-batch pair kernel (k_eval16_pair<3>) — parity tests, then C1 A/B: kl = CWs in LDS, default = global CW loads
set -o pipefail
O=gpurun_out/r03p2; mkdir -p $O
DCF_HIP_LIB=$PWD/dcf_amd/libdcf_hip_kl.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_configs.py tests/test_lat_threads.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for rep in 1 2 3; do for v in kl ""; do
  L=$PWD/dcf_amd/libdcf_hip.so; [ -n "$v" ] && L=$PWD/dcf_amd/libdcf_hip_$v.so
  DCF_HIP_LIB=$L timeout -k 10 300 python bench.py --workload c1 --steps 300 --warmup 100 --no-cpu --no-compare > $O/c1_$v$rep.json 2> $O/c1_$v$rep.err || { tail -5 $O/c1_$v$rep.err; exit 1; }
  python -c "import json; d=json.load(open('$O/c1_$v$rep.json')); r=d['roofline']; h=d['host_path']; print('c1', '${v:-global}', round(d['value']/1e6,2), round(r['frac'],4), round(d['ms_per_step'],4), 'host', round(h['value']/1e6,1))"
done; done
