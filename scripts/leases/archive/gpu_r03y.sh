# r03y: latency micro (round-key XOR share), threshold-boundary latency tests, mid host path buffer reuse, C1 host path coarse- vs fine-grained mid buffer
set -o pipefail
O=gpurun_out/r03y; mkdir -p $O
timeout -k 10 60 ./scripts/micro/lat_chain > $O/lat_chain.json || exit 1
cat $O/lat_chain.json
timeout -k 10 600 python -u -m pytest tests/test_lat_threads.py tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
DCF_HIP_LIB=$PWD/dcf_amd/libdcf_hip_coh.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k host_mid --timeout 300 --timeout-method thread > $O/pytest_coh.log 2>&1 || { tail -30 $O/pytest_coh.log; exit 1; }
tail -1 $O/pytest_coh.log
for rep in 1 2 3; do for v in "" coh; do
  L=$PWD/dcf_amd/libdcf_hip.so; [ -n "$v" ] && L=$PWD/dcf_amd/libdcf_hip_$v.so
  DCF_HIP_LIB=$L timeout -k 10 300 python bench.py --workload c1 --steps 100 --warmup 30 --no-cpu --no-compare > $O/c1_$v$rep.json 2> $O/c1_$v$rep.err || { tail -5 $O/c1_$v$rep.err; exit 1; }
  python -c "import json; d=json.load(open('$O/c1_$v$rep.json')); h=d['host_path']; print('c1 host', '${v:-noncoh}', round(d['value']/1e6,1), round(h['value']/1e6,1), round(h['ms_per_step'],3), h['matches_device_path'])"
done; done
