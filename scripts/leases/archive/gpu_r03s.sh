# r03s: mid-size host path through a mapped buffer (DCF_HOST_MID) — host / small-batch / wide tests on it, then C1 host-path A/B vs the previous lib
set -o pipefail
O=gpurun_out/r03s; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "host or threads or lat or eval_random or multi or largest or c1" > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
for rep in 1 2 3; do for v in "" old; do
  L=$PWD/dcf_amd/libdcf_hip.so; [ -n "$v" ] && L=$PWD/dcf_amd/libdcf_hip_$v.so
  DCF_HIP_LIB=$L timeout -k 10 300 python bench.py --workload c1 --steps 100 --warmup 30 --no-cpu --no-compare > $O/c1_$v$rep.json 2> $O/c1_$v$rep.err || { tail -5 $O/c1_$v$rep.err; exit 1; }
  python -c "import json; d=json.load(open('$O/c1_$v$rep.json')); h=d['host_path']; print('c1 host', '${v:-new}', round(d['value']/1e6,1), round(h['value']/1e6,1), round(h['ms_per_step'],3), h['matches_device_path'])"
done; done
