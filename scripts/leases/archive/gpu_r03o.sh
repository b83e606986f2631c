# r03o: full domain's upper levels by one k_prefix_build16 launch (DCF_FD_BUILD) — FD / prefix parity, then FD A/B vs the previous lib
set -o pipefail
O=gpurun_out/r03o; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "full_domain or prefix or fd" > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
for rep in 1 2 3; do for v in "" old; do
  L=$PWD/dcf_amd/libdcf_hip.so; [ -n "$v" ] && L=$PWD/dcf_amd/libdcf_hip_$v.so
  DCF_HIP_LIB=$L timeout -k 10 300 python bench.py --workload fd --steps 3 --warmup 1 --no-cpu > $O/fd_$v$rep.json 2> $O/fd_$v$rep.err || { tail -5 $O/fd_$v$rep.err; exit 1; }
  python -c "import json; d=json.load(open('$O/fd_$v$rep.json')); r=d['roofline']; print('fd', '${v:-new}', round(d['value']/1e9,3), round(r['frac'],4), round(r.get('kernel_ms',0),2), d.get('sample_check', d.get('check')))"
done; done
