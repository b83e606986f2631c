# r03r: table build with SGPR round keys (DCF_PFX_GK=0) — prefix / FD parity on it, then C2 / FD A/B vs default
set -o pipefail
O=gpurun_out/r03r; mkdir -p $O
DCF_HIP_LIB=$PWD/dcf_amd/libdcf_hip_pgk0.so timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "prefix or full_domain or c2" > $O/pytest_pgk0.log 2>&1 || { tail -30 $O/pytest_pgk0.log; exit 1; }
tail -1 $O/pytest_pgk0.log
for rep in 1 2 3; do for v in "" pgk0; do
  L=$PWD/dcf_amd/libdcf_hip.so; [ -n "$v" ] && L=$PWD/dcf_amd/libdcf_hip_$v.so
  DCF_HIP_LIB=$L timeout -k 10 300 python bench.py --workload c2 --steps 60 --warmup 20 --no-cpu --no-compare > $O/c2_$v$rep.json 2> $O/c2_$v$rep.err || { tail -5 $O/c2_$v$rep.err; exit 1; }
  python -c "import json; d=json.load(open('$O/c2_$v$rep.json')); r=d['roofline']; p=d.get('phases',{}); print('c2', '${v:-default}', round(d['value']/1e6,1), round(r['frac'],4), round(r['kernel_ms'],3), round(p.get('table_ms',0),3))"
  DCF_HIP_LIB=$L timeout -k 10 300 python bench.py --workload fd --steps 3 --warmup 1 --no-cpu > $O/fd_$v$rep.json 2> $O/fd_$v$rep.err || { tail -5 $O/fd_$v$rep.err; exit 1; }
  python -c "import json; d=json.load(open('$O/fd_$v$rep.json')); r=d['roofline']; print('fd', '${v:-default}', round(d['value']/1e9,3), round(r['frac'],4), round(r.get('kernel_ms',0),2))"
done; done
