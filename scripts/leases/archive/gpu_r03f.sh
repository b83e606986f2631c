# r03f: C4 head round keys by uniform loads (gk2) — parity + A/B; C2 refill-latency probes (row0 / xhash / both: wrong bytes, timing only)
set -o pipefail
O=gpurun_out/r03f; mkdir -p $O
DCF_HIP_LIB=$PWD/dcf_amd/libdcf_hip_gk2.so timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  -k "wide or large_lambda or c4 or prg32" > $O/pytest_gk2.log 2>&1 || { tail -30 $O/pytest_gk2.log; exit 1; }
tail -1 $O/pytest_gk2.log
for rep in 1 2; do for v in "" gk2; do
  L=$PWD/dcf_amd/libdcf_hip.so; [ -n "$v" ] && L=$PWD/dcf_amd/libdcf_hip_$v.so
  DCF_HIP_LIB=$L timeout -k 10 300 python bench.py --workload c4 --steps 10 --warmup 3 --no-cpu > $O/c4_$v$rep.json 2> $O/c4_$v$rep.err || { tail -5 $O/c4_$v$rep.err; exit 1; }
  python -c "import json; d=json.load(open('$O/c4_$v$rep.json')); r=d['roofline']; print('c4', '${v:-default}', round(d['value']/1e6,2), round(r['frac'],4), round(r['kernel_ms'],2))"
done; done
for rep in 1 2; do for v in "" row0 xhash both; do
  L=$PWD/dcf_amd/libdcf_hip.so; [ -n "$v" ] && L=$PWD/dcf_amd/libdcf_hip_$v.so
  DCF_HIP_LIB=$L timeout -k 10 300 python bench.py --workload c2 --steps 60 --warmup 20 --no-cpu --no-compare > $O/c2_$v$rep.json 2> $O/c2_$v$rep.err || { tail -5 $O/c2_$v$rep.err; exit 1; }
  python -c "import json; d=json.load(open('$O/c2_$v$rep.json')); r=d['roofline']; p=d.get('phases',{}); print('c2', '${v:-default}', round(d['value']/1e6,1), round(r['frac'],4), round(r['kernel_ms'],3), round(p.get('table_ms',0),3), round(p.get('walk_ms',0),3))"
done; done
