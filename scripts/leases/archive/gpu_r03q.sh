# r03q: C4 tail with row 0 folded into the constant (Tail2Layout<9, 2, 1>, 22 reads) — wide parity on it, then C4 A/B vs the previous lib
set -o pipefail
O=gpurun_out/r03q; mkdir -p $O
DCF_HIP_LIB=$PWD/dcf_amd/libdcf_hip_r0.so timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "wide or large_lambda or c4 or tail or full_domain" > $O/pytest_r0.log 2>&1 || { tail -30 $O/pytest_r0.log; exit 1; }
tail -1 $O/pytest_r0.log
for rep in 1 2 3; do for v in "" r0; do
  L=$PWD/dcf_amd/libdcf_hip.so; [ -n "$v" ] && L=$PWD/dcf_amd/libdcf_hip_$v.so
  DCF_HIP_LIB=$L timeout -k 10 300 python bench.py --workload c4 --steps 10 --warmup 3 --no-cpu > $O/c4_$v$rep.json 2> $O/c4_$v$rep.err || { tail -5 $O/c4_$v$rep.err; exit 1; }
  python -c "import json; d=json.load(open('$O/c4_$v$rep.json')); r=d['roofline']; print('c4', '${v:-old}', round(d['value']/1e6,2), round(r['frac'],4), round(r['kernel_ms'],2))"
done; done
