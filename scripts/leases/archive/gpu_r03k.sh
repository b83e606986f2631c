# r03k: uniform CW reads as vector loads (vload) — GPU suite, then A/B vs the previous lib on C1 / C2 / FD
set -o pipefail
O=gpurun_out/r03k; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
for rep in 1 2; do for v in "" old; do
  L=$PWD/dcf_amd/libdcf_hip.so; [ -n "$v" ] && L=$PWD/dcf_amd/libdcf_hip_$v.so
  for w in c1 c2 fd; do
    case $w in c1) SW="--steps 300 --warmup 100";; c2) SW="--steps 60 --warmup 20";; *) SW="--steps 3 --warmup 1";; esac
    DCF_HIP_LIB=$L timeout -k 10 300 python bench.py --workload $w $SW --no-cpu --no-compare > $O/${w}_$v$rep.json 2> $O/${w}_$v$rep.err || { tail -5 $O/${w}_$v$rep.err; exit 1; }
    python -c "import json; d=json.load(open('$O/${w}_$v$rep.json')); r=d['roofline']; p=d.get('phases',{}); print('$w', '${v:-new}', round(d['value']/1e6,2), round(r['frac'],4), round(r.get('kernel_ms',0),4), round(p.get('table_ms',0),3))"
  done
done; done
