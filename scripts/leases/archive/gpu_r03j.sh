# r03j: pair2 with the next pass's cw_s read ahead — small-batch parity subset, C1 A/B vs nop2
set -o pipefail
O=gpurun_out/r03j; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "eval_random or c1 or small or host or lat or gpu_parity" > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
for rep in 1 2 3; do for v in "" nop2; do
  L=$PWD/dcf_amd/libdcf_hip.so; [ -n "$v" ] && L=$PWD/dcf_amd/libdcf_hip_$v.so
  DCF_HIP_LIB=$L timeout -k 10 300 python bench.py --workload c1 --steps 300 --warmup 100 --no-cpu --no-compare > $O/c1_$v$rep.json 2> $O/c1_$v$rep.err || { tail -5 $O/c1_$v$rep.err; exit 1; }
  python -c "import json; d=json.load(open('$O/c1_$v$rep.json')); r=d['roofline']; print('c1', '${v:-default}', round(d['value']/1e6,2), round(r['frac'],4), round(r['kernel_ms'],4), round(r.get('executed_blocks_per_eval',0),1))"
done; done
