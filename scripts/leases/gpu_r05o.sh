# r05o: B reuse over whole runs of right steps at t = 0 in the single-key x-in-register stream
# instances (default) vs single-step reuse (libdcf_hip_nochain.so, -DDCF_REUSE_CHAIN=0): the
# eval parity tests with the default build, then C3 / C2 / C1 A/B, 3 alternating runs each,
# with the executed block count per eval.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05o; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_lat_threads.py tests/test_configs.py -x -q --timeout 300 --timeout-method thread -k "not wide and not large_lambda and not c4" > $O/pytest_eval.log 2>&1 || { tail -60 $O/pytest_eval.log; exit 1; }
tail -1 $O/pytest_eval.log
for rep in 1 2 3; do
for v in default nochain; do
  if [ $v = default ]; then L=dcf_amd/libdcf_hip.so; else L=dcf_amd/libdcf_hip_$v.so; fi
  DCF_HIP_LIB=$PWD/$L timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu --no-compare > $O/c3_${v}_$rep.json 2> $O/c3_${v}_$rep.err || { tail -20 $O/c3_${v}_$rep.err; exit 1; }
  python -c "import json; d=json.load(open('$O/c3_${v}_$rep.json')); r=d['roofline']; print('c3', '$v', $rep, round(d['ms_per_step'],3), '%.4g' % d['value'], round(r['frac'],4), r.get('executed_blocks_per_eval') or d.get('executed_blocks_per_eval'))" | tee -a $O/ab.txt
  DCF_HIP_LIB=$PWD/$L timeout -k 10 300 python bench.py --workload c2 --steps 60 --warmup 10 --no-cpu --no-compare > $O/c2_${v}_$rep.json 2> $O/c2_${v}_$rep.err || { tail -20 $O/c2_${v}_$rep.err; exit 1; }
  python -c "import json; d=json.load(open('$O/c2_${v}_$rep.json')); r=d['roofline']; print('c2', '$v', $rep, round(d['ms_per_step'],4), '%.4g' % d['value'], round(r['frac'],4), r.get('executed_blocks_per_eval') or d.get('executed_blocks_per_eval'))" | tee -a $O/ab.txt
  DCF_HIP_LIB=$PWD/$L timeout -k 10 300 python bench.py --workload c1 --steps 300 --warmup 100 --no-cpu --no-compare > $O/c1_${v}_$rep.json 2> $O/c1_${v}_$rep.err || { tail -20 $O/c1_${v}_$rep.err; exit 1; }
  python -c "import json; d=json.load(open('$O/c1_${v}_$rep.json')); r=d['roofline']; print('c1', '$v', $rep, round(d['ms_per_step'],4), '%.4g' % d['value'], round(r['frac'],4), r.get('executed_blocks_per_eval') or d.get('executed_blocks_per_eval'))" | tee -a $O/ab.txt
done
done
