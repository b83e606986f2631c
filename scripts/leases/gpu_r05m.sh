# r05m: C2 refill latency — L2 prefetch of the table row of the point 128 places ahead (LDS-DMA
# load into a dump area, issued after the iteration's refills) x round keys from the device copy
# (default) or SGPRs, N = 4 single-key instance: parity of each build, then C2, 3 alternating runs.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05m; mkdir -p $O
for v in default c2a1k0 c2a0k1 c2a1k1; do
  if [ $v = default ]; then L=dcf_amd/libdcf_hip.so; else L=dcf_amd/libdcf_hip_$v.so; fi
  DCF_HIP_LIB=$PWD/$L timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -k "eval_random_vs or prefix_table or device_large" > $O/pytest_$v.log 2>&1 || { tail -40 $O/pytest_$v.log; exit 1; }
  echo "$v $(tail -1 $O/pytest_$v.log)"
done
for rep in 1 2 3; do
for v in default c2a1k0 c2a0k1 c2a1k1; do
  if [ $v = default ]; then L=dcf_amd/libdcf_hip.so; else L=dcf_amd/libdcf_hip_$v.so; fi
  DCF_HIP_LIB=$PWD/$L timeout -k 10 300 python bench.py --workload c2 --steps 60 --warmup 10 --no-cpu --no-compare > $O/c2_${v}_$rep.json 2> $O/c2_${v}_$rep.err || { tail -20 $O/c2_${v}_$rep.err; exit 1; }
  python -c "import json; d=json.load(open('$O/c2_${v}_$rep.json')); print('c2', '$v', $rep, round(d['ms_per_step'],4), '%.4g' % d['value'], round(d['roofline']['frac'],4))" | tee -a $O/ab.txt
done
done
