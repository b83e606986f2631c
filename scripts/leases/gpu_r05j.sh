# r05j: sorted tail (k_sort_* + k_eval_wide_tail2<9,2,1,true>, default) vs the same tree without it
# (libdcf_hip_nosort.so, -DDCF_T2_SORT=0) vs the committed round-5 library (libdcf_hip_head.so):
# LAMBDA >= 32 parity + the two-pass sorted config test, then C4 A/B, 3 alternating runs, + a trace.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05j; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -k "wide or large_lambda" > $O/pytest_wide.log 2>&1 || { tail -60 $O/pytest_wide.log; exit 1; }
tail -1 $O/pytest_wide.log
timeout -k 10 600 python -u -m pytest tests/test_configs.py -x -q --timeout 300 --timeout-method thread -k "sorted or c4" > $O/pytest_cfg.log 2>&1 || { tail -60 $O/pytest_cfg.log; exit 1; }
tail -1 $O/pytest_cfg.log
for rep in 1 2 3; do
for v in default nosort head; do
  if [ $v = default ]; then L=dcf_amd/libdcf_hip.so; else L=dcf_amd/libdcf_hip_$v.so; fi
  DCF_HIP_LIB=$PWD/$L timeout -k 10 300 python bench.py --workload c4 --steps 10 --warmup 3 --no-cpu --no-compare > $O/c4_${v}_$rep.json 2> $O/c4_${v}_$rep.err || { tail -20 $O/c4_${v}_$rep.err; exit 1; }
  python -c "import json; d=json.load(open('$O/c4_${v}_$rep.json')); print('c4', '$v', $rep, round(d['ms_per_step'],3), round(d['roofline']['frac'],4))" | tee -a $O/ab.txt
done
done
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/trace_c4 -o trace -- python3 bench.py --workload c4 --steps 5 --warmup 2 --no-cpu --no-compare > $O/bench_trace_c4.json 2> $O/bench_trace_c4.err || { tail -20 $O/bench_trace_c4.err; exit 1; }
python scripts/trace_summary.py $O/trace_c4 --tail 14 > $O/prof_c4_sorted.md && rm -rf $O/trace_c4
head -12 $O/prof_c4_sorted.md
