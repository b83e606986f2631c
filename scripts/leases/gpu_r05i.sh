# r05i: C4 head round keys from scalar loads (k0 and k0 ^ k17 per round, aes_tt_lka SK; libdcf_hip_hsk.so)
# vs per-lane LDS reads (default): LAMBDA >= 32 parity with the variant, then C4 A/B, 3 alternating runs.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05i; mkdir -p $O
DCF_HIP_LIB=$PWD/dcf_amd/libdcf_hip_hsk.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -k "wide or large_lambda" > $O/pytest_wide_hsk.log 2>&1 || { tail -60 $O/pytest_wide_hsk.log; exit 1; }
tail -1 $O/pytest_wide_hsk.log
for rep in 1 2 3; do
for v in default hsk; do
  if [ $v = default ]; then L=dcf_amd/libdcf_hip.so; else L=dcf_amd/libdcf_hip_$v.so; fi
  DCF_HIP_LIB=$PWD/$L timeout -k 10 300 python bench.py --workload c4 --steps 10 --warmup 3 --no-cpu --no-compare > $O/c4_${v}_$rep.json 2> $O/c4_${v}_$rep.err || { tail -20 $O/c4_${v}_$rep.err; exit 1; }
  python -c "import json; d=json.load(open('$O/c4_${v}_$rep.json')); print('c4', '$v', $rep, round(d['ms_per_step'],3), round(d['roofline']['frac'],4))" | tee -a $O/ab.txt
done
done
DCF_HIP_LIB=$PWD/dcf_amd/libdcf_hip_hsk.so timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/trace_c4 -o trace -- python3 bench.py --workload c4 --steps 5 --warmup 2 --no-cpu --no-compare > $O/bench_trace_c4.json 2> $O/bench_trace_c4.err || { tail -20 $O/bench_trace_c4.err; exit 1; }
python scripts/trace_summary.py $O/trace_c4 --tail 12 > $O/prof_c4_hsk.md && rm -rf $O/trace_c4
head -9 $O/prof_c4_hsk.md
