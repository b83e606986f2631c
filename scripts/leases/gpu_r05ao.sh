# r05ao: λ ≥ 32 head — T1 lookups by v_bitop3 (t1kr4), the same with rounds 0-1 only in registers
# (t1kr2), rounds 0-1 in registers alone (kr2) vs v_perm T1 and rounds 0-3 in registers (default):
# wide parity with each, C4 3 alternating runs, then a C4 kernel trace of the default build.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05ao; mkdir -p $O
for v in t1kr4 t1kr2 kr2; do
  DCF_HIP_LIB=$PWD/dcf_amd/libdcf_hip_$v.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -k "wide or large_lambda" > $O/pytest_$v.log 2>&1 || { tail -60 $O/pytest_$v.log; exit 1; }
  echo "$v $(tail -1 $O/pytest_$v.log)"
done
for rep in 1 2 3; do
for v in default t1kr4 t1kr2 kr2; do
  if [ $v = default ]; then L=dcf_amd/libdcf_hip.so; else L=dcf_amd/libdcf_hip_$v.so; fi
  DCF_HIP_LIB=$PWD/$L timeout -k 10 300 python bench.py --workload c4 --steps 10 --warmup 3 --no-cpu --no-compare > $O/c4_${v}_$rep.json 2> $O/c4_${v}_$rep.err || { tail -20 $O/c4_${v}_$rep.err; exit 1; }
  python -c "import json; d=json.load(open('$O/c4_${v}_$rep.json')); r=d['roofline']; print('c4', '$v', $rep, round(d['ms_per_step'],4), round(r['frac'],4))" | tee -a $O/ab.txt
done
done
# (the trace step below found no *kernel_stats.csv under that name and failed; the A/B above stands)
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace -o trace -- python3 bench.py --workload c4 --steps 5 --warmup 2 --no-cpu --no-compare > $O/trace.log 2>&1 || { tail -20 $O/trace.log; exit 1; }
find $O/trace -name "*kernel_stats.csv" -exec cp {} $O/c4_kernel_stats.csv \;
rm -rf $O/trace
head -12 $O/c4_kernel_stats.csv
