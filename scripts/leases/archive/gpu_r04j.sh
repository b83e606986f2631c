# r04j: C4 head — rounds 0 .. KR-1 of both key schedules in registers, picked per lane (wkrKR), the
# other rounds' keys read per lane from LDS as before (wkr0): parity (wide / C4 tests) and 2 same-box
# runs each.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r04j; mkdir -p $O
for v in wkr2 wkr4; do
  DCF_HIP_LIB=$PWD/dcf_amd/libdcf_hip_$v.so timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread -k "wide or c4" > $O/pytest_$v.log 2>&1 || { tail -40 $O/pytest_$v.log; exit 1; }
  echo "$v $(tail -1 $O/pytest_$v.log)"
done
for rep in 1 2; do for v in wkr0 wkr2 wkr4; do
  DCF_HIP_LIB=$PWD/dcf_amd/libdcf_hip_$v.so timeout -k 10 300 python bench.py --workload c4 --steps 10 --warmup 3 --no-cpu --no-compare > $O/c4_${v}_$rep.json 2> $O/c4_${v}_$rep.err || { tail -20 $O/c4_${v}_$rep.err; exit 1; }
  python -c "import json; d=json.load(open('$O/c4_${v}_$rep.json')); r=d['roofline']; print('c4 $v', round(d['value']/1e6,2), round(d['ms_per_step'],3), round(r['frac'],4))"
done; done
for v in wkr0 wkr4; do
  DCF_HIP_LIB=$PWD/dcf_amd/libdcf_hip_$v.so timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace_$v -o trace -- python3 bench.py --workload c4 --steps 5 --warmup 2 --no-cpu --no-compare > $O/trace_$v.log 2>&1 || { tail -20 $O/trace_$v.log; exit 1; }
  python scripts/trace_summary.py $O/trace_$v --tail 4 > $O/prof_c4_$v.md && rm -rf $O/trace_$v
  sed -n 5,7p $O/prof_c4_$v.md
done
