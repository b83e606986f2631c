# r04d: GPU suite (N >= 32 at LAMBDA >= 32), then the C4 tail with LDS + L2-resident global 8-bit chunk tables: parity of each split (wide tests) and
# a same-box A/B against the LDS-only tail (default lib: (5,7,0); t3gG: G 8-bit chunks in global memory).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r04d2; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -60 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
for v in t3g3 t3g4 t3g5; do
  DCF_HIP_LIB=$PWD/dcf_amd/libdcf_hip_$v.so timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread -k "wide or c4" > $O/pytest_$v.log 2>&1 || { tail -40 $O/pytest_$v.log; exit 1; }
  echo "$v $(tail -1 $O/pytest_$v.log)"
done
for rep in 1 2; do for v in default t3g3 t3g4 t3g5; do
  L=$PWD/dcf_amd/libdcf_hip.so; [ $v != default ] && L=$PWD/dcf_amd/libdcf_hip_$v.so
  DCF_HIP_LIB=$L timeout -k 10 300 python bench.py --workload c4 --steps 10 --warmup 3 --no-cpu --no-compare > $O/c4_${v}_$rep.json 2>/dev/null || exit 1
  python -c "import json; d=json.load(open('$O/c4_${v}_$rep.json')); r=d['roofline']; print('c4 $v', round(d['value']/1e6,2), round(d['ms_per_step'],3), round(r['frac'],4))"
done; done
# C2 in-kernel timeline (prefix-table build phases vs the walk), clock-stamp build
DCF_HIP_LIB=$PWD/dcf_amd/libdcf_hip_clk.so timeout -k 10 300 python scripts/c2_timeline.py > $O/c2_timeline.json 2> $O/c2_timeline.err || { tail -30 $O/c2_timeline.err; exit 1; }
cat $O/c2_timeline.json
