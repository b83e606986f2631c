# r04o: tail2 with register rows (N = 16: 9 six-bit + 1 five-bit regions + 11 register rows, 20 LDS
# reads per 16 B of y) vs the (5,7) layout (24 reads): wide parity on the default build, then C4
# A/B, three alternating same-box runs (rr = default layouts, r57 = -DDCF_TAIL2_R57).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r04o; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread -k "wide or c4" > $O/pytest_wide.log 2>&1 || { tail -60 $O/pytest_wide.log; exit 1; }
tail -1 $O/pytest_wide.log
for rep in 1 2 3; do for v in rr r57; do
  DCF_HIP_LIB=$PWD/dcf_amd/libdcf_hip_$v.so timeout -k 10 300 python bench.py --workload c4 --steps 10 --warmup 3 --no-cpu --no-compare > $O/c4_${v}_$rep.json 2> $O/c4_${v}_$rep.err || { tail -20 $O/c4_${v}_$rep.err; exit 1; }
  python -c "import json; d=json.load(open('$O/c4_${v}_$rep.json')); r=d['roofline']; print('c4 $v', round(d['value']/1e6,2), round(d['ms_per_step'],3), round(r['frac'],4))"
done; done
