# r04g: GPU suite (root path of the table build on 16-lane rows; no counter fill before the first walk);
# C2 A/B: + the first build levels (<= 32 nodes) on 16-lane rows too (c2r); in-kernel timelines of both.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r04g; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -60 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
DCF_HIP_LIB=$PWD/dcf_amd/libdcf_hip_c2r.so timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread -k "prefix or full_domain or fd or c2 or c3 or config" > $O/pytest_c2r.log 2>&1 || { tail -40 $O/pytest_c2r.log; exit 1; }
echo "c2r $(tail -1 $O/pytest_c2r.log)"
for rep in 1 2 3; do for v in default c2r; do
  L=$PWD/dcf_amd/libdcf_hip.so; [ $v != default ] && L=$PWD/dcf_amd/libdcf_hip_$v.so
  DCF_HIP_LIB=$L timeout -k 10 300 python bench.py --workload c2 --steps 60 --warmup 5 --no-cpu --no-compare > $O/c2_${v}_$rep.json 2>/dev/null || exit 1
  python -c "import json; d=json.load(open('$O/c2_${v}_$rep.json')); r=d['roofline']; print('c2 $v', round(d['value']/1e9,3), round(d['ms_per_step'],3), round(r['frac'],4), round(d['phases']['table_ms'],3), round(d['phases']['walk_ms'],3))"
done; done
for v in clk clk_c2r; do
  DCF_HIP_LIB=$PWD/dcf_amd/libdcf_hip_$v.so timeout -k 10 300 python scripts/c2_timeline.py > $O/c2_timeline_$v.json 2> $O/c2_timeline_$v.err || { tail -30 $O/c2_timeline_$v.err; exit 1; }
  cat $O/c2_timeline_$v.json
done
