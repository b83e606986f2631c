# r04e: C5 A/B — tiled key-major digest (c5v1), one-thread-per-key depth-first top trees (c5v2),
# both (c5v3) vs the current kernels: parity of each variant (multi-key tests), 2 same-box bench
# runs each, and a kernel trace of c5v3.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r04e; mkdir -p $O
for v in c5v1 c5v2 c5v3; do
  DCF_HIP_LIB=$PWD/dcf_amd/libdcf_hip_$v.so timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread -k "multikey or c5 or multi_gpu" > $O/pytest_$v.log 2>&1 || { tail -40 $O/pytest_$v.log; exit 1; }
  echo "$v $(tail -1 $O/pytest_$v.log)"
done
for rep in 1 2; do for v in default c5v1 c5v2 c5v3; do
  L=$PWD/dcf_amd/libdcf_hip.so; [ $v != default ] && L=$PWD/dcf_amd/libdcf_hip_$v.so
  DCF_HIP_LIB=$L timeout -k 10 300 python bench.py --workload c5 --steps 3 --warmup 1 --no-cpu --no-compare > $O/c5_${v}_$rep.json 2>/dev/null || exit 1
  python -c "import json; d=json.load(open('$O/c5_${v}_$rep.json')); r=d['roofline']; print('c5 $v', round(d['value']/1e6,2), round(d['ms_per_step'],2), round(r['frac'],4), 'eval_only', round(r['eval_only']['frac'],4), d['phases_ms'])"
done; done
DCF_HIP_LIB=$PWD/dcf_amd/libdcf_hip_c5v3.so timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace_c5 -o trace -- python3 bench.py --workload c5 --steps 2 --warmup 1 --no-cpu --no-compare > $O/trace_c5.log 2>&1 || { tail -20 $O/trace_c5.log; exit 1; }
python scripts/trace_summary.py $O/trace_c5 --tail 10 > $O/prof_c5v3.md && rm -rf $O/trace_c5
head -14 $O/prof_c5v3.md
# C2: narrow levels of the table build in LDS (c2v) vs global buffers: parity (prefix / full-domain / C2 tests), 3 same-box runs each
DCF_HIP_LIB=$PWD/dcf_amd/libdcf_hip_c2v.so timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread -k "prefix or full_domain or fd or c2 or c3" > $O/pytest_c2v.log 2>&1 || { tail -40 $O/pytest_c2v.log; exit 1; }
echo "c2v $(tail -1 $O/pytest_c2v.log)"
for rep in 1 2 3; do for v in default c2v; do
  L=$PWD/dcf_amd/libdcf_hip.so; [ $v != default ] && L=$PWD/dcf_amd/libdcf_hip_$v.so
  DCF_HIP_LIB=$L timeout -k 10 300 python bench.py --workload c2 --steps 60 --warmup 5 --no-cpu --no-compare > $O/c2_${v}_$rep.json 2>/dev/null || exit 1
  python -c "import json; d=json.load(open('$O/c2_${v}_$rep.json')); r=d['roofline']; print('c2 $v', round(d['value']/1e9,3), round(d['ms_per_step'],3), round(r['frac'],4), d.get('phases'))"
done; done
