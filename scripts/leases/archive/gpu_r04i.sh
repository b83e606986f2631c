# r04i: C2 — a unit's x words loaded at claim and handed out by ds_bpermute (xpf1) vs loaded per point
# (xpf0): GPU suite on xpf1, 3 same-box runs each.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r04i; mkdir -p $O
DCF_HIP_LIB=$PWD/dcf_amd/libdcf_hip_xpf1.so timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > $O/pytest_xpf1.log 2>&1 || { tail -60 $O/pytest_xpf1.log; exit 1; }
tail -1 $O/pytest_xpf1.log
for rep in 1 2 3; do for v in xpf1 xpf0; do
  DCF_HIP_LIB=$PWD/dcf_amd/libdcf_hip_$v.so timeout -k 10 300 python bench.py --workload c2 --steps 60 --warmup 20 --no-cpu --no-compare > $O/c2_${v}_$rep.json 2> $O/c2_${v}_$rep.err || { tail -20 $O/c2_${v}_$rep.err; exit 1; }
  python -c "import json; d=json.load(open('$O/c2_${v}_$rep.json')); r=d['roofline']; print('c2 $v', round(d['value']/1e9,3), round(d['ms_per_step'],3), round(r['frac'],4), round(d['phases']['table_ms'],3), round(d['phases']['walk_ms'],3))"
done; done
