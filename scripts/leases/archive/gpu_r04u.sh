# r04u: C4 tail2 workgroup rounds continued: 8, 16, 32, 64 (64 = 32768-point ranges) — three alternating same-box runs each.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r04u; mkdir -p $O
for rep in 1 2 3; do for v in tr8 tr16 tr32 tr64; do
  DCF_HIP_LIB=$PWD/dcf_amd/libdcf_hip_$v.so timeout -k 10 300 python bench.py --workload c4 --steps 10 --warmup 3 --no-cpu --no-compare > $O/c4_${v}_$rep.json 2> $O/c4_${v}_$rep.err || { tail -20 $O/c4_${v}_$rep.err; exit 1; }
  python -c "import json; d=json.load(open('$O/c4_${v}_$rep.json')); r=d['roofline']; print('c4 $v', round(d['value']/1e6,2), round(d['ms_per_step'],3), round(r['frac'],4))"
done; done
