# r04l: C4 head at 8 waves per CU with more key rounds in registers (whv1: 2 streams/lane, all 15
# rounds — spills; whv2: 2 streams, 8 rounds; whv3: 1 stream, 15 rounds; whv4: 2 streams, 10 rounds)
# vs the default (whv0: 16 waves, 1 stream, 4 rounds): parity of whv2/whv4, 2 same-box runs each.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r04l; mkdir -p $O
for v in whv2 whv4; do
  DCF_HIP_LIB=$PWD/dcf_amd/libdcf_hip_$v.so timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread -k "wide or c4" > $O/pytest_$v.log 2>&1 || { tail -40 $O/pytest_$v.log; exit 1; }
  echo "$v $(tail -1 $O/pytest_$v.log)"
done
for rep in 1 2; do for v in whv0 whv1 whv2 whv3 whv4; do
  DCF_HIP_LIB=$PWD/dcf_amd/libdcf_hip_$v.so timeout -k 10 300 python bench.py --workload c4 --steps 10 --warmup 3 --no-cpu --no-compare > $O/c4_${v}_$rep.json 2> $O/c4_${v}_$rep.err || { tail -20 $O/c4_${v}_$rep.err; exit 1; }
  python -c "import json; d=json.load(open('$O/c4_${v}_$rep.json')); r=d['roofline']; print('c4 $v', round(d['value']/1e6,2), round(d['ms_per_step'],3), round(r['frac'],4))"
done; done
