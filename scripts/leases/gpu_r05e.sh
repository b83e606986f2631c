# r05e: C4 tail A/B — r04 layout (5,7) with the LDS block counter (t2r0) vs the party-folded (9,2)
# layout with a global per-workgroup counter claimed 1 / 4 (default) / 16 blocks at a time, one
# 128-B line per counter (t2s1: packed counters).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05e; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -k "wide_tail2 or large_lambda" > $O/pytest_wide.log 2>&1 || { tail -60 $O/pytest_wide.log; exit 1; }
tail -1 $O/pytest_wide.log
for rep in 1 2; do
for v in t2r0 default t2c1 t2c16 t2s1; do
  if [ $v = default ]; then L=dcf_amd/libdcf_hip.so; else L=dcf_amd/libdcf_hip_$v.so; fi
  DCF_HIP_LIB=$PWD/$L timeout -k 10 300 python bench.py --workload c4 --steps 10 --warmup 3 --no-cpu --no-compare > $O/c4_${v}_$rep.json 2> $O/c4_${v}_$rep.err || { tail -20 $O/c4_${v}_$rep.err; exit 1; }
  python -c "import json; d=json.load(open('$O/c4_${v}_$rep.json')); print('$v', $rep, round(d['ms_per_step'],3), round(d['roofline']['frac'],4))" | tee -a $O/ab.txt
done
done
