# r05h: same-box A/B of the round-4 library (git 2fda27a, libdcf_hip_r04.so) against this tree's on
# C3 (the driver's command shape, fewer steps) and C4: alternating, 3 runs each.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05h; mkdir -p $O
for rep in 1 2 3; do
for v in r04 r05; do
  if [ $v = r05 ]; then L=dcf_amd/libdcf_hip.so; else L=dcf_amd/libdcf_hip_r04.so; fi
  DCF_HIP_LIB=$PWD/$L timeout -k 10 300 python bench.py --steps 8 --warmup 3 --no-cpu --no-compare > $O/c3_${v}_$rep.json 2> $O/c3_${v}_$rep.err || { tail -20 $O/c3_${v}_$rep.err; exit 1; }
  python -c "import json; d=json.load(open('$O/c3_${v}_$rep.json')); print('c3', '$v', $rep, round(d['ms_per_step'],3), round(d['roofline']['frac'],4))" | tee -a $O/ab.txt
  DCF_HIP_LIB=$PWD/$L timeout -k 10 300 python bench.py --workload c4 --steps 10 --warmup 3 --no-cpu --no-compare > $O/c4_${v}_$rep.json 2> $O/c4_${v}_$rep.err || { tail -20 $O/c4_${v}_$rep.err; exit 1; }
  python -c "import json; d=json.load(open('$O/c4_${v}_$rep.json')); print('c4', '$v', $rep, round(d['ms_per_step'],3), round(d['roofline']['frac'],4))" | tee -a $O/ab.txt
done
done
