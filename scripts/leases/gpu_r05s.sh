# r05s: T1 lookups at state byte 1 addressed by one 2-cycle v_bitop3 ((w & 0xFF00) | slot) instead of
# a 4-cycle v_perm, in every T-table kernel (default) vs v_perm everywhere (libdcf_hip_t1off.so,
# -DDCF_T1_BITOP3=0): GPU suite with the default build, then C4 / C3 / C5 A/B, alternating runs.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05s; mkdir -p $O
timeout -k 10 800 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -60 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
for rep in 1 2 3; do
for v in default t1off; do
  if [ $v = default ]; then L=dcf_amd/libdcf_hip.so; else L=dcf_amd/libdcf_hip_$v.so; fi
  for w in c4 c3 c5; do
    case $w in c4) SW="--steps 10 --warmup 3";; c3) SW="--steps 10 --warmup 3";; c5) SW="--steps 5 --warmup 2";; esac
    DCF_HIP_LIB=$PWD/$L timeout -k 10 300 python bench.py --workload $w $SW --no-cpu --no-compare > $O/${w}_${v}_$rep.json 2> $O/${w}_${v}_$rep.err || { tail -20 $O/${w}_${v}_$rep.err; exit 1; }
    python -c "import json; d=json.load(open('$O/${w}_${v}_$rep.json')); r=d['roofline']; print('$w', '$v', $rep, round(d['ms_per_step'],3), round(r['frac'],4))" | tee -a $O/ab.txt
  done
done
done
