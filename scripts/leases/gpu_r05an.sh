# r05an: wave-priority skew — odd waves run their AES rounds at s_setprio 2, even waves at 1 (skew),
# vs all at 1 (default), in the stream engine and the λ ≥ 32 head: parity with the variant, then
# C3 / C4 / C2 / C5, 3 alternating runs.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05an; mkdir -p $O
DCF_HIP_LIB=$PWD/dcf_amd/libdcf_hip_skew.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -k "eval_random or prefix_table or multikey or device_large or wide" > $O/pytest_skew.log 2>&1 || { tail -60 $O/pytest_skew.log; exit 1; }
echo "skew $(tail -1 $O/pytest_skew.log)"
for rep in 1 2 3; do
for v in default skew; do
  if [ $v = default ]; then L=dcf_amd/libdcf_hip.so; else L=dcf_amd/libdcf_hip_$v.so; fi
  for w in c3 c4 c2 c5; do
    case $w in c3) SW="--steps 10 --warmup 3";; c4) SW="--steps 10 --warmup 3";; c2) SW="--steps 60 --warmup 10";; c5) SW="--steps 5 --warmup 2";; esac
    DCF_HIP_LIB=$PWD/$L timeout -k 10 300 python bench.py --workload $w $SW --no-cpu --no-compare > $O/${w}_${v}_$rep.json 2> $O/${w}_${v}_$rep.err || { tail -20 $O/${w}_${v}_$rep.err; exit 1; }
    python -c "import json; d=json.load(open('$O/${w}_${v}_$rep.json')); r=d['roofline']; print('$w', '$v', $rep, round(d['ms_per_step'],4), round(r['frac'],4))" | tee -a $O/ab.txt
  done
done
done
