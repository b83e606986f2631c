# r05aj: stream loop wave priority beyond the AES rounds: the CW loads at the loop top at 1 too (sp3),
# and the stores / refill as well, only the level update at 0 (sp4), vs the default (AES rounds at 1):
# eval parity with each, then C3 / C2 / C5, 3 alternating runs.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05aj; mkdir -p $O
for v in sp3 sp4; do
  DCF_HIP_LIB=$PWD/dcf_amd/libdcf_hip_$v.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -k "eval_random or prefix_table or multikey or device_large" > $O/pytest_$v.log 2>&1 || { tail -60 $O/pytest_$v.log; exit 1; }
  echo "$v $(tail -1 $O/pytest_$v.log)"
done
for rep in 1 2 3; do
for v in default sp3 sp4; do
  if [ $v = default ]; then L=dcf_amd/libdcf_hip.so; else L=dcf_amd/libdcf_hip_$v.so; fi
  for w in c3 c2 c5; do
    case $w in c3) SW="--steps 10 --warmup 3";; c2) SW="--steps 60 --warmup 10";; c5) SW="--steps 5 --warmup 2";; esac
    DCF_HIP_LIB=$PWD/$L timeout -k 10 300 python bench.py --workload $w $SW --no-cpu --no-compare > $O/${w}_${v}_$rep.json 2> $O/${w}_${v}_$rep.err || { tail -20 $O/${w}_${v}_$rep.err; exit 1; }
    python -c "import json; d=json.load(open('$O/${w}_${v}_$rep.json')); r=d['roofline']; print('$w', '$v', $rep, round(d['ms_per_step'],4), round(r['frac'],4))" | tee -a $O/ab.txt
  done
done
done
