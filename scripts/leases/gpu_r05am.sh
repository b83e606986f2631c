# r05am: B reuse over whole runs of right steps at t = 0 (DCF_REUSE_RUN, rrun), retried now that the
# walk runs below the AES rounds in wave priority, vs the default: eval parity (incl. the fuzz sweep) with
# the variant, then C3 / C2 / C5, 3 alternating runs.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05am; mkdir -p $O
for v in rrun; do
  DCF_HIP_LIB=$PWD/dcf_amd/libdcf_hip_$v.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fuzz.py tests/test_configs.py -x -q --timeout 300 --timeout-method thread -k "eval or reuse or multikey or fuzz or c1 or c2 or c3 or c5" > $O/pytest_$v.log 2>&1 || { tail -60 $O/pytest_$v.log; exit 1; }
  echo "$v $(tail -1 $O/pytest_$v.log)"
done
for rep in 1 2 3; do
for v in default rrun; do
  if [ $v = default ]; then L=dcf_amd/libdcf_hip.so; else L=dcf_amd/libdcf_hip_$v.so; fi
  for w in c3 c2 c5; do
    case $w in c3) SW="--steps 10 --warmup 3";; c2) SW="--steps 60 --warmup 10";; c5) SW="--steps 5 --warmup 2";; esac
    DCF_HIP_LIB=$PWD/$L timeout -k 10 300 python bench.py --workload $w $SW --no-cpu --no-compare > $O/${w}_${v}_$rep.json 2> $O/${w}_${v}_$rep.err || { tail -20 $O/${w}_${v}_$rep.err; exit 1; }
    python -c "import json; d=json.load(open('$O/${w}_${v}_$rep.json')); r=d['roofline']; print('$w', '$v', $rep, round(d['ms_per_step'],4), round(r['frac'],4))" | tee -a $O/ab.txt
  done
done
done
