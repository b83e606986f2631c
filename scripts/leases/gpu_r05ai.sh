# r05ai: wave priority in the small-batch pair walk (pairprio: k_eval16_pair / k_eval16 AES at
# s_setprio 1) vs none: parity with the variant, then C1, 4 alternating runs.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05ai; mkdir -p $O
DCF_HIP_LIB=$PWD/dcf_amd/libdcf_hip_pairprio.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fuzz.py -x -q --timeout 300 --timeout-method thread -k "eval_random or small_pair or golden or multikey or host_mid" > $O/pytest_pairprio.log 2>&1 || { tail -60 $O/pytest_pairprio.log; exit 1; }
echo "pairprio $(tail -1 $O/pytest_pairprio.log)"
for rep in 1 2 3 4; do
for v in default pairprio; do
  if [ $v = default ]; then L=dcf_amd/libdcf_hip.so; else L=dcf_amd/libdcf_hip_$v.so; fi
  DCF_HIP_LIB=$PWD/$L timeout -k 10 300 python bench.py --workload c1 --steps 300 --warmup 100 --no-cpu --no-compare > $O/c1_${v}_$rep.json 2> $O/c1_${v}_$rep.err || { tail -20 $O/c1_${v}_$rep.err; exit 1; }
  python -c "import json; d=json.load(open('$O/c1_${v}_$rep.json')); r=d['roofline']; print('c1', '$v', $rep, round(d['ms_per_step'],4), round(r['frac'],4))" | tee -a $O/ab.txt
done
done
