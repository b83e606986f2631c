# r05aa: C5 multi-key instance with point -> key by a shift for a power-of-two points per key
# (default) vs the division sequence (libdcf_hip_pk2off.so, -DDCF_MK_PK2=0): multi-key parity,
# fuzz sweep, C5 config, then C5 A/B, 3 alternating runs.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05aa; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fuzz.py tests/test_configs.py -x -q --timeout 300 --timeout-method thread -k "multikey or gen_batch or fuzz or c5" > $O/pytest.log 2>&1 || { tail -60 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for rep in 1 2 3; do
for v in default pk2off; do
  if [ $v = default ]; then L=dcf_amd/libdcf_hip.so; else L=dcf_amd/libdcf_hip_$v.so; fi
  DCF_HIP_LIB=$PWD/$L timeout -k 10 300 python bench.py --workload c5 --steps 5 --warmup 2 --no-cpu --no-compare > $O/c5_${v}_$rep.json 2> $O/c5_${v}_$rep.err || { tail -20 $O/c5_${v}_$rep.err; exit 1; }
  python -c "import json; d=json.load(open('$O/c5_${v}_$rep.json')); r=d['roofline']; print('c5', '$v', $rep, round(d['ms_per_step'],3), round(r['frac'],4), round(r['eval_only']['frac'],4))" | tee -a $O/ab.txt
done
done
