# r05ad: C4 paired-slot tail, regions per read batch (reads issued before their XORs): 2 (default)
# vs 3 (libdcf_hip_bt3.so) vs 4 (libdcf_hip_bt4.so): LAMBDA >= 32 parity with each, then C4,
# 3 alternating runs.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05ad; mkdir -p $O
for v in bt3 bt4; do
  DCF_HIP_LIB=$PWD/dcf_amd/libdcf_hip_$v.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -k "wide or large_lambda" > $O/pytest_$v.log 2>&1 || { tail -60 $O/pytest_$v.log; exit 1; }
  echo "$v $(tail -1 $O/pytest_$v.log)"
done
for rep in 1 2 3; do
for v in default bt3 bt4; do
  if [ $v = default ]; then L=dcf_amd/libdcf_hip.so; else L=dcf_amd/libdcf_hip_$v.so; fi
  DCF_HIP_LIB=$PWD/$L timeout -k 10 300 python bench.py --workload c4 --steps 10 --warmup 3 --no-cpu --no-compare > $O/c4_${v}_$rep.json 2> $O/c4_${v}_$rep.err || { tail -20 $O/c4_${v}_$rep.err; exit 1; }
  python -c "import json; d=json.load(open('$O/c4_${v}_$rep.json')); print('c4', '$v', $rep, round(d['ms_per_step'],3), round(d['roofline']['frac'],4))" | tee -a $O/ab.txt
done
done
