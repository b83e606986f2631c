# r05al: λ ≥ 32 head round keys by DPP row broadcast from 8 VGPRs (no LDS key reads): compiler
# form (dppk: 2 v_mov_b32_dpp + v_bitop3 per word) and inline-asm form (dppk2: v_and_b32_dpp +
# v_xor_b32_dpp) vs the LDS key reads (default): wide parity with each, then C4, 3 alternating runs.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05al; mkdir -p $O
for v in dppk dppk2; do
  DCF_HIP_LIB=$PWD/dcf_amd/libdcf_hip_$v.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -k "wide or large_lambda" > $O/pytest_$v.log 2>&1 || { tail -60 $O/pytest_$v.log; exit 1; }
  echo "$v $(tail -1 $O/pytest_$v.log)"
done
for rep in 1 2 3; do
for v in default dppk dppk2; do
  if [ $v = default ]; then L=dcf_amd/libdcf_hip.so; else L=dcf_amd/libdcf_hip_$v.so; fi
  for w in c4; do
    SW="--steps 10 --warmup 3"
    DCF_HIP_LIB=$PWD/$L timeout -k 10 300 python bench.py --workload $w $SW --no-cpu --no-compare > $O/${w}_${v}_$rep.json 2> $O/${w}_${v}_$rep.err || { tail -20 $O/${w}_${v}_$rep.err; exit 1; }
    python -c "import json; d=json.load(open('$O/${w}_${v}_$rep.json')); r=d['roofline']; print('$w', '$v', $rep, round(d['ms_per_step'],4), round(r['frac'],4))" | tee -a $O/ab.txt
  done
done
done
