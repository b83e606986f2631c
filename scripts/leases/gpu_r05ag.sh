# r05ag: wave priority in the full-domain / prefix-build AES (fdprio: fd_children, k_fd_level16)
# and in the MMO engine (mmoprio) vs the current default (head/tail prio on): parity with each
# variant, the GPU suite with the default build, then FD / C3 / C3-MMO, 3 alternating runs.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05ag; mkdir -p $O
timeout -k 10 800 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -60 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
for v in fdprio mmoprio; do
  DCF_HIP_LIB=$PWD/dcf_amd/libdcf_hip_$v.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_mmo.py -x -q --timeout 300 --timeout-method thread -k "full_domain or prefix or mmo or eval_random" > $O/pytest_$v.log 2>&1 || { tail -60 $O/pytest_$v.log; exit 1; }
  echo "$v $(tail -1 $O/pytest_$v.log)"
done
for rep in 1 2 3; do
for v in default fdprio mmoprio; do
  if [ $v = default ]; then L=dcf_amd/libdcf_hip.so; else L=dcf_amd/libdcf_hip_$v.so; fi
  for w in fd c3 c3mmo; do
    case $w in fd) SW="--workload fd --steps 10 --warmup 3";; c3) SW="--workload c3 --steps 10 --warmup 3";; c3mmo) SW="--workload c3 --prg mmo --steps 10 --warmup 3";; esac
    DCF_HIP_LIB=$PWD/$L timeout -k 10 300 python bench.py $SW --no-cpu --no-compare > $O/${w}_${v}_$rep.json 2> $O/${w}_${v}_$rep.err || { tail -20 $O/${w}_${v}_$rep.err; exit 1; }
    python -c "import json; d=json.load(open('$O/${w}_${v}_$rep.json')); r=d['roofline']; print('$w', '$v', $rep, round(d['ms_per_step'],4), round(r['frac'],4))" | tee -a $O/ab.txt
  done
done
done
