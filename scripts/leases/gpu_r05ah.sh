# r05ah: wave priority in k_gen16 (genprio), k_gen16 + the full-domain / top-tree builds (gfdprio),
# and the λ ≥ 32 MMO engine (mmowprio) vs the current default (stream / head / tail / MMO prio on):
# parity with each, then C5 and C4-MMO, 3 alternating runs.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05ah; mkdir -p $O
for v in genprio gfdprio mmowprio; do
  DCF_HIP_LIB=$PWD/dcf_amd/libdcf_hip_$v.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_mmo.py tests/test_gpu_fuzz.py -x -q --timeout 300 --timeout-method thread -k "gen or multikey or mmo or full_domain" > $O/pytest_$v.log 2>&1 || { tail -60 $O/pytest_$v.log; exit 1; }
  echo "$v $(tail -1 $O/pytest_$v.log)"
done
for rep in 1 2 3; do
for v in default genprio gfdprio mmowprio; do
  if [ $v = default ]; then L=dcf_amd/libdcf_hip.so; else L=dcf_amd/libdcf_hip_$v.so; fi
  case $v in mmowprio) WS="c4mmo";; default) WS="c5 c4mmo";; *) WS="c5";; esac
  for w in $WS; do
    case $w in c5) SW="--workload c5 --steps 5 --warmup 2";; c4mmo) SW="--workload c4 --prg mmo --steps 3 --warmup 1";; esac
    DCF_HIP_LIB=$PWD/$L timeout -k 10 300 python bench.py $SW --no-cpu --no-compare > $O/${w}_${v}_$rep.json 2> $O/${w}_${v}_$rep.err || { tail -20 $O/${w}_${v}_$rep.err; exit 1; }
    python -c "import json; d=json.load(open('$O/${w}_${v}_$rep.json')); r=d['roofline']; print('$w', '$v', $rep, round(d['ms_per_step'],4), round(r['frac'],4), d.get('gen_frac', ''))" | tee -a $O/ab.txt
  done
done
done
