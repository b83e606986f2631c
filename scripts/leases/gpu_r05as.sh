# r05as (3rd lease): C2 with prefix rows staged ahead into LDS by DMA — stg (SGPR round keys, DMA at
# the iteration's end), stge (SGPR keys, DMA right after the CW wait), stggke (device-copy keys, DMA
# after the CW wait) — vs the default.  2nd lease (r05as2): stg / stggk / sk (SGPR keys alone).
# parity with both staged builds (prefix / device / fuzz / C2 config tests), then C2, 4 alternating
# runs.  (The first lease of this script, gpurun_out/r05as, also ran lds32 — the 32 KiB area
# allocated, unused: no change — and found 32-point counter claims 2x slower: contention.)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05as3; mkdir -p $O
for pv in stge stggke; do
DCF_HIP_LIB=$PWD/dcf_amd/libdcf_hip_$pv.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fuzz.py tests/test_configs.py -x -q --timeout 300 --timeout-method thread -k "prefix or device_large or eval_random or fuzz_single or c2" > $O/pytest_$pv.log 2>&1 || { tail -60 $O/pytest_$pv.log; exit 1; }
echo "$pv $(tail -1 $O/pytest_$pv.log)"
done
for rep in 1 2 3 4; do
for v in default stg stge stggke; do
  if [ $v = default ]; then L=dcf_amd/libdcf_hip.so; else L=dcf_amd/libdcf_hip_$v.so; fi
  DCF_HIP_LIB=$PWD/$L timeout -k 10 300 python bench.py --workload c2 --steps 60 --warmup 10 --no-cpu --no-compare > $O/c2_${v}_$rep.json 2> $O/c2_${v}_$rep.err || { tail -20 $O/c2_${v}_$rep.err; exit 1; }
  python -c "import json; d=json.load(open('$O/c2_${v}_$rep.json')); r=d['roofline']; print('c2', '$v', $rep, round(d['ms_per_step'],4), round(r['frac'],4), round(d['phases']['walk_ms'],3))" | tee -a $O/ab.txt
done
done
