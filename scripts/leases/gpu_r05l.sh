# r05l: batched gen (k_gen16) with round keys from the device copy (default) vs 60 SGPR keys
# (libdcf_hip_gensgpr.so, -DDCF_GEN_GK=0): gen parity + C5 config, then C5 A/B (gen phase),
# 3 alternating runs.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05l; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_lat_threads.py -x -q --timeout 300 --timeout-method thread -k "gen" > $O/pytest_gen.log 2>&1 || { tail -60 $O/pytest_gen.log; exit 1; }
tail -1 $O/pytest_gen.log
timeout -k 10 600 python -u -m pytest tests/test_configs.py -x -q --timeout 300 --timeout-method thread -k "c5" > $O/pytest_cfg.log 2>&1 || { tail -60 $O/pytest_cfg.log; exit 1; }
tail -1 $O/pytest_cfg.log
for rep in 1 2 3; do
for v in default gensgpr; do
  if [ $v = default ]; then L=dcf_amd/libdcf_hip.so; else L=dcf_amd/libdcf_hip_$v.so; fi
  DCF_HIP_LIB=$PWD/$L timeout -k 10 300 python bench.py --workload c5 --steps 10 --warmup 3 --no-cpu --no-compare > $O/c5_${v}_$rep.json 2> $O/c5_${v}_$rep.err || { tail -20 $O/c5_${v}_$rep.err; exit 1; }
  python -c "import json; d=json.load(open('$O/c5_${v}_$rep.json')); print('c5', '$v', $rep, round(d['ms_per_step'],3), round(d['roofline']['frac'],4), 'gen_ms', round(d['phases_ms']['gen'],3), 'gen_frac', round(d['roofline']['gen_only']['frac'],4))" | tee -a $O/ab.txt
done
done
