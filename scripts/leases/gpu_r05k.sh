# r05k: C5 multi-key stream instance with the x width fixed at N = 16 (default) vs the runtime-width
# instance (libdcf_hip_nbc0.so, -DDCF_MK_NBC16=0): multi-key parity + C5 config, then C5 A/B,
# 3 alternating runs, + a same-lease trace of the default.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05k; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -k "multikey or gen_batch" > $O/pytest_mk.log 2>&1 || { tail -60 $O/pytest_mk.log; exit 1; }
tail -1 $O/pytest_mk.log
timeout -k 10 600 python -u -m pytest tests/test_configs.py -x -q --timeout 300 --timeout-method thread -k "c5" > $O/pytest_cfg.log 2>&1 || { tail -60 $O/pytest_cfg.log; exit 1; }
tail -1 $O/pytest_cfg.log
for rep in 1 2 3; do
for v in default nbc0; do
  if [ $v = default ]; then L=dcf_amd/libdcf_hip.so; else L=dcf_amd/libdcf_hip_$v.so; fi
  DCF_HIP_LIB=$PWD/$L timeout -k 10 300 python bench.py --workload c5 --steps 10 --warmup 3 --no-cpu --no-compare > $O/c5_${v}_$rep.json 2> $O/c5_${v}_$rep.err || { tail -20 $O/c5_${v}_$rep.err; exit 1; }
  python -c "import json; d=json.load(open('$O/c5_${v}_$rep.json')); print('c5', '$v', $rep, round(d['ms_per_step'],3), round(d['roofline']['frac'],4), round(d['roofline']['eval_only']['frac'],4))" | tee -a $O/ab.txt
done
done
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/trace_c5 -o trace -- python3 bench.py --workload c5 --steps 5 --warmup 2 --no-cpu --no-compare > $O/bench_trace_c5.json 2> $O/bench_trace_c5.err || { tail -20 $O/bench_trace_c5.err; exit 1; }
python scripts/trace_summary.py $O/trace_c5 --tail 8 > $O/prof_c5.md && rm -rf $O/trace_c5
head -12 $O/prof_c5.md
