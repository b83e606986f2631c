# r04h: GPU suite; C5 A/B: per-key top trees on a second stream beside a 32-key x 16-level digest
# (default) vs the round's previous tree (c5old: serial, 16-key digest); a C5 kernel trace.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r04h; mkdir -p $O
# (the GPU suite of this tree ran in the first r04h call: profiles/r04h_pytest_gpu.log)
for rep in 1 2 3; do for v in default c5old; do
  L=$PWD/dcf_amd/libdcf_hip.so; [ $v != default ] && L=$PWD/dcf_amd/libdcf_hip_$v.so
  DCF_HIP_LIB=$L timeout -k 10 300 python bench.py --workload c5 --steps 3 --warmup 1 --no-cpu --no-compare > $O/c5_${v}_$rep.json 2> $O/c5_${v}_$rep.err || { tail -20 $O/c5_${v}_$rep.err; exit 1; }
  python -c "import json; d=json.load(open('$O/c5_${v}_$rep.json')); r=d['roofline']; print('c5 $v', round(d['value']/1e6,2), round(d['ms_per_step'],2), round(r['frac'],4), 'eval_only', round(r['eval_only']['frac'],4), round(d['phases_ms']['eval_party0'],2), round(d['phases_ms']['eval_party1'],2))"
done; done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace_c5 -o trace -- python3 bench.py --workload c5 --steps 2 --warmup 1 --no-cpu --no-compare > $O/trace_c5.log 2>&1 || { tail -20 $O/trace_c5.log; exit 1; }
python scripts/trace_summary.py $O/trace_c5 --tail 12 > $O/prof_c5.md && rm -rf $O/trace_c5
cat $O/prof_c5.md
timeout -k 10 300 python scripts/wide_mk_bench.py 128 4096 64 > $O/wide_mk_128.json 2> $O/wide_mk.err || { tail -20 $O/wide_mk.err; exit 1; }
cat $O/wide_mk_128.json
timeout -k 10 300 python scripts/wide_mk_bench.py 1024 2048 32 > $O/wide_mk_1024.json 2>> $O/wide_mk.err || { tail -20 $O/wide_mk.err; exit 1; }
cat $O/wide_mk_1024.json
