# r05g: round-5 kernel traces (C2, C4, C5) and PMC passes (FETCH_SIZE / WRITE_SIZE / SQ in separate
# runs, MI355X_MICROARCH.md) of the C3 and C4 launch shapes for bench.py's roofline.traffic.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05g; mkdir -p $O
for w in c2 c4 c5; do
  case $w in c2) SW="--steps 30 --warmup 5";; c4) SW="--steps 5 --warmup 2";; *) SW="--steps 2 --warmup 1";; esac
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/trace_$w -o trace -- python3 bench.py --workload $w $SW --no-cpu > $O/bench_trace_$w.json 2> $O/bench_trace_$w.err || { tail -20 $O/bench_trace_$w.err; exit 1; }
  python scripts/trace_summary.py $O/trace_$w --tail 12 > $O/prof_$w.md && rm -rf $O/trace_$w
  head -8 $O/prof_$w.md
done
TRAFFIC="k_eval_wide_head_stream+k_eval_wide_tail C4 4194304 16 16384 21 68786585600" bash scripts/leases/gpu_profile_w.sh r05g c4 || exit 1
TRAFFIC="k_eval16_stream C3 268435456 16 16 26 17179869184" bash scripts/leases/gpu_profile_w.sh r05g c3 || exit 1
