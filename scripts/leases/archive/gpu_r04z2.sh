# r04z2: final round-4 tree, second lease — C5 / full-domain / single-call / MMO bench lines and the
# C4 / C2 / C5 kernel traces.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r04z; mkdir -p $O
for w in c5 fd lat; do
  case $w in c1) SW="--steps 300 --warmup 100";; c2) SW="--steps 60 --warmup 20";; c4) SW="--steps 10 --warmup 3";; lat) SW="";; *) SW="--steps 3 --warmup 1";; esac
  timeout -k 10 500 python bench.py --workload $w $SW > $O/bench_$w.json 2> $O/bench_$w.err || { tail -20 $O/bench_$w.err; exit 1; }
  python -c "import json; d=json.load(open('$O/bench_$w.json')); r=d.get('roofline') or {}; print('$w', d['value'], r.get('frac'), (r.get('eval_only') or {}).get('frac'), (d.get('cpu_baseline') or {}).get('value'), (d.get('host_path') or {}).get('value'))"
done
timeout -k 10 500 python bench.py --prg mmo --steps 3 --warmup 1 > $O/bench_mmo.json 2> $O/bench_mmo.err || { tail -20 $O/bench_mmo.err; exit 1; }
python -c "import json; d=json.load(open('$O/bench_mmo.json')); r=d['roofline']; print('mmo', d['value'], r['frac'])"
for w in c4 c2 c5; do
  case $w in c2) SW="--steps 30 --warmup 5";; c4) SW="--steps 5 --warmup 2";; *) SW="--steps 2 --warmup 1";; esac
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/trace_$w -o trace -- python3 bench.py --workload $w $SW --no-cpu > $O/bench_trace_$w.json 2> $O/bench_trace_$w.err || { tail -20 $O/bench_trace_$w.err; exit 1; }
  python scripts/trace_summary.py $O/trace_$w --tail 12 > $O/prof_$w.md && rm -rf $O/trace_$w
  head -8 $O/prof_$w.md
done
