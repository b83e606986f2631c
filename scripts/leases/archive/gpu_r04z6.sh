# r04z6: the round's last tree (after r04z5's suite) — every bench line (C3 as the driver runs it), the
# headline's rocprofv3 kernel trace in the same lease, C2 / C5 kernel traces.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r04z6; mkdir -p $O
timeout -k 10 600 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_c3.json 2> $O/bench_c3.err || { tail -20 $O/bench_c3.err; exit 1; }
python -c "import json; d=json.load(open('$O/bench_c3.json')); r=d['roofline']; print('c3', round(d['value']/1e6,1), round(r['frac'],4), d['ms_per_step'], d['cpu_baseline']['value'])"
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/trace -o trace -- python3 bench.py --steps 5 --warmup 2 --no-cpu --no-compare > $O/bench_trace.log 2>&1 || { tail -20 $O/bench_trace.log; exit 1; }
python scripts/lease_c3.py $O > $O/prof_c3.md && head -12 $O/prof_c3.md
for w in c1 c2 c4; do
  case $w in c1) SW="--steps 300 --warmup 100";; c2) SW="--steps 60 --warmup 20";; c4) SW="--steps 10 --warmup 3";; lat) SW="";; *) SW="--steps 3 --warmup 1";; esac
  timeout -k 10 500 python bench.py --workload $w $SW > $O/bench_$w.json 2> $O/bench_$w.err || { tail -20 $O/bench_$w.err; exit 1; }
  python -c "import json; d=json.load(open('$O/bench_$w.json')); r=d.get('roofline') or {}; print('$w', d['value'], r.get('frac'), (r.get('eval_only') or {}).get('frac'), (d.get('cpu_baseline') or {}).get('value'), (d.get('host_path') or {}).get('value'))"
done
for w in c5 fd lat; do
  case $w in c1) SW="--steps 300 --warmup 100";; c2) SW="--steps 60 --warmup 20";; c4) SW="--steps 10 --warmup 3";; lat) SW="";; *) SW="--steps 3 --warmup 1";; esac
  timeout -k 10 500 python bench.py --workload $w $SW > $O/bench_$w.json 2> $O/bench_$w.err || { tail -20 $O/bench_$w.err; exit 1; }
  python -c "import json; d=json.load(open('$O/bench_$w.json')); r=d.get('roofline') or {}; print('$w', d['value'], r.get('frac'), (r.get('eval_only') or {}).get('frac'), (d.get('cpu_baseline') or {}).get('value'), (d.get('host_path') or {}).get('value'))"
done
timeout -k 10 500 python bench.py --prg mmo --steps 3 --warmup 1 > $O/bench_mmo.json 2> $O/bench_mmo.err || { tail -20 $O/bench_mmo.err; exit 1; }
python -c "import json; d=json.load(open('$O/bench_mmo.json')); r=d['roofline']; print('mmo', d['value'], r['frac'])"
for w in c2 c5; do
  case $w in c2) SW="--steps 30 --warmup 5";; c4) SW="--steps 5 --warmup 2";; *) SW="--steps 2 --warmup 1";; esac
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/trace_$w -o trace -- python3 bench.py --workload $w $SW --no-cpu > $O/bench_trace_$w.json 2> $O/bench_trace_$w.err || { tail -20 $O/bench_trace_$w.err; exit 1; }
  python scripts/trace_summary.py $O/trace_$w --tail 12 > $O/prof_$w.md && rm -rf $O/trace_$w
  head -8 $O/prof_$w.md
done
