# r05at: final round-5 tree with the C2 staged rows (DCF_STG) — GPU suite, smoke, every bench line (C3 as the driver runs it) with the
# headline's rocprofv3 kernel trace in the same lease as its bench line.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05at; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -60 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 600 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_c3.json 2> $O/bench_c3.err || { tail -20 $O/bench_c3.err; exit 1; }
python -c "import json; d=json.load(open('$O/bench_c3.json')); r=d['roofline']; print('c3', round(d['value']/1e6,1), round(r['frac'],4), d['ms_per_step'], d['cpu_baseline']['value'])"
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/trace -o trace -- python3 bench.py --steps 5 --warmup 2 --no-cpu --no-compare > $O/bench_trace.log 2>&1 || { tail -20 $O/bench_trace.log; exit 1; }
python scripts/lease_c3.py $O > $O/prof_c3.md && rm -rf $O/trace && head -12 $O/prof_c3.md
for w in c1 c2 c4 c5 fd lat; do
  case $w in c1) SW="--steps 300 --warmup 100";; c2) SW="--steps 60 --warmup 20";; c4) SW="--steps 10 --warmup 3";; lat) SW="";; *) SW="--steps 3 --warmup 1";; esac
  timeout -k 10 500 python bench.py --workload $w $SW > $O/bench_$w.json 2> $O/bench_$w.err || { tail -20 $O/bench_$w.err; exit 1; }
  python -c "import json; d=json.load(open('$O/bench_$w.json')); r=d.get('roofline') or {}; print('$w', d['value'], r.get('frac'), (r.get('eval_only') or {}).get('frac'), (d.get('cpu_baseline') or {}).get('value'), (d.get('host_path') or {}).get('value'))"
done
timeout -k 10 500 python bench.py --prg mmo --steps 3 --warmup 1 > $O/bench_mmo.json 2> $O/bench_mmo.err || { tail -20 $O/bench_mmo.err; exit 1; }
python -c "import json; d=json.load(open('$O/bench_mmo.json')); r=d['roofline']; print('mmo', d['value'], r['frac'])"
