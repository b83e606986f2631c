# r05y: C2 shared-prefix depth sweep on the current tree (D = 21 .. 25, auto = 24), and C3
# (D = 25 .. 28, auto = 26), 2 alternating runs each.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05y; mkdir -p $O
for rep in 1 2; do
  for D in 21 22 23 24 25; do
    timeout -k 10 300 python bench.py --workload c2 --prefix $D --steps 60 --warmup 10 --no-cpu --no-compare > $O/c2_D${D}_$rep.json 2> $O/c2_D${D}_$rep.err || { tail -20 $O/c2_D${D}_$rep.err; exit 1; }
    python -c "import json; d=json.load(open('$O/c2_D${D}_$rep.json')); r=d['roofline']; print('c2', $D, $rep, round(d['ms_per_step'],4), round(r['frac'],4))" | tee -a $O/sweep.txt
  done
  for D in 25 26 27 28; do
    timeout -k 10 300 python bench.py --prefix $D --steps 6 --warmup 2 --no-cpu --no-compare > $O/c3_D${D}_$rep.json 2> $O/c3_D${D}_$rep.err || { tail -20 $O/c3_D${D}_$rep.err; exit 1; }
    python -c "import json; d=json.load(open('$O/c3_D${D}_$rep.json')); r=d['roofline']; print('c3', $D, $rep, round(d['ms_per_step'],3), round(r['frac'],4))" | tee -a $O/sweep.txt
  done
done
