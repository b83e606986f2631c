# r04q: LAMBDA >= 32 at any N (multi-pass 4-bit tail for N >= 160, MMO t-vectors past 8 words):
# wide / MMO parity, then a C4 line (the default path's launch arguments changed).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r04q; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "wide or mmo" > $O/pytest_wide_mmo.log 2>&1 || { tail -60 $O/pytest_wide_mmo.log; exit 1; }
tail -1 $O/pytest_wide_mmo.log
timeout -k 10 300 python bench.py --workload c4 --steps 10 --warmup 3 --no-cpu --no-compare > $O/c4.json 2> $O/c4.err || { tail -20 $O/c4.err; exit 1; }
python -c "import json; d=json.load(open('$O/c4.json')); r=d['roofline']; print('c4', round(d['value']/1e6,2), round(d['ms_per_step'],3), round(r['frac'],4))"
