# Round-end check: GPU tests, smoke, rocprof + PMC of the default bench, extra workloads.
# Usage (GPU box): bash scripts/leases/gpu_final.sh <tag>
set -o pipefail
TAG=${1:-final}
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
EXTRA="${EXTRA:-c1 c2 c4 c5 fd}" bash scripts/leases/gpu_profile.sh $TAG || exit 1
timeout -k 10 300 python bench.py --prg mmo --steps 3 --warmup 1 --no-cpu > $O/bench_mmo.log 2>&1 || exit 1
tail -1 $O/bench_mmo.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('mmo', round(d['value']/1e6,1), d['roofline']['frac'])"
