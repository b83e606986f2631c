# C5 HBM traffic per step (2 x FETCH_SIZE + WRITE_SIZE over gen, both parties' top trees,
# digests and evals; separate --pmc passes), recorded into profiles/pmc_traffic.json, then
# the C5 bench line with it.   bash scripts/leases/pmc_c5.sh <tag>
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/$1; mkdir -p $O
B="python bench.py --workload c5 --steps 2 --warmup 1 --no-cpu --no-compare"
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $O/pmc_fetch_c5 -o pmc -- $B > $O/pmc_fetch_c5.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $O/pmc_write_c5 -o pmc -- $B > $O/pmc_write_c5.log 2>&1 || exit 1
python scripts/prof_summary.py $O --traffic profiles/pmc_traffic.json "k_gen16+2*k_mk_prefix16+2*k_cw_keymajor+2*k_eval16_stream" C5 67108864 16 16 0 35416702976 --suffix _c5 > $O/traffic_c5.txt || exit 1
cp profiles/pmc_traffic.json $O/pmc_traffic.json
timeout -k 10 300 python bench.py --workload c5 --steps 3 --warmup 1 > $O/bench_c5.json 2> $O/bench_c5.err
