# Effective engine clock per kernel: GRBM_GUI_ACTIVE (summed over the 8 XCDs) / kernel time,
# both from one rocprofv3 run (--kernel-trace with one GRBM counter).
#   bash scripts/leases/pmc_clock.sh <tag> [workload:steps ...]   -> gpurun_out/<tag>/clock.md
set -o pipefail
export TMPDIR=/tmp
T=$1; shift
O=gpurun_out/$T; mkdir -p $O
[ $# -eq 0 ] && set -- c3:1 c4:5 c2:30
for ws in "$@"; do
  w=${ws%%:*}; s=${ws##*:}
  timeout -s KILL 300 rocprofv3 --kernel-trace --pmc GRBM_GUI_ACTIVE -d $O/clk_$w -o clk -- python bench.py --workload $w --steps $s --warmup 2 --no-cpu --no-compare > $O/clk_$w.log 2>&1 || exit 1
done
python scripts/clock_summary.py $O > $O/clock.md
