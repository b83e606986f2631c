# r04n: HBM write bandwidth of 32 / 64-byte tiles with the siblings of a line on one XCD.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r04n; mkdir -p $O
timeout -k 10 120 ./scripts/micro/tile_xcd_bw > $O/tile_xcd_bw.log 2>&1 || { cat $O/tile_xcd_bw.log; exit 1; }
cat $O/tile_xcd_bw.log
