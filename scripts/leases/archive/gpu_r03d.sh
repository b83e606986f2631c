# Latency breakdown: in-kernel clock + duration of k_eval16_oct, and a kernel trace of the lat workload.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r03d; mkdir -p $O
DCF_HIP_LIB=$PWD/dcf_amd/libdcf_hip_clk.so timeout -k 10 200 python scripts/lat_probe.py > $O/lat_probe.json 2> $O/lat_probe.err || { tail -20 $O/lat_probe.err; exit 1; }
cat $O/lat_probe.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace -o trace -- python3 bench.py --workload lat > $O/lat_trace.log 2>&1 || { tail -20 $O/lat_trace.log; exit 1; }
tail -1 $O/lat_trace.log
python scripts/prof_summary.py $O | head -20
