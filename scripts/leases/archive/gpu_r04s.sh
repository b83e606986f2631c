# r04s: C4 wide-prefix build timeline (k_wpfx_build stamps, diagnostic library).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r04s; mkdir -p $O
DCF_HIP_LIB=$PWD/dcf_amd/libdcf_hip_clk.so timeout -k 10 300 python scripts/c4_build_timeline.py > $O/c4_build_timeline.json 2> $O/c4_build_timeline.err || { tail -20 $O/c4_build_timeline.err; exit 1; }
cat $O/c4_build_timeline.json
