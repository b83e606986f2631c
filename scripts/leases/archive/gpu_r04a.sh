# r04a: knob-free kernels: GPU suite (incl. RCCL at world 1), a C3 bench line over nccl, C4 kernel trace,
# and the C4 in-kernel timeline (entry / table-build / loop stamps of head and tail).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r04a; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -60 $O/pytest_gpu.log; exit 1; }
tail -3 $O/pytest_gpu.log
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 1 --force-dist --dist-backend nccl --steps 10 --warmup 3 --no-compare > $O/bench_c3_nccl.json 2> $O/bench_c3_nccl.err || { tail -30 $O/bench_c3_nccl.err; exit 1; }
python -c "import json; d=json.load(open('$O/bench_c3_nccl.json')); print('c3 nccl', d['value'], d['roofline']['frac'], d['key_broadcast'])"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace_c4 -o trace -- python3 bench.py --workload c4 --steps 5 --warmup 2 --no-cpu > $O/bench_c4_trace.json 2> $O/bench_c4_trace.err || { tail -30 $O/bench_c4_trace.err; exit 1; }
find $O/trace_c4 -name "*kernel_stats.csv" | head -1 | xargs cat | head -14
DCF_HIP_LIB=$PWD/dcf_amd/libdcf_hip_clk.so timeout -k 10 300 python scripts/c4_timeline.py > $O/c4_timeline.json 2> $O/c4_timeline.err || { tail -30 $O/c4_timeline.err; exit 1; }
cat $O/c4_timeline.json
