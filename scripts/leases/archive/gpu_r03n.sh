# r03n: reproduce the 2-rank gloo bench abort (test_bench_dist) with full stderr, default lib then chain2 (stop at the first failure)
set -o pipefail
O=gpurun_out/r03n; mkdir -p $O
for v in "" chain2; do
  L=$PWD/dcf_amd/libdcf_hip.so; [ -n "$v" ] && L=$PWD/dcf_amd/libdcf_hip_$v.so
  DCF_HIP_LIB=$L OMP_NUM_THREADS=4 timeout -k 10 240 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29561 bench.py --gpus 2 --steps 2 --warmup 1 --points 4194307 --no-cpu --no-compare --dist-backend gloo --check > $O/dist_$v.out 2> $O/dist_$v.err || { echo "lib ${v:-default} FAILED"; tail -c 2000 $O/dist_$v.err; exit 1; }
  echo "lib ${v:-default} ok"
  tail -c 200 $O/dist_$v.out
done
