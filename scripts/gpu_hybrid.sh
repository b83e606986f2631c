set -o pipefail
OUT=gpurun_out/${1:-hyb}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -m pytest tests -m gpu -x -q > $OUT/pytest_gpu.log 2>&1 || { tail -40 $OUT/pytest_gpu.log; exit 1; }
tail -2 $OUT/pytest_gpu.log
for cfg in "1 6" "2 6" "3 4" "3 5" "3 6" "3 7" "3 8" "3 9"; do
  set -- $cfg
  timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu --eval-mode $1 --hybrid-split $2 > $OUT/bench_$1_$2.log 2>&1 || { tail -20 $OUT/bench_$1_$2.log; exit 1; }
  python -c "import json;d=json.loads(open('$OUT/bench_$1_$2.log').read().splitlines()[-1]);print('mode $1 split $2', d['value'], d['roofline']['kernel_ms'])"
done
rocprofv3 -L > $OUT/counters.txt 2>&1 || true
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_WAIT_INST_ANY -d $OUT/pmc_bs -o pmc -- python bench.py --steps 1 --warmup 0 --no-cpu --eval-mode 2 --points 67108864 > $OUT/pmc_bs.log 2>&1 || echo pmc_bs failed
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_WAIT_INST_ANY -d $OUT/pmc_tt -o pmc -- python bench.py --steps 1 --warmup 0 --no-cpu --eval-mode 1 --points 67108864 > $OUT/pmc_tt.log 2>&1 || echo pmc_tt failed
