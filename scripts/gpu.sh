# One parameterised script for every GPU-box step (replaces the round 1-5 one-shot lease scripts).
# Run on the box through gpurun, e.g.
#   gpurun --timeout 1200 -- 'bash scripts/gpu.sh r06a suite && bash scripts/gpu.sh r06a bench c3 c4'
#   bash scripts/gpu.sh TAG SUB-COMMAND [args]    (TAG names the output directory gpurun_out/<TAG>)
# Sub-commands:
#   suite   [pytest args]           GPU suite (-m gpu, or the given tests) + smoke()
#   bench   W... [-- bench args]    bench lines of workloads W (c1 c2 c3 c4 c5 fd lat mmo; "all");
#                                   c3 runs as the driver runs it (--gpus 1 --steps 20 --warmup 5)
#   trace                           C3 bench line + a rocprofv3 kernel trace of the same workload in the
#                                   same lease, reduced by scripts/lease_c3.py to prof_c3.md
#   profile W [bench args]          kernel trace + FETCH_SIZE / WRITE_SIZE / SQ PMC passes (one pass
#                                   each, MI355X_MICROARCH.md) of one workload, reduced to prof_<W>.md;
#                                   TRAFFIC="<kernels> <W> <points> <N> <lambda> <prefix> <alg bytes>"
#                                   also writes pmc_traffic_<W>.json
#   ab      W REPS VARIANT... [-- bench args]  alternating same-box runs of library builds
#                                   (VARIANT "default" = dcf_amd/libdcf_hip.so, else
#                                   dcf_amd/libdcf_hip_<VARIANT>.so from scripts/build_variant.sh),
#                                   one summary line per run appended to ab.txt
#   abtest  VARIANT... [-- pytest args]  parity of each variant build on the GPU suite subset
#   pmc     W "COUNTERS" [bench args]    one extra PMC pass (mean per dispatch per kernel printed)
set -o pipefail
export TMPDIR=/tmp
TAG=$1; CMD=$2; shift 2
O=gpurun_out/$TAG
mkdir -p $O

libof() { if [ "$1" = default ]; then echo $PWD/dcf_amd/libdcf_hip.so; else echo $PWD/dcf_amd/libdcf_hip_$1.so; fi; }

steps_of() {  # default steps / warmup per workload (a few seconds of GPU time each)
  case $1 in
    c1) echo "--workload c1 --steps 300 --warmup 100";;
    c2) echo "--workload c2 --steps 60 --warmup 20";;
    c3) echo "--gpus 1 --steps 20 --warmup 5";;
    c4) echo "--workload c4 --steps 10 --warmup 3";;
    c5) echo "--workload c5 --steps 3 --warmup 1";;
    fd) echo "--workload fd --steps 3 --warmup 1";;
    lat) echo "--workload lat";;
    mmo) echo "--prg mmo --steps 3 --warmup 1";;
    *) echo "--workload $1";;
  esac
}

summary() {  # one line per bench JSON
  python - "$1" "$2" "$3" <<'EOF'
import json, sys
f, w, tag = sys.argv[1:4]
d = json.loads(open(f).read().strip().splitlines()[-1])
r = d.get("roofline") or {}
print(w, tag, "value=%.4g" % d["value"], "ms=%.4f" % d["ms_per_step"], "frac=%s" % (round(r["frac"], 4) if "frac" in r else None),
      "eval_only=%s" % (round(r["eval_only"]["frac"], 4) if "eval_only" in r else None),
      "cpu=%s" % ((d.get("cpu_baseline") or {}).get("value")), "phases=%s" % (d.get("phases") or d.get("phases_ms")))
EOF
}

case $CMD in
suite)
  ARGS=${*:-tests -m gpu}
  timeout -k 10 900 python -u -m pytest $ARGS -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 \
    || { tail -60 $O/pytest_gpu.log; exit 1; }
  tail -1 $O/pytest_gpu.log
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 \
    || { tail -20 $O/smoke.log; exit 1; }
  tail -1 $O/smoke.log
  ;;
bench)
  WS=(); while [ $# -gt 0 ] && [ "$1" != -- ]; do WS+=("$1"); shift; done; [ "$1" = -- ] && shift
  [ "${WS[0]}" = all ] && WS=(c3 c1 c2 c4 c5 fd lat mmo)
  for w in "${WS[@]}"; do
    timeout -k 10 600 python bench.py $(steps_of $w) "$@" > $O/bench_$w.json 2> $O/bench_$w.err \
      || { tail -20 $O/bench_$w.err; exit 1; }
    summary $O/bench_$w.json $w "" | tee -a $O/bench.txt
  done
  ;;
trace)
  timeout -k 10 600 python bench.py $(steps_of c3) > $O/bench_c3.json 2> $O/bench_c3.err || { tail -20 $O/bench_c3.err; exit 1; }
  summary $O/bench_c3.json c3 ""
  timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/trace -o trace -- python3 bench.py --steps 5 --warmup 2 --no-cpu \
    --no-compare > $O/bench_trace.log 2>&1 || { tail -20 $O/bench_trace.log; exit 1; }
  python scripts/lease_c3.py $O > $O/prof_c3.md && rm -rf $O/trace && head -12 $O/prof_c3.md
  ;;
profile)
  W=$1; shift
  B="bench.py $(steps_of $W | sed -e 's/--steps [0-9]*/--steps 2/' -e 's/--warmup [0-9]*/--warmup 1/') --no-cpu --no-compare $*"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace_$W -o trace -- python $B > $O/trace_$W.log 2>&1 \
    || { tail -5 $O/trace_$W.log; exit 1; }
  grep "^{\"metric" $O/trace_$W.log > $O/bench_prof_$W.json || true
  timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE -d $O/pmc_fetch_$W -o pmc -- python $B > $O/pmc_fetch_$W.log 2>&1 \
    || { tail -5 $O/pmc_fetch_$W.log; exit 1; }
  timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE -d $O/pmc_write_$W -o pmc -- python $B > $O/pmc_write_$W.log 2>&1 \
    || { tail -5 $O/pmc_write_$W.log; exit 1; }
  timeout -s KILL 240 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVE_CYCLES \
    SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_INSTS_SALU GRBM_GUI_ACTIVE -d $O/pmc_sq_$W -o pmc -- python $B \
    > $O/pmc_sq_$W.log 2>&1 || { tail -5 $O/pmc_sq_$W.log; exit 1; }
  python scripts/prof_summary.py $O --suffix _$W > $O/prof_$W.md || exit 1
  if [ -n "$TRAFFIC" ]; then
    python scripts/prof_summary.py $O --suffix _$W --traffic $O/pmc_traffic_$W.json $TRAFFIC > /dev/null || exit 1
  fi
  rm -rf $O/trace_$W $O/pmc_fetch_$W $O/pmc_write_$W $O/pmc_sq_$W
  echo "profiled $W"; head -20 $O/prof_$W.md
  ;;
pmc)  # one extra PMC pass of one workload: pmc W "COUNTERS" [bench args] (<= 8 SQ_, 4 TCC_, 2 TA_ ... per pass)
  W=$1; C=$2; shift 2
  B="bench.py $(steps_of $W | sed -e 's/--steps [0-9]*/--steps 2/' -e 's/--warmup [0-9]*/--warmup 1/') --no-cpu --no-compare $*"
  N=pmc_x_${W}_$(echo $C | md5sum | cut -c1-6)
  timeout -s KILL 240 rocprofv3 --pmc $C -d $O/$N -o pmc -- python $B > $O/$N.log 2>&1 || { tail -5 $O/$N.log; exit 1; }
  python - "$O/$N" <<'PY'
import glob, sqlite3, sys
from collections import defaultdict
sys.path.insert(0, "scripts")
from prof_summary import short
agg = defaultdict(lambda: defaultdict(list))
for db in glob.glob(sys.argv[1] + "/**/*.db", recursive=True):
    for k, c, v in sqlite3.connect(db).execute("select kernel_name, counter_name, value from counters_collection"):
        agg[short(k)][c].append(v)
for k, cs in agg.items():
    if k.startswith("k_"):
        print(k, " ".join(f"{c}={sum(v) / len(v):.4g}" for c, v in sorted(cs.items())))
PY
  rm -rf $O/$N
  ;;
ab)
  W=$1; REPS=$2; shift 2
  VS=(); while [ $# -gt 0 ] && [ "$1" != -- ]; do VS+=("$1"); shift; done; [ "$1" = -- ] && shift
  for rep in $(seq 1 $REPS); do
    for v in "${VS[@]}"; do
      DCF_HIP_LIB=$(libof $v) timeout -k 10 300 python bench.py $(steps_of $W) --no-cpu --no-compare "$@" \
        > $O/${W}_${v}_$rep.json 2> $O/${W}_${v}_$rep.err || { tail -20 $O/${W}_${v}_$rep.err; exit 1; }
      summary $O/${W}_${v}_$rep.json $W "$v/$rep" | tee -a $O/ab.txt
    done
  done
  ;;
abtest)
  VS=(); while [ $# -gt 0 ] && [ "$1" != -- ]; do VS+=("$1"); shift; done; [ "$1" = -- ] && shift
  for v in "${VS[@]}"; do
    DCF_HIP_LIB=$(libof $v) timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
      "$@" > $O/pytest_$v.log 2>&1 || { tail -60 $O/pytest_$v.log; exit 1; }
    echo "$v $(tail -1 $O/pytest_$v.log)"
  done
  ;;
*)
  echo "unknown sub-command $CMD"; exit 2;;
esac
