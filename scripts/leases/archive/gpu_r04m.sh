# r04m: the new multi-key parity cases (N = 17 / 32 multi-key stream, two-pass batched wide multi-key).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r04m; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread -k "multikey" > $O/pytest_multikey.log 2>&1 || { tail -60 $O/pytest_multikey.log; exit 1; }
grep -c PASSED $O/pytest_multikey.log; tail -1 $O/pytest_multikey.log
