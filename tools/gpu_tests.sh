#!/bin/bash
# GPU-box session: the -m gpu parity tests, smoke(), and one default bench line.
# Usage (repo root, via gpurun): bash tools/gpu_tests.sh <tag> [pytest -k expression]
set -o pipefail
TAG=${1:-scratch}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
K=${2:+-k "$2"}
echo "== tests $(date)"
timeout -k 10 1000 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread $K > $OUT/pytest_gpu.log 2>&1; rc=$?
tail -3 $OUT/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
echo "== smoke" && timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 && cat $OUT/smoke.log && \
echo "== bench" && timeout -k 10 300 python bench.py > $OUT/bench.json 2> $OUT/bench.err && cat $OUT/bench.json
