#!/bin/bash
# GPU-box session after a change: the -m gpu suite, smoke(), one default C2 bench line and its
# rocprofv3 kernel trace (per-kernel stats + the timeline of one chain).
# usage (via gpurun, repo root): bash tools/gpu_check.sh TAG [pytest -k expression]
set -o pipefail
TAG=${1:-check}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
K=${2:+-k "$2"}
echo "== tests $(date)"
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread $K > $OUT/pytest_gpu.log 2>&1; rc=$?
tail -3 $OUT/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
echo "== smoke" && timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 && cat $OUT/smoke.log && \
echo "== bench $(date)" && timeout -k 10 400 python bench.py > $OUT/bench.json 2> $OUT/bench.err && cat $OUT/bench.json && \
echo "== rocprof $(date)" && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python3 bench.py --steps 5 --warmup 1 --no-cpu --no-f32-leg --no-warm-leg > $OUT/prof_bench.json 2> $OUT/prof.err && \
echo "== done $(date)"
