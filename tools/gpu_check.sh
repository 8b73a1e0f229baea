#!/bin/bash
# Short GPU-box session: gpu parity tests, smoke, the default bench (C2) and its rocprofv3
# kernel-trace summary.  Usage (via gpurun, from the repo root): bash tools/gpu_check.sh [tag]
set -o pipefail
TAG=${1:-r01}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
echo "== tests $(date)"
timeout -k 10 600 python -u -m pytest tests -x -v -m gpu --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1; rc=$?
tail -3 $OUT/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
echo "== smoke" && timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 && cat $OUT/smoke.log && \
echo "== bench" && timeout -k 10 300 python bench.py > $OUT/bench_c2.json 2> $OUT/bench_c2.err && cat $OUT/bench_c2.json && \
echo "== rocprof" && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python3 bench.py --steps 5 --warmup 1 --no-cpu --no-f32-leg > $OUT/prof_bench.json 2> $OUT/prof.err && \
echo "== done $(date)"
