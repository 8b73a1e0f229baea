#!/bin/bash
# One GPU-box session: parity tests, smoke, bench, rocprofv3 kernel-trace summary.
# Usage (from the repo root, via gpurun): bash tools/gpu_round.sh [tag]
set -o pipefail
TAG=${1:-r01}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
echo "== tests $(date)" && \
timeout -k 10 900 python -m pytest tests -q -m gpu > $OUT/pytest_gpu.log 2>&1; rc=$?; tail -3 $OUT/pytest_gpu.log; [ $rc -eq 0 ] && \
echo "== smoke" && timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 && cat $OUT/smoke.log && \
echo "== bench" && timeout -k 10 600 python bench.py > $OUT/bench.json 2> $OUT/bench.err && cat $OUT/bench.json && \
echo "== rocprof" && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python3 bench.py --steps 5 --warmup 1 --no-cpu --no-f32-leg > $OUT/prof_bench.json 2> $OUT/prof.err && \
echo "== done"
