#!/bin/bash
# A/B of every built variant on C2, C4 and C5 (bench rounds + per-kernel times), then the -m gpu
# suite on the main build.  usage (via gpurun): bash tools/ab_cfgs.sh TAG ["C2 C4 C5"]
set -o pipefail
export TMPDIR=/tmp
T=${1:-abc}; CFGS=${2:-"C2 C4 C5"}
for c in $CFGS; do
  TAG=${T}_$c ROUNDS=${ROUNDS:-1} EXTRA="--config $c --no-warm-leg" timeout -k 10 600 bash tools/variants.sh || exit 1
  TAG=${T}_${c}_prof BENCH_ARGS="--config $c --no-warm-leg" timeout -k 10 600 bash tools/variant_prof.sh || exit 1
done
mkdir -p gpurun_out/$T
if [ -n "$TESTS" ]; then
  timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/$T/pytest_gpu.log 2>&1; rc=$?; tail -3 gpurun_out/$T/pytest_gpu.log; exit $rc
fi
