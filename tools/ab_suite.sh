#!/bin/bash
# A/B of the built variants on C2, then the full -m gpu suite on the main build.
# usage (via gpurun): bash tools/ab_suite.sh TAG [ROUNDS]
set -o pipefail
export TMPDIR=/tmp
T=${1:-abs}; R=${2:-2}; mkdir -p gpurun_out/$T
TAG=$T ROUNDS=$R timeout -k 10 900 bash tools/variants.sh || exit 1
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/$T/pytest_gpu.log 2>&1; rc=$?
tail -5 gpurun_out/$T/pytest_gpu.log; exit $rc
