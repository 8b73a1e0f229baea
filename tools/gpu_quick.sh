#!/bin/bash
# GPU-box check after a host-side change: the -m gpu suite, then the Fortran call-pattern benchmark.
# usage (via gpurun): bash tools/gpu_quick.sh TAG [pytest -k expression]
set -o pipefail
export TMPDIR=/tmp
T=${1:-quick}; mkdir -p gpurun_out/$T
K=${2:+-k "$2"}
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread $K > gpurun_out/$T/pytest_gpu.log 2>&1; rc=$?
tail -3 gpurun_out/$T/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
OMP_NUM_THREADS=16 timeout -k 10 300 tests/fortran/build/bench_callpattern 100000 > gpurun_out/$T/callpattern.txt 2>&1 && cat gpurun_out/$T/callpattern.txt
