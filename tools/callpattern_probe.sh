#!/bin/bash
# Single-call path breakdown (GPU box): the Fortran call-pattern benchmark at 1 and 16 threads with
# the query path's statistics (resident service: round trip and device time per call).
# usage (via gpurun): bash tools/callpattern_probe.sh TAG [n1] [n16]
set -o pipefail
export TMPDIR=/tmp
T=${1:-cp}; N1=${2:-5000}; N16=${3:-50000}
OUT=gpurun_out/$T; mkdir -p $OUT
B=tests/fortran/build/bench_callpattern
OMP_NUM_THREADS=1 GJKEPA_QUERY_STATS=1 timeout -k 10 200 $B $N1 > $OUT/cp1.txt 2>&1 && cat $OUT/cp1.txt && \
OMP_NUM_THREADS=16 GJKEPA_QUERY_STATS=1 timeout -k 10 200 $B $N16 > $OUT/cp16.txt 2>&1 && cat $OUT/cp16.txt && \
OMP_NUM_THREADS=64 GJKEPA_QUERY_STATS=1 timeout -k 10 200 $B $N16 > $OUT/cp64.txt 2>&1 && cat $OUT/cp64.txt
# the 64-thread run again with passive OpenMP waiting: after the parallel loop, 63 idle OpenMP threads
# no longer spin on the 16-CPU share while the master runs GJKEPA_BATCH (the suspected cause of its
# 3x slowdown in round 3)
OMP_NUM_THREADS=64 OMP_WAIT_POLICY=passive GJKEPA_QUERY_STATS=1 timeout -k 10 200 $B $N16 > $OUT/cp64p.txt 2>&1 && cat $OUT/cp64p.txt
