#!/bin/bash
# A/B of the built variants (collision-detect-gjk-epa_amd/build/variants/*) on the reference's call
# pattern: the Fortran OpenMP loop of single GJKEPA calls at 1 and 16 threads, interleaved rounds.
# The Fortran driver's RUNPATH lets LD_LIBRARY_PATH pick the variant's libgjkepa_hip.so.
# usage (via gpurun): bash tools/ab_callpattern.sh TAG [ROUNDS] [n1] [n16]
set -o pipefail
export TMPDIR=/tmp
T=${1:-abcp}; R=${2:-2}; N1=${3:-3000}; N16=${4:-60000}
OUT=gpurun_out/$T; mkdir -p $OUT
B=tests/fortran/build/bench_callpattern
for r in $(seq 1 $R); do
  for v in collision-detect-gjk-epa_amd/build/variants/*/; do
    n=$(basename $v)
    for th in 1 16; do
      N=$N1; [ $th -gt 1 ] && N=$N16
      LD_LIBRARY_PATH=$v OMP_NUM_THREADS=$th GJKEPA_QUERY_STATS=1 timeout -k 10 200 $B $N > $OUT/$n.t$th.r$r.txt 2>&1 || { echo "$n t$th failed"; tail -3 $OUT/$n.t$th.r$r.txt; exit 1; }
      echo "$n round $r threads $th: $(grep OMP $OUT/$n.t$th.r$r.txt | awk '{print $(NF-1), $NF}') | $(grep 'service:' $OUT/$n.t$th.r$r.txt | sed 's/.*calls, //')"
    done
  done
done
