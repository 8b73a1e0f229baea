#!/bin/bash
# Phase stamps of the diag build on the given configs.  usage (via gpurun): bash tools/stamps_run.sh TAG "C2 C5"
set -o pipefail
export TMPDIR=/tmp
T=${1:-st}; CFGS=${2:-C2}; OUT=gpurun_out/$T; mkdir -p $OUT
for c in $CFGS; do
  GJKEPA_LIB=collision-detect-gjk-epa_amd/build/diag/stamps/libgjkepa_hip.so timeout -k 10 200 python tools/stamps.py $c > $OUT/stamps_$c.txt 2>&1 || { tail -5 $OUT/stamps_$c.txt; exit 1; }
  cat $OUT/stamps_$c.txt
done
