#!/bin/bash
# Round-5 session p: the in-tree build through the GPU suite, A/B against variants (build/variants/NAME),
# then the per-phase wave-time split (tools/stamps.py) of C2 and C5 from the stamps variant.
# usage (via gpurun): bash tools/gpu_r5p.sh <tag> <variant>...
set -o pipefail
TAG=$1; shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
D=collision-detect-gjk-epa_amd/build
echo "== tests $(date)"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
echo "== ab $(date)" && bash tools/gpu_r5_ab.sh $TAG 2 "C2 C4 C5" "$@" || exit 1
if [ -f $D/variants/stamps/libgjkepa_hip.so ]; then
  for c in C2 C5; do
    echo "== stamps $c $(date)"
    GJKEPA_LIB=$D/variants/stamps/libgjkepa_hip.so timeout -k 10 240 python -u tools/stamps.py $c > $OUT/stamps_$c.txt 2>&1 || { tail -5 $OUT/stamps_$c.txt; exit 1; }
    cat $OUT/stamps_$c.txt
  done
fi
echo "== done $(date)"
