#!/bin/bash
# Round-5 session c: GPU suite on the in-tree build (contact case_04 deferral, three GJK tiers), then the
# variant A/Bs (tools/gpu_r5_ab.sh).  usage (via gpurun): bash tools/gpu_r5c.sh <tag>
set -o pipefail
TAG=${1:-r5c}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
echo "== tests $(date)"
timeout -k 10 900 python -u -m pytest tests -v -m gpu --timeout 420 --timeout-method thread > $OUT/pytest_gpu.log 2>&1; rc=$?
tail -3 $OUT/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
echo "== ab C2 $(date)" && bash tools/gpu_r5_ab.sh $TAG 2 "C2" base d04 d04w4 || exit 1
echo "== ab C4 C5 $(date)" && bash tools/gpu_r5_ab.sh $TAG 2 "C4 C5" base g3 g3w2 || exit 1
echo "== done $(date)"
