#!/bin/bash
# Round-5 session g: contact tier 1 at 32 lanes x 8 (two pairs per wave) vs 64 x 4 on C4 / C5; the
# service's cost to a concurrent batch with each chain's own GPU span (is it the GPU or the host?).
# usage (via gpurun): bash tools/gpu_r5g.sh <tag>
set -o pipefail
TAG=${1:-r5g}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
echo "== ab $(date)" && bash tools/gpu_r5_ab.sh $TAG 2 "C4 C5" c1g32 || exit 1
echo "== service cost, chain spans $(date)"
timeout -k 10 300 python tools/svc_concurrent.py 4 16 > $OUT/svc_chain.json 2>> $OUT/svc.err || exit 1
tail -1 $OUT/svc_chain.json
echo "== done $(date)"
