#!/bin/bash
# Round-5 session f: variant A/Bs (contact fork after EPA tier 3; GJK tier 2 at two waves per SIMD) on
# C2 / C4 / C5, and what the resident service costs a concurrent batch at 4 / 8 / 16 hardware queues per
# process (is the cost the shared hardware queue?).  usage (via gpurun): bash tools/gpu_r5f.sh <tag>
set -o pipefail
TAG=${1:-r5f}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
echo "== ab $(date)" && bash tools/gpu_r5_ab.sh $TAG 2 "C2 C4 C5" fork3 g2w2 || exit 1
echo "== service vs hardware queues $(date)"
for q in 4 8 16; do
  GPU_MAX_HW_QUEUES=$q timeout -k 10 300 python tools/svc_concurrent.py 4 16 > $OUT/svc_hwq$q.json 2>> $OUT/svc.err || exit 1
  echo "hwq $q $(tail -1 $OUT/svc_hwq$q.json)"
done
echo "== done $(date)"
