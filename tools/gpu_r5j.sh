#!/bin/bash
# Kernel traces of C2 with EPA tier 0's second contact pass on its own stream (GJKEPA_PART_PASS_STREAMS=2)
# vs the default: where does the 13% go?  usage (via gpurun): bash tools/gpu_r5j.sh <tag>
set -o pipefail
TAG=${1:-r5j}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
for v in 1 2; do
  GJKEPA_PART_PASS_STREAMS=$v timeout -k 10 300 rocprofv3 --kernel-trace -d $OUT/pp$v -o run --output-format csv -- python3 bench.py --steps 5 --warmup 1 --no-cpu --no-f32-leg --no-warm-leg --legs none --launch-timing off > $OUT/pp$v.json 2> $OUT/pp$v.err || exit 1
done
echo "== done $(date)"
