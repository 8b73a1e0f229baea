#!/bin/bash
# Round-5 session i: EPA tier 0's second part's contact pass on a stream of its own
# (GJKEPA_PART_PASS_STREAMS=2) at 4 / 8 / 16 hardware queues per process (GPU_MAX_HW_QUEUES), against
# the default, on C2 (and C4 / C5 for the queue count), two interleaved rounds.
# usage (via gpurun): bash tools/gpu_r5i.sh <tag>
set -o pipefail
TAG=${1:-r5i}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
run() {  # name, config, env...
  local name=$1 cfg=$2; shift 2
  env "$@" timeout -k 10 240 python bench.py --config $cfg --legs none --no-cpu --no-f32-leg --no-warm-leg --launch-timing off \
    > $OUT/ab_${name}_${cfg}_$r.json 2>> $OUT/ab.err || { echo "FAIL $name"; tail -5 $OUT/ab.err; exit 1; }
  echo "$r $name $cfg $(python3 -c "import json;d=json.loads(open('$OUT/ab_${name}_${cfg}_$r.json').read().splitlines()[-1]);print(d['value'], d['ms_per_step'])")"
}
for r in 1 2; do
  run hwq4 C2 GPU_MAX_HW_QUEUES=4
  run pp2_hwq4 C2 GPU_MAX_HW_QUEUES=4 GJKEPA_PART_PASS_STREAMS=2
  run hwq8 C2 GPU_MAX_HW_QUEUES=8
  run pp2_hwq8 C2 GPU_MAX_HW_QUEUES=8 GJKEPA_PART_PASS_STREAMS=2
  run pp2_hwq16 C2 GPU_MAX_HW_QUEUES=16 GJKEPA_PART_PASS_STREAMS=2
  run e23_hwq8 C4 GPU_MAX_HW_QUEUES=8 GJKEPA_E23_STREAMS=2
  run hwq8 C4 GPU_MAX_HW_QUEUES=8
done
echo "== done $(date)"
