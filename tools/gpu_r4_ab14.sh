#!/bin/bash
# A/B: EPA tier 0 in three parts on two streams (GJKEPA_EPA0_PARTS=3) vs the shipped two parts (65/35);
# C2, 3 rounds.
set -o pipefail
OUT=gpurun_out/${1:-r4ab14}; mkdir -p $OUT; export TMPDIR=/tmp
run() { # tag env cfg round
  env $2 timeout -k 10 300 python bench.py --config $3 --no-cpu --no-f32-leg --no-warm-leg --steps 10 --warmup 2 > $OUT/$1.$3.r$4.json 2> $OUT/$1.$3.err || { tail -3 $OUT/$1.$3.err; return 1; }
  python3 -c "import json; d=json.load(open('$OUT/$1.$3.r$4.json')); print('$1 $3 round $4', d['value'], d['roofline']['kernel_ms'])"
}
for r in 1 2 3; do
  run p2 "X=0" C2 $r || exit 1
  run p3 "GJKEPA_EPA0_PARTS=3" C2 $r || exit 1
  run p2f700 "GJKEPA_EPA0_FIRST=700" C2 $r || exit 1
done
