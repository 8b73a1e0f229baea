#!/bin/bash
# A/B: hardware queues per process (GPU_MAX_HW_QUEUES 4 = HIP's default, 8, 16): the chain uses the
# caller's stream, the EPA-0 second stream and up to four contact-pass streams; C2 / C5 / C4, 2 rounds.
set -o pipefail
OUT=gpurun_out/${1:-r4ab8}; mkdir -p $OUT; export TMPDIR=/tmp
run() { # tag env cfg round
  env $2 timeout -k 10 300 python bench.py --config $3 --no-cpu --no-f32-leg --no-warm-leg --steps 10 --warmup 2 > $OUT/$1.$3.r$4.json 2> $OUT/$1.$3.err || { tail -3 $OUT/$1.$3.err; return 1; }
  python3 -c "import json; d=json.load(open('$OUT/$1.$3.r$4.json')); print('$1 $3 round $4', d['value'], d['roofline']['kernel_ms'])"
}
for r in 1 2; do
  for c in C2 C5 C4; do
    run q4 "GPU_MAX_HW_QUEUES=4" $c $r || exit 1
    run q8 "GPU_MAX_HW_QUEUES=8" $c $r || exit 1
    run q16 "GPU_MAX_HW_QUEUES=16" $c $r || exit 1
  done
  run q8pps2 "GPU_MAX_HW_QUEUES=8 GJKEPA_PART_PASS_STREAMS=2" C2 $r || exit 1
  run q8p4 "GPU_MAX_HW_QUEUES=8 GJKEPA_EPA0_PARTS=4" C2 $r || exit 1
done
