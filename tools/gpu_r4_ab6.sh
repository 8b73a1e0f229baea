#!/bin/bash
# A/B: contact passes of odd EPA-0 parts on their own stream (GJKEPA_PART_PASS_STREAMS) x parts, C2 (+ C4, C5 at 2 parts); 2 rounds.
set -o pipefail
OUT=gpurun_out/${1:-r4ab6}; mkdir -p $OUT; export TMPDIR=/tmp
run() { # tag env cfg round
  env $2 timeout -k 10 300 python bench.py --config $3 --no-cpu --no-f32-leg --no-warm-leg --steps 10 --warmup 2 > $OUT/$1.$3.r$4.json 2> $OUT/$1.$3.err || { tail -3 $OUT/$1.$3.err; return 1; }
  python3 -c "import json; d=json.load(open('$OUT/$1.$3.r$4.json')); print('$1 $3 round $4', d['value'], d['roofline']['kernel_ms'])"
}
for r in 1 2; do
  run p2pps1 "GJKEPA_EPA0_PARTS=2 GJKEPA_PART_PASS_STREAMS=1" C2 $r || exit 1
  run p2pps2 "GJKEPA_EPA0_PARTS=2 GJKEPA_PART_PASS_STREAMS=2" C2 $r || exit 1
  run p3pps2 "GJKEPA_EPA0_PARTS=3 GJKEPA_PART_PASS_STREAMS=2" C2 $r || exit 1
  run p4pps2 "GJKEPA_EPA0_PARTS=4 GJKEPA_PART_PASS_STREAMS=2" C2 $r || exit 1
  for c in C5 C4; do
    run p2pps1 "GJKEPA_PART_PASS_STREAMS=1" $c $r || exit 1
    run p2pps2 "GJKEPA_PART_PASS_STREAMS=2" $c $r || exit 1
  done
done
GJKEPA_PART_PASS_STREAMS=2 timeout -k 10 300 python bench.py --config C2 --no-f32-leg --no-warm-leg --steps 3 > $OUT/parity_c2.json 2>/dev/null && python3 -c "import json; print('parity C2 pps2', json.load(open('$OUT/parity_c2.json'))['parity_sample'])"
GJKEPA_PART_PASS_STREAMS=2 timeout -k 10 300 python -u -m pytest tests/test_graph.py -q --timeout 200 --timeout-method thread 2>&1 | tail -2
