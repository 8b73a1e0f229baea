#!/bin/bash
# A/B: GJK tier 0 in the EPA-0 halves (GJKEPA_GJK_SPLIT), C2 / C5 / C4, 2 rounds; parity of the split path.
set -o pipefail
OUT=gpurun_out/${1:-r4ab7}; mkdir -p $OUT; export TMPDIR=/tmp
run() { # tag env cfg round
  env $2 timeout -k 10 300 python bench.py --config $3 --no-cpu --no-f32-leg --no-warm-leg --steps 10 --warmup 2 > $OUT/$1.$3.r$4.json 2> $OUT/$1.$3.err || { tail -3 $OUT/$1.$3.err; return 1; }
  python3 -c "import json; d=json.load(open('$OUT/$1.$3.r$4.json')); print('$1 $3 round $4', d['value'], d['roofline']['kernel_ms'])"
}
for r in 1 2; do
  for c in C2 C5 C4; do
    run split0 "GJKEPA_GJK_SPLIT=0" $c $r || exit 1
    run split1 "GJKEPA_GJK_SPLIT=1" $c $r || exit 1
  done
done
for c in C2 C5 C4; do
  GJKEPA_GJK_SPLIT=1 timeout -k 10 300 python bench.py --config $c --no-f32-leg --no-warm-leg --steps 3 > $OUT/parity_$c.json 2>/dev/null && python3 -c "import json; print('parity $c split', json.load(open('$OUT/parity_$c.json'))['parity_sample'])" || exit 1
done
GJKEPA_GJK_SPLIT=1 timeout -k 10 300 python -u -m pytest tests/test_graph.py tests/test_park.py tests/test_warm.py -q --timeout 200 --timeout-method thread 2>&1 | tail -2
