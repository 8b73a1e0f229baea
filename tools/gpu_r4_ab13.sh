#!/bin/bash
# A/B: share of EPA tier 0's first part (GJKEPA_EPA0_FIRST per mille; 500 = even halves), C2, 2 rounds;
# then C4 / C5 at the best candidates and a parity sample.
set -o pipefail
OUT=gpurun_out/${1:-r4ab13}; mkdir -p $OUT; export TMPDIR=/tmp
run() { # tag env cfg round
  env $2 timeout -k 10 300 python bench.py --config $3 --no-cpu --no-f32-leg --no-warm-leg --steps 10 --warmup 2 > $OUT/$1.$3.r$4.json 2> $OUT/$1.$3.err || { tail -3 $OUT/$1.$3.err; return 1; }
  python3 -c "import json; d=json.load(open('$OUT/$1.$3.r$4.json')); print('$1 $3 round $4', d['value'], d['roofline']['kernel_ms'])"
}
for r in 1 2 3; do
  for f in 500 650 700 750 800 300; do run f$f "GJKEPA_EPA0_FIRST=$f" C2 $r || exit 1; done
done
for r in 1 2; do for c in C4 C5; do for f in 500 700; do run f$f "GJKEPA_EPA0_FIRST=$f" $c $r || exit 1; done; done; done
GJKEPA_EPA0_FIRST=700 timeout -k 10 300 python bench.py --config C2 --no-f32-leg --no-warm-leg --steps 2 --cpu-sample 262144 > $OUT/parity_f700.json 2>/dev/null && python3 -c "import json; print('parity C2 f700', json.load(open('$OUT/parity_f700.json'))['parity_sample'])"
