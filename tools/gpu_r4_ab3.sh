#!/bin/bash
# A/B: product build vs the variants in build/variants (C2, C4, C5), 2 interleaved rounds, + parity of the product.
set -o pipefail
OUT=gpurun_out/${1:-r4ab3}; mkdir -p $OUT; export TMPDIR=/tmp
one() { # name lib cfg round
  env ${2:+GJKEPA_LIB=$2} timeout -k 10 300 python bench.py --config $3 --no-cpu --no-f32-leg --no-warm-leg --steps 8 --warmup 2 > $OUT/$1.$3.r$4.json 2> $OUT/$1.$3.err || { tail -3 $OUT/$1.$3.err; return 1; }
  python3 -c "import json; d=json.load(open('$OUT/$1.$3.r$4.json')); print('$1 $3 round $4', d['value'], d['roofline']['kernel_ms'])"
}
for r in 1 2; do
  for c in C4 C2 C5; do
    one product "" $c $r || exit 1
    for v in collision-detect-gjk-epa_amd/build/variants/*/; do one $(basename $v) $v/libgjkepa_hip.so $c $r || exit 1; done
  done
done
timeout -k 10 300 python bench.py --config C4 --no-f32-leg --no-warm-leg --steps 3 --cpu-sample 262144 > $OUT/parity_c4.json 2>/dev/null && python3 -c "import json; print('parity C4', json.load(open('$OUT/parity_c4.json'))['parity_sample'])"
timeout -k 10 300 python -u -m pytest tests/test_graph.py tests/test_park.py -q --timeout 200 --timeout-method thread 2>&1 | tail -2
