#!/bin/bash
# A/B: slot skipping per scan (variants: slotG = -DGJKEPA_SLOT_SKIP=5, GJK fp32 screen + sphere radii;
# slotD = -DGJKEPA_SLOT_SKIP=2, support dots) vs the product library; C4 / C5, 2 rounds; parity of each.
set -o pipefail
OUT=gpurun_out/${1:-r4ab10}; mkdir -p $OUT; export TMPDIR=/tmp
VD=collision-detect-gjk-epa_amd/build/variants
run() { # tag env cfg round
  env $2 timeout -k 10 300 python bench.py --config $3 --no-cpu --no-f32-leg --no-warm-leg --steps 10 --warmup 2 > $OUT/$1.$3.r$4.json 2> $OUT/$1.$3.err || { tail -3 $OUT/$1.$3.err; return 1; }
  python3 -c "import json; d=json.load(open('$OUT/$1.$3.r$4.json')); print('$1 $3 round $4', d['value'], d['roofline']['kernel_ms'])"
}
for r in 1 2; do
  for c in C4 C5; do
    run prod "X=0" $c $r || exit 1
    run slotG "GJKEPA_LIB=$VD/slotG/libgjkepa_hip.so" $c $r || exit 1
    run slotD "GJKEPA_LIB=$VD/slotD/libgjkepa_hip.so" $c $r || exit 1
  done
done
for v in slotG slotD; do for c in C4 C5; do
  GJKEPA_LIB=$VD/$v/libgjkepa_hip.so timeout -k 10 300 python bench.py --config $c --no-f32-leg --no-warm-leg --steps 2 --cpu-sample 262144 > $OUT/parity_$v.$c.json 2>/dev/null && python3 -c "import json; print('parity $c $v', json.load(open('$OUT/parity_$v.$c.json'))['parity_sample'])" || exit 1
done; done
