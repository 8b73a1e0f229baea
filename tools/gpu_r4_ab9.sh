#!/bin/bash
# A/B: support scans skip unused hull register slots in the large-hull tiers (variant built with
# -DGJKEPA_SLOT_SKIP=1, tools/build_variant.sh slot1) vs the product library; C4 / C5 / C2, 2 rounds;
# then full-batch parity of the variant on C4 / C5 and its GPU parity tests.
set -o pipefail
OUT=gpurun_out/${1:-r4ab9}; mkdir -p $OUT; export TMPDIR=/tmp
V=collision-detect-gjk-epa_amd/build/variants/slot1/libgjkepa_hip.so
run() { # tag env cfg round
  env $2 timeout -k 10 300 python bench.py --config $3 --no-cpu --no-f32-leg --no-warm-leg --steps 10 --warmup 2 > $OUT/$1.$3.r$4.json 2> $OUT/$1.$3.err || { tail -3 $OUT/$1.$3.err; return 1; }
  python3 -c "import json; d=json.load(open('$OUT/$1.$3.r$4.json')); print('$1 $3 round $4', d['value'], d['roofline']['kernel_ms'])"
}
for r in 1 2; do
  for c in C4 C5 C2; do
    run prod "X=0" $c $r || exit 1
    run slot1 "GJKEPA_LIB=$V" $c $r || exit 1
  done
done
for c in C4 C5; do
  GJKEPA_LIB=$V timeout -k 10 300 python bench.py --config $c --no-f32-leg --no-warm-leg --steps 3 > $OUT/parity_$c.json 2>/dev/null && python3 -c "import json; print('parity $c slot1', json.load(open('$OUT/parity_$c.json'))['parity_sample'])" || exit 1
done
GJKEPA_LIB=$V timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_park.py -x -q --timeout 200 --timeout-method thread > $OUT/pytest_slot1.log 2>&1; tail -3 $OUT/pytest_slot1.log
