#!/bin/bash
# Generic A/B of built variants (tools/build_variant.sh NAME ...) against the product library:
# interleaved rounds of bench.py per config, then an oracle parity sample of every variant.
# usage (via gpurun): bash tools/ab_variants.sh TAG "C4 C5" "var1 var2" [rounds]
set -o pipefail
OUT=gpurun_out/$1; CFGS=$2; VARS=$3; R=${4:-2}
mkdir -p $OUT; export TMPDIR=/tmp
VD=collision-detect-gjk-epa_amd/build/variants
run() { # tag env cfg round
  env $2 timeout -k 10 300 python bench.py --config $3 --no-cpu --no-f32-leg --no-warm-leg --steps 10 --warmup 2 > $OUT/$1.$3.r$4.json 2> $OUT/$1.$3.err || { tail -3 $OUT/$1.$3.err; return 1; }
  python3 -c "import json; d=json.load(open('$OUT/$1.$3.r$4.json')); print('$1 $3 round $4', d['value'], d['roofline']['kernel_ms'])"
}
for r in $(seq 1 $R); do
  for c in $CFGS; do
    run prod "X=0" $c $r || exit 1
    for v in $VARS; do run $v "GJKEPA_LIB=$VD/$v/libgjkepa_hip.so" $c $r || exit 1; done
  done
done
for v in $VARS; do for c in $CFGS; do
  GJKEPA_LIB=$VD/$v/libgjkepa_hip.so timeout -k 10 300 python bench.py --config $c --no-f32-leg --no-warm-leg --steps 2 --cpu-sample 262144 > $OUT/parity_$v.$c.json 2>/dev/null && python3 -c "import json; print('parity $c $v', json.load(open('$OUT/parity_$v.$c.json'))['parity_sample'])" || exit 1
done; done
