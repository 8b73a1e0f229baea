#!/bin/bash
# Round-4 A/B session: EPA tier 0 split into parts (GJKEPA_EPA0_PARTS, runtime) on C2, and the
# built variants (tools/build_variant.sh) on C2 / C5; interleaved rounds, one box session.
# usage (via gpurun): bash tools/gpu_r4_ab.sh <tag> [rounds]
set -o pipefail
TAG=${1:-r4ab}; R=${2:-2}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
one() {   # name, env, config
  local n=$1 env=$2 cfg=$3 r=$4
  env $env timeout -k 10 300 python bench.py --config $cfg --no-cpu --no-f32-leg --no-warm-leg --steps 10 --warmup 2 > $OUT/$n.$cfg.r$r.json 2> $OUT/$n.$cfg.err || { echo "$n $cfg failed"; tail -3 $OUT/$n.$cfg.err; return 1; }
  python3 -c "import json; d=json.load(open('$OUT/$n.$cfg.r$r.json')); print('$n $cfg round $r', d['value'], 'Mq/s', d['roofline']['kernel_ms'], 'ms')"
}
for r in $(seq 1 $R); do
  for p in 1 2 4 8; do one parts$p GJKEPA_EPA0_PARTS=$p C2 $r || exit 1; done
  for v in collision-detect-gjk-epa_amd/build/variants/*/; do
    n=$(basename $v)
    for c in C2 C5; do one var_$n GJKEPA_LIB=$v/libgjkepa_hip.so $c $r || exit 1; done
  done
done
for p in 1 4; do
  GJKEPA_EPA0_PARTS=$p timeout -k 10 300 python bench.py --config C2 --no-f32-leg --no-warm-leg --steps 3 --cpu-sample 131072 > $OUT/parity_parts$p.json 2>/dev/null || exit 1
  python3 -c "import json; d=json.load(open('$OUT/parity_parts$p.json')); print('parts$p parity', d['parity_sample'])"
done
