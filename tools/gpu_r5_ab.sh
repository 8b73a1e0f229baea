#!/bin/bash
# A/B of library variants (tools/build_variant.sh NAME flags -> build/variants/NAME) against the in-tree
# build, interleaved rounds; each line is a bench.py run of one config with GJKEPA_LIB pointing at the
# variant.  usage (via gpurun): bash tools/gpu_r5_ab.sh <tag> <rounds> "<configs>" <variant>...
set -o pipefail
TAG=$1; ROUNDS=$2; CFGS=$3; shift 3
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
D=collision-detect-gjk-epa_amd/build
for r in $(seq 1 $ROUNDS); do
  for v in main "$@"; do
    lib=$D/libgjkepa_hip.so
    [ "$v" != main ] && lib=$D/variants/$v/libgjkepa_hip.so
    for c in $CFGS; do
      GJKEPA_LIB=$lib timeout -k 10 240 python bench.py --config $c --legs none --no-cpu --no-f32-leg --no-warm-leg --launch-timing off \
        > $OUT/ab_${v}_${c}_$r.json 2>> $OUT/ab.err || { echo "FAIL $v $c"; tail -5 $OUT/ab.err; exit 1; }
      echo "$r $v $c $(python3 -c "import json;d=json.loads(open('$OUT/ab_${v}_${c}_$r.json').read().splitlines()[-1]);print(d['value'], d['ms_per_step'])")"
    done
  done
done
