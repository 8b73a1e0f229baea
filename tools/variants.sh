#!/bin/bash
# Time every built variant (collision-detect-gjk-epa_amd/build/variants/*) on the bench workload,
# interleaved rounds in one box session, plus a parity spot check of each against the oracle.
set -o pipefail
OUT=gpurun_out/${TAG:-var}
mkdir -p $OUT
ROUNDS=${ROUNDS:-2}
EXTRA=${EXTRA:-}
for r in $(seq 1 $ROUNDS); do
  for v in collision-detect-gjk-epa_amd/build/variants/*/; do
    n=$(basename $v)
    GJKEPA_LIB=$v/libgjkepa_hip.so timeout -k 10 300 python bench.py --no-cpu --no-f32-leg --steps 10 $EXTRA > $OUT/$n.r$r.json 2> $OUT/$n.err || { echo "$n failed"; tail -3 $OUT/$n.err; exit 1; }
    python3 -c "import json; d=json.load(open('$OUT/$n.r$r.json')); print('$n', 'round $r', d['value'], 'Mq/s', d['ms_per_step'], 'ms')"
  done
done
for v in collision-detect-gjk-epa_amd/build/variants/*/; do
  n=$(basename $v)
  GJKEPA_LIB=$v/libgjkepa_hip.so timeout -k 10 300 python tools/diag_parity.py > $OUT/$n.parity 2>&1 || { echo "$n parity run failed"; exit 1; }
  echo "$n parity: $(grep -c "'ok': True" $OUT/$n.parity) ok / $(grep -c "'ok'" $OUT/$n.parity)"
done
