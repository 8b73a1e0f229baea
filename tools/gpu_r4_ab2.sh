#!/bin/bash
# A/B: EPA tier 0 parts (GJKEPA_EPA0_PARTS) x part streams (GJKEPA_EPA0_STREAMS) on C2; 2 interleaved rounds.
set -o pipefail
OUT=gpurun_out/${1:-r4ab2}; mkdir -p $OUT; export TMPDIR=/tmp
for r in 1 2; do
  for cfg in "1 1" "2 1" "2 2" "4 2" "6 2" "8 2"; do
    set -- $cfg
    GJKEPA_EPA0_PARTS=$1 GJKEPA_EPA0_STREAMS=$2 timeout -k 10 300 python bench.py --no-cpu --no-f32-leg --no-warm-leg --steps 10 --warmup 2 > $OUT/p$1s$2.r$r.json 2> $OUT/p$1s$2.err || { tail -3 $OUT/p$1s$2.err; exit 1; }
    python3 -c "import json; d=json.load(open('$OUT/p$1s$2.r$r.json')); print('parts $1 streams $2 round $r', d['value'], d['roofline']['kernel_ms'])"
  done
done
GJKEPA_EPA0_PARTS=4 GJKEPA_EPA0_STREAMS=2 timeout -k 10 300 python bench.py --no-f32-leg --no-warm-leg --steps 3 --cpu-sample 131072 > $OUT/parity.json 2>/dev/null && python3 -c "import json; print('parity p4s2', json.load(open('$OUT/parity.json'))['parity_sample'])"
