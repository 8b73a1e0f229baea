#!/bin/bash
# A/B: EPA tier 2 in parts (GJKEPA_EPA2_PARTS) on C5 / C4 / C2, 2 interleaved rounds; parity + graph/park tests at 2 parts.
set -o pipefail
OUT=gpurun_out/${1:-r4ab5}; mkdir -p $OUT; export TMPDIR=/tmp
for r in 1 2; do
  for c in C5 C4 C2; do
    for p in 1 2 3; do
      GJKEPA_EPA2_PARTS=$p timeout -k 10 300 python bench.py --config $c --no-cpu --no-f32-leg --no-warm-leg --steps 8 --warmup 2 > $OUT/e2p$p.$c.r$r.json 2> $OUT/e2p$p.$c.err || { tail -3 $OUT/e2p$p.$c.err; exit 1; }
      python3 -c "import json; d=json.load(open('$OUT/e2p$p.$c.r$r.json')); print('e2 parts $p $c round $r', d['value'], d['roofline']['kernel_ms'])"
    done
  done
done
GJKEPA_EPA2_PARTS=2 timeout -k 10 300 python bench.py --config C5 --no-f32-leg --no-warm-leg --steps 3 > $OUT/parity_c5.json 2>/dev/null && python3 -c "import json; print('parity C5 e2p2', json.load(open('$OUT/parity_c5.json'))['parity_sample'])"
GJKEPA_EPA2_PARTS=2 timeout -k 10 300 python -u -m pytest tests/test_graph.py tests/test_park.py -q --timeout 200 --timeout-method thread 2>&1 | tail -2
