#!/bin/bash
# GPU tests (all), then the bench on C2, C4 and C5 (no CPU leg).
set -o pipefail
mkdir -p gpurun_out/q3
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 200 --timeout-method thread > gpurun_out/q3/pytest.log 2>&1; rc=$?
tail -3 gpurun_out/q3/pytest.log; [ $rc -eq 0 ] || exit $rc
for c in C2 C4 C5; do
  timeout -k 10 300 python bench.py --config $c --no-cpu --no-f32-leg > gpurun_out/q3/$c.json 2> gpurun_out/q3/$c.err || exit 1
  python3 -c "import json; d=json.load(open('gpurun_out/q3/$c.json')); print('$c', d['value'], 'Mq/s', d['ms_per_step'], 'ms', d.get('parity_sample'))"
done
