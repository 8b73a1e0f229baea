#!/bin/bash
# Main build on the GPU box: the -m gpu suite, then the C2 / C4 / C5 bench lines (no CPU leg) and the
# call-pattern probe.  usage (via gpurun): bash tools/gpu_check2.sh TAG
set -o pipefail
export TMPDIR=/tmp
T=${1:-chk}; OUT=gpurun_out/$T; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1; rc=$?
tail -3 $OUT/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
for c in C2 C4 C5; do
  timeout -k 10 400 python bench.py --config $c --no-cpu --no-f32-leg --no-warm-leg > $OUT/bench_$c.json 2> $OUT/bench_$c.err || { tail -5 $OUT/bench_$c.err; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/bench_$c.json')); print('$c', d['value'], d['ms_per_step'], d['parity_sample'])"
done
bash tools/callpattern_probe.sh $T/cp 5000 100000
