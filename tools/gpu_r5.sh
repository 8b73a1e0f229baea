#!/bin/bash
# Round-5 session (one gpurun call, each GPU step under its own limit, chained so a failure ends it):
# GPU suite + smoke, default bench line (C2 + C4/C5 legs), launch-timing overhead A/B, EPA tiers 2/3
# side by side vs in sequence (C4 / C5), rocprofv3 kernel trace of the bench command, C5 fp32 sweep.
# usage (via gpurun): bash tools/gpu_r5.sh <tag> [skip-tests]
set -o pipefail
TAG=${1:-r05}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
if [ "$2" != "skip-tests" ]; then
  echo "== tests $(date)"
  timeout -k 10 900 python -u -m pytest tests -v -m gpu --timeout 420 --timeout-method thread > $OUT/pytest_gpu.log 2>&1; rc=$?
  tail -3 $OUT/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
  echo "== smoke" && timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 && cat $OUT/smoke.log || exit 1
fi
echo "== bench default $(date)"
timeout -k 10 500 python bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail -5 $OUT/bench.err; exit 1; }
python3 tools/r5_summary.py $OUT/bench.json
for i in 1 2; do
  for lt in off timed; do
    timeout -k 10 200 python bench.py --legs none --no-cpu --no-f32-leg --no-warm-leg --launch-timing $lt > $OUT/ab_lt_${lt}_$i.json 2>> $OUT/ab.err || exit 1
  done
  for e in 1 2; do
    GJKEPA_E23_STREAMS=$e timeout -k 10 300 python bench.py --config C4 --legs C5 --no-cpu --no-f32-leg --no-warm-leg --leg-sample 0 > $OUT/ab_e23_${e}_$i.json 2>> $OUT/ab.err || exit 1
  done
done
python3 tools/r5_summary.py --ab $OUT
echo "== rocprof C2 $(date)"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/prof_C2 -o run --output-format csv -- python3 bench.py --steps 5 --warmup 1 --no-cpu --no-f32-leg --no-warm-leg --legs none > $OUT/prof_C2.json 2> $OUT/prof_C2.err || exit 1
echo "== c5 sweep $(date)"
timeout -k 10 500 python tools/c5_sweep.py 1048576 $OUT/c5_fp32_sweep.json > $OUT/c5_sweep.log 2>&1 && tail -2 $OUT/c5_sweep.log || exit 1
echo "== done $(date)"
