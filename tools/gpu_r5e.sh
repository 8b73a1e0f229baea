#!/bin/bash
# Round-5 measurement session at the shipped source: GPU suite + smoke, the default bench line, rocprofv3
# kernel traces of C2 / C4 / C5, and the PMC passes (tools/pmc.sh) of all three for the traffic figures.
# usage (via gpurun): bash tools/gpu_r5e.sh <tag> [skip-tests]
set -o pipefail
TAG=${1:-r5e}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
if [ "$2" != "skip-tests" ]; then
  echo "== tests $(date)"
  timeout -k 10 900 python -u -m pytest tests -v -m gpu --timeout 420 --timeout-method thread > $OUT/pytest_gpu.log 2>&1; rc=$?
  tail -3 $OUT/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
  echo "== smoke" && timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 && tail -1 $OUT/smoke.log || exit 1
fi
echo "== bench default $(date)"
timeout -k 10 500 python bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail -5 $OUT/bench.err; exit 1; }
python3 tools/r5_summary.py $OUT/bench.json
for c in C2 C4 C5; do
  echo "== rocprof $c $(date)"
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/prof_$c -o run --output-format csv -- python3 bench.py --config $c --steps 5 --warmup 1 --no-cpu --no-f32-leg --no-warm-leg --legs none --launch-timing off > $OUT/prof_$c.json 2> $OUT/prof_$c.err || exit 1
done
echo "== pmc C2 $(date)" && timeout -k 10 600 bash tools/pmc.sh ${TAG}_c2 > $OUT/pmc_c2.log 2>&1 && cat $OUT/pmc_c2.log || exit 1
echo "== pmc C4 $(date)" && timeout -k 10 900 bash tools/pmc.sh ${TAG}_c4 --config C4 > $OUT/pmc_c4.log 2>&1 && cat $OUT/pmc_c4.log || exit 1
echo "== pmc C5 $(date)" && timeout -k 10 600 bash tools/pmc.sh ${TAG}_c5 --config C5 > $OUT/pmc_c5.log 2>&1 && cat $OUT/pmc_c5.log || exit 1
echo "== done $(date)"
