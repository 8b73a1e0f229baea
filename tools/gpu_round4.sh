#!/bin/bash
# Round-4 measurement session on the shipped build (one gpurun call, each step under its own limit):
# GPU suite + smoke, fp32 full-batch check, bench C2 / C4 / C5, rocprofv3 kernel traces of the same
# commands, PMC passes (C2, C5), the Fortran call pattern, the service-concurrency probe.
# usage (via gpurun): bash tools/gpu_round4.sh <tag> [skip-tests]
set -o pipefail
TAG=${1:-r04}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
if [ "$2" != "skip-tests" ]; then
  echo "== tests $(date)"
  timeout -k 10 700 python -u -m pytest tests -v -m gpu --timeout 200 --timeout-method thread > $OUT/pytest_gpu.log 2>&1; rc=$?
  tail -3 $OUT/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
  echo "== smoke" && timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 && cat $OUT/smoke.log || exit 1
fi
echo "== fp32 check $(date)" && timeout -k 10 400 python -u tools/fp32_check.py C2 C5 C4 > $OUT/fp32_check.log 2>&1 || exit 1
for c in C2 C4 C5; do
  lc=$(echo $c | tr C c)
  echo "== bench $c $(date)"
  timeout -k 10 400 python bench.py --config $c --steps 10 --warmup 3 > $OUT/bench_$lc.json 2> $OUT/bench_$lc.err || { tail -5 $OUT/bench_$lc.err; exit 1; }
  python3 -c "import json;d=json.load(open('$OUT/bench_$lc.json'));print('$c',d['value'],d['ms_per_step'],d.get('parity_sample'))"
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/prof_$c -o run --output-format csv -- python3 bench.py --config $c --steps 5 --warmup 1 --no-cpu --no-f32-leg --no-warm-leg > $OUT/prof_$c.json 2> $OUT/prof_$c.err || exit 1
done
echo "== pmc C2 $(date)" && timeout -k 10 600 bash tools/pmc.sh $TAG > $OUT/pmc.log 2>&1 && cat $OUT/pmc.log || exit 1
echo "== pmc C5 $(date)" && timeout -k 10 600 bash tools/pmc.sh ${TAG}_c5 --config C5 > $OUT/pmc_c5.log 2>&1 && cat $OUT/pmc_c5.log || exit 1
echo "== call pattern $(date)" && timeout -k 10 700 bash tools/callpattern_probe.sh $TAG/callpattern 5000 100000 || exit 1
echo "== service concurrency $(date)" && timeout -k 10 300 python tools/svc_concurrent.py 1 4 16 > $OUT/svc_concurrent.json 2>&1 && cat $OUT/svc_concurrent.json || exit 1
echo "== done $(date)"
