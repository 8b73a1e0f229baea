#!/bin/bash
# Round-4 GPU session: fp32 full-batch check, the GPU suite, bench C2 / C4 / C5 (each its own time limit).
# usage (via gpurun): bash tools/gpu_r4.sh <tag> [skip-tests]
set -o pipefail
TAG=${1:-r4}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
echo "== fp32 check $(date)"
timeout -k 10 400 python -u tools/fp32_check.py C2 C5 C4 > $OUT/fp32_check.log 2>&1; rc=$?
cut -c1-1200 $OUT/fp32_check.log; [ $rc -eq 0 ] || exit $rc
if [ "$2" != "skip-tests" ]; then
  echo "== tests $(date)"
  timeout -k 10 700 python -u -m pytest tests -q -m gpu --timeout 200 --timeout-method thread -x > $OUT/pytest.log 2>&1; rc=$?
  tail -15 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
fi
for c in C2 C4 C5; do
  echo "== bench $c $(date)"
  timeout -k 10 400 python bench.py --config $c --steps 5 --warmup 2 > $OUT/bench_$c.json 2> $OUT/bench_$c.err || { tail -5 $OUT/bench_$c.err; exit 1; }
  python -c "import json;d=json.load(open('$OUT/bench_$c.json'));print('$c',d['value'],d['ms_per_step'],d.get('parity_sample'),{k:d.get('fp32_compute',{}).get(k) for k in ('value','gate_passed','depth_relerr_max','normal_angle_rad_max_nontie','normal_ties')})"
done
echo "== done $(date)"
