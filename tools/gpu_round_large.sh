#!/bin/bash
# Large-hull half of a measurement session (GPU box): C4 and C5 bench lines with their rocprofv3
# kernel-trace summaries, then the C5 PMC passes.  The C2 half is tools/gpu_round.sh.
# Usage (repo root, via gpurun): bash tools/gpu_round_large.sh <tag> [skip-pmc]
set -o pipefail
TAG=${1:-r03}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
for c in C4 C5; do
  lc=$(echo $c | tr C c)
  echo "== bench $c $(date)" && timeout -k 10 400 python bench.py --config $c > $OUT/bench_$lc.json 2> $OUT/bench_$c.err && cat $OUT/bench_$lc.json || exit 1
  echo "== rocprof $c $(date)" && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/prof_$c -o run --output-format csv -- python3 bench.py --config $c --steps 3 --warmup 1 --no-cpu --no-f32-leg --no-warm-leg > $OUT/prof_$c.json 2> $OUT/prof_$c.err || exit 1
done
if [ "$2" != "skip-pmc" ]; then
  echo "== pmc C5 $(date)" && timeout -k 10 600 bash tools/pmc.sh ${TAG}_c5 --config C5 > $OUT/pmc_c5.log 2>&1 && cat $OUT/pmc_c5.log || exit 1
fi
echo "== done $(date)"
