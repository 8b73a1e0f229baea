#!/bin/bash
# One GPU-box session on the shipped build: parity tests + smoke, the default C2 bench line, its
# rocprofv3 kernel-trace summary, the PMC passes for its traffic / VALU fields, and the Fortran
# call-pattern benchmark (OpenMP loop of single GJKEPA calls vs one GJKEPA_BATCH).
# Usage (from the repo root, via gpurun): bash tools/gpu_round.sh <tag> [skip-tests]
set -o pipefail
TAG=${1:-r03}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
if [ "$2" != "skip-tests" ]; then
  echo "== tests $(date)"
  timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1; rc=$?
  tail -3 $OUT/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
  echo "== smoke" && timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 && cat $OUT/smoke.log || exit 1
fi
echo "== bench C2 $(date)" && timeout -k 10 400 python bench.py > $OUT/bench_c2.json 2> $OUT/bench_c2.err && cat $OUT/bench_c2.json && \
echo "== rocprof C2 $(date)" && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python3 bench.py --steps 5 --warmup 1 --no-cpu --no-f32-leg --no-warm-leg > $OUT/prof_bench.json 2> $OUT/prof.err && \
echo "== pmc $(date)" && timeout -k 10 600 bash tools/pmc.sh $TAG > $OUT/pmc.log 2>&1 && cat $OUT/pmc.log && \
echo "== call pattern $(date)" && bash tools/callpattern_probe.sh $TAG/callpattern 5000 100000 && \
echo "== done $(date)" || exit 1
if [ -n "$CFGS45" ]; then
  for c in C4 C5; do
    echo "== bench $c $(date)" && timeout -k 10 400 python bench.py --config $c > $OUT/bench_$(echo $c | tr C c).json 2> $OUT/bench_$c.err && cat $OUT/bench_$(echo $c | tr C c).json || exit 1
    timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/prof_$c -o run --output-format csv -- python3 bench.py --config $c --steps 3 --warmup 1 --no-cpu --no-f32-leg --no-warm-leg > $OUT/prof_$c.json 2> $OUT/prof_$c.err || exit 1
  done
fi
if [ -n "$PMC5" ]; then
  echo "== pmc C5 $(date)" && timeout -k 10 600 bash tools/pmc.sh ${TAG}_c5 --config C5 > $OUT/pmc_c5.log 2>&1 || exit 1
fi
if [ -n "$GLOO2" ]; then
  echo "== 2-rank gloo rehearsal $(date)" && timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --backend gloo --steps 3 --warmup 1 --pairs-per-gpu 262144 > $OUT/bench_2rank_gloo.json 2> $OUT/bench_2rank_gloo.err && cat $OUT/bench_2rank_gloo.json || exit 1
fi
