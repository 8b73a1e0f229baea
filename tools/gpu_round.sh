#!/bin/bash
# One GPU-box session: parity tests, smoke, bench (C2 + C4 + C5), a 2-rank gloo rehearsal of the
# multi-rank bench path, the C5 fp64/fp32 sweep, a rocprofv3 kernel-trace summary of the default
# bench and the PMC passes for its traffic / VALU fields.
# Usage (from the repo root, via gpurun): bash tools/gpu_round.sh [tag] [skip-tests]
set -o pipefail
TAG=${1:-r01}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
if [ "$2" != "skip-tests" ]; then
  echo "== tests $(date)"
  timeout -k 10 900 python -m pytest tests -q -m gpu > $OUT/pytest_gpu.log 2>&1; rc=$?; tail -3 $OUT/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
  echo "== smoke" && timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 && cat $OUT/smoke.log || exit 1
fi
echo "== pmc" && timeout -k 10 900 bash tools/pmc.sh $TAG > $OUT/pmc.log 2>&1 && \
echo "== rocprof" && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python3 bench.py --steps 5 --warmup 1 --no-cpu --no-f32-leg > $OUT/prof_bench.json 2> $OUT/prof.err && \
echo "== c5 sweep" && timeout -k 10 600 python tools/c5_sweep.py 262144 $OUT/c5_fp32_sweep.json > $OUT/c5.log 2>&1 && \
echo "== bench C4" && timeout -k 10 600 python bench.py --config C4 > $OUT/bench_c4.json 2> $OUT/bench_c4.err && cat $OUT/bench_c4.json && \
echo "== bench C5" && timeout -k 10 600 python bench.py --config C5 > $OUT/bench_c5.json 2> $OUT/bench_c5.err && cat $OUT/bench_c5.json && \
echo "== 2-rank gloo rehearsal" && timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --backend gloo --steps 3 --warmup 1 --pairs-per-gpu 262144 > $OUT/bench_2rank_gloo.json 2> $OUT/bench_2rank_gloo.err && cat $OUT/bench_2rank_gloo.json && \
echo "== done"
