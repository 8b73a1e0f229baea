#!/bin/bash
# Round-5 session m: the in-tree build (case_04 over LDS, collision type before the contact point) through
# the whole GPU suite, the fence variants' parity and A/B against it, then the EPA tail probe.
# usage (via gpurun): bash tools/gpu_r5m.sh <tag> <variant>...
set -o pipefail
TAG=$1; shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
echo "== tests $(date)"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
echo "== tail probe $(date)"
timeout -k 10 300 python -u tools/tail_probe.py $OUT/tail_probe.json > $OUT/tail_probe.log 2>&1 || { tail -30 $OUT/tail_probe.log; exit 1; }
cat $OUT/tail_probe.log
bash tools/gpu_r5k.sh $TAG "$@"
