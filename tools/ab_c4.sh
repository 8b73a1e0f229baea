#!/bin/bash
# A/B of the built variants on C4 (2 rounds) with the kernel trace of each.  usage: bash tools/ab_c4.sh TAG
set -o pipefail
export TMPDIR=/tmp
T=${1:-abc4}
TAG=$T ROUNDS=2 EXTRA="--config C4" timeout -k 10 900 bash tools/variants.sh || exit 1
for v in collision-detect-gjk-epa_amd/build/variants/*/; do
  n=$(basename $v)
  GJKEPA_LIB=$v/libgjkepa_hip.so timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/$T/tr_$n -o run --output-format csv -- python3 bench.py --config C4 --steps 2 --warmup 1 --no-cpu --no-f32-leg --no-warm-leg > /dev/null 2>&1 || { echo "trace $n failed"; exit 1; }
  python3 tools/trace_chain.py gpurun_out/$T/tr_$n/run_kernel_trace.csv 2 | tail -9 | sed "s/^/$n /"
done
