#!/bin/bash
# Quick GPU check: gpu tests (stop at first failure), variant timings, C2 stamp breakdown.
set -o pipefail
mkdir -p gpurun_out/st
timeout -k 10 600 python -m pytest tests -q -m gpu -x > gpurun_out/pt.log 2>&1; rc=$?
tail -15 gpurun_out/pt.log
[ $rc -eq 0 ] || exit $rc
TAG=${TAG:-v} ROUNDS=${ROUNDS:-2} bash tools/variants.sh || exit 1
if [ -f collision-detect-gjk-epa_amd/build/diag/stamps/libgjkepa_hip.so ]; then
  for c in ${STAMP_CFGS:-C2}; do
    GJKEPA_LIB=collision-detect-gjk-epa_amd/build/diag/stamps/libgjkepa_hip.so timeout -k 10 200 python tools/stamps.py $c > gpurun_out/st/$c.txt 2>&1 || exit 1
    cat gpurun_out/st/$c.txt
  done
fi
# per-kernel times of the in-tree library on the default bench (rocprofv3 kernel trace)
export TMPDIR=/tmp
rm -rf gpurun_out/qprof
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/qprof -o run --output-format csv -- python3 bench.py --steps 5 --warmup 1 --no-cpu --no-f32-leg ${BENCH_ARGS:-} > gpurun_out/qprof.json 2> gpurun_out/qprof.err || exit 1
python3 - <<'PY'
import csv
for r in csv.DictReader(open("gpurun_out/qprof/run_kernel_stats.csv")):
    print(f"  {r['Name'][:70]:70s} {r['Calls']:>4} {float(r['AverageNs'])/1e3:10.1f} us")
PY
