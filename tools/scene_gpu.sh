#!/bin/bash
# GPU-box session for the broad phase / collision step: bench + rocprofv3 kernel-trace summary.
set -o pipefail
mkdir -p gpurun_out/scene
export TMPDIR=/tmp
timeout -k 10 300 python tools/bench_scene.py > gpurun_out/scene/bench.json 2> gpurun_out/scene/bench.err || exit 1
cat gpurun_out/scene/bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/scene/prof -o run --output-format csv -- python3 tools/bench_scene.py --no-cpu > gpurun_out/scene/prof.json 2> gpurun_out/scene/prof.err || exit 1
python3 - <<'PY'
import csv
for r in csv.DictReader(open("gpurun_out/scene/prof/run_kernel_stats.csv")):
    print(f"  {r['Name'][:90]:90s} {r['Calls']:>4} {float(r['AverageNs'])/1e3:10.1f} us")
PY
