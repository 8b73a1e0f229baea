#!/bin/bash
# Per-kernel times of the narrow phase on configs C4 and C5 (rocprofv3 kernel trace).
set -o pipefail
export TMPDIR=/tmp
for c in C4 C5; do
  rm -rf gpurun_out/prof_$c
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$c -o run --output-format csv -- python3 bench.py --config $c --steps 3 --warmup 1 --no-cpu --no-f32-leg > gpurun_out/prof_$c.json 2> gpurun_out/prof_$c.err || exit 1
  python3 - $c <<'PY'
import csv, sys, json
c = sys.argv[1]
print(c, json.loads(open(f"gpurun_out/prof_{c}.json").read())["value"], "Mq/s")
for r in csv.DictReader(open(f"gpurun_out/prof_{c}/run_kernel_stats.csv")):
    if "gk::" in r["Name"]:
        print(f"  {r['Name'][:75]:75s} {float(r['AverageNs'])/1e3:10.1f} us")
PY
done
