#!/bin/bash
# Per-kernel times (rocprofv3 kernel trace) of every built variant on the bench workload.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-vprof}
mkdir -p $OUT
for v in collision-detect-gjk-epa_amd/build/variants/*/; do
  n=$(basename $v)
  GJKEPA_LIB=$v/libgjkepa_hip.so timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/$n -o run --output-format csv -- python3 bench.py --steps 5 --warmup 1 --no-cpu --no-f32-leg ${BENCH_ARGS:-} > $OUT/$n.json 2> $OUT/$n.err || { echo "$n failed"; tail -3 $OUT/$n.err; exit 1; }
  python3 - $OUT/$n/run_kernel_stats.csv $n <<'PY'
import csv, sys
rows = [r for r in csv.DictReader(open(sys.argv[1])) if "gk::" in r["Name"]]
tot = sum(float(r["AverageNs"]) for r in rows) / 1e3
top = sorted(rows, key=lambda r: -float(r["AverageNs"]))[:4]
print(f"{sys.argv[2]:10s} total {tot:8.1f} us | " + " | ".join(f"{r['Name'].split('<')[0].replace('void gk::','')}<{r['Name'].split('<')[1].split(',')[2].strip()}> {float(r['AverageNs'])/1e3:.1f}" for r in top))
PY
done
