#!/bin/bash
# Per-kernel rocprofv3 stats for the given bench configs, plus phase stamps from the diag build.
# usage (via gpurun): bash tools/prof_cfgs.sh TAG "C4 C5"
set -o pipefail
TAG=${1:-pc}; CFGS=${2:-"C4 C5"}
OUT=gpurun_out/$TAG; mkdir -p $OUT
export TMPDIR=/tmp
for c in $CFGS; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_$c -o run --output-format csv -- python3 bench.py --config $c --steps 3 --warmup 1 --no-cpu --no-f32-leg > $OUT/prof_$c.json 2> $OUT/prof_$c.err || { echo "prof $c failed"; tail -5 $OUT/prof_$c.err; exit 1; }
  python3 - $OUT/prof_$c/run_kernel_stats.csv <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    print(f"  {r['Name'][:80]:80s} {r['Calls']:>4} {float(r['AverageNs'])/1e3:10.1f} us")
PY
  if [ -f collision-detect-gjk-epa_amd/build/diag/stamps/libgjkepa_hip.so ]; then
    GJKEPA_LIB=collision-detect-gjk-epa_amd/build/diag/stamps/libgjkepa_hip.so timeout -k 10 200 python tools/stamps.py $c > $OUT/stamps_$c.txt 2>&1 || { echo "stamps $c failed"; tail -5 $OUT/stamps_$c.txt; exit 1; }
    cat $OUT/stamps_$c.txt
  fi
done
