#!/bin/bash
# The bench lines of the shipped build with the committed PMC figures (profiles/pmc_traffic.json at the
# same source hash): C2 / C4 / C5, as the driver runs bench.py.  usage (via gpurun): bash tools/bench_lines.sh TAG
set -o pipefail
OUT=gpurun_out/${1:-lines}; mkdir -p $OUT; export TMPDIR=/tmp
for c in C2 C4 C5; do
  lc=$(echo $c | tr C c)
  timeout -k 10 400 python bench.py --config $c --steps 10 --warmup 3 > $OUT/bench_$lc.json 2> $OUT/bench_$lc.err || { tail -5 $OUT/bench_$lc.err; exit 1; }
  python3 -c "import json;d=json.load(open('$OUT/bench_$lc.json'));r=d['roofline'];print('$c',d['value'],d['ms_per_step'],r['traffic'],r['pmc_src'],d.get('parity_sample'))"
done
timeout -k 10 300 python bench.py > $OUT/bench_default.json 2> $OUT/bench_default.err && cat $OUT/bench_default.json
