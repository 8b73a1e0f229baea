#!/bin/bash
# Copy a tools/gpu_round4.sh session (gpurun_out/TAG) into profiles/DEST and merge its PMC passes into
# profiles/pmc_traffic.json.  usage (CPU side): bash tools/collect_round4.sh TAG [DEST]
set -e
TAG=$1; DEST=profiles/${2:-r04}
S=gpurun_out/$TAG
mkdir -p $DEST
cp $S/pytest_gpu.log $DEST/pytest_gpu.log
cp $S/smoke.log $DEST/smoke.log
cp $S/fp32_check.log $DEST/fp32_check.log
for c in c2 c4 c5; do cp $S/bench_$c.json $DEST/bench_$c.json; done
for c in C2 C4 C5; do
  lc=$(echo $c | tr C c)
  cp $S/prof_$c/run_kernel_stats.csv $DEST/rocprof_${lc}_kernel_stats.csv
  python3 tools/trace_chain.py $S/prof_$c/run_kernel_trace.csv > $DEST/chain_$c.txt
done
cp $S/pmc.log $DEST/pmc_c2.log; cp $S/pmc_c5.log $DEST/pmc_c5.log
for t in 1 16 64 64p; do [ -f $S/callpattern/cp$t.txt ] && cp $S/callpattern/cp$t.txt $DEST/callpattern_$t.txt; done
cp $S/svc_concurrent.json $DEST/svc_concurrent.json
python3 tools/pmc_report.py $TAG f64_C2_1048576 1048576
python3 tools/pmc_report.py ${TAG}_c5 f64_C5_1048576 1048576
echo "collected $S -> $DEST"
