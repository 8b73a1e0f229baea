#!/bin/bash
# Copy one measurement session's results (tools/gpu_round.sh + tools/gpu_round_large.sh, run under
# gpurun with tag TAG) from gpurun_out/TAG into profiles/DEST, and merge its PMC passes into
# profiles/pmc_traffic.json (keyed by precision/config/batch, stamped with the library source hash).
# usage (CPU side, after the gpurun call): bash tools/collect_round.sh TAG DEST
set -e
TAG=$1; DEST=profiles/${2:-r03}
S=gpurun_out/$TAG
mkdir -p $DEST
cp $S/pytest_gpu.log $DEST/pytest_gpu.log
for c in c2 c4 c5; do [ -f $S/bench_$c.json ] && cp $S/bench_$c.json $DEST/bench_$c.json; done
cp $S/prof/run_kernel_stats.csv $DEST/rocprof_c2_kernel_stats.csv
python3 tools/trace_chain.py $S/prof/run_kernel_trace.csv > $DEST/chain_C2.txt
for c in C4 C5; do
  lc=$(echo $c | tr C c)
  if [ -f $S/prof_$c/run_kernel_stats.csv ]; then
    cp $S/prof_$c/run_kernel_stats.csv $DEST/rocprof_${lc}_kernel_stats.csv
    python3 tools/trace_chain.py $S/prof_$c/run_kernel_trace.csv > $DEST/chain_$c.txt
  fi
done
[ -f $S/pmc.log ] && cp $S/pmc.log $DEST/pmc_c2.log
[ -f $S/pmc_c5.log ] && cp $S/pmc_c5.log $DEST/pmc_c5.log
for t in 1 16 64; do [ -f $S/callpattern/cp$t.txt ] && cp $S/callpattern/cp$t.txt $DEST/callpattern_${t}thread$([ $t -gt 1 ] && echo s).txt; done
python3 tools/pmc_report.py $TAG f64_C2_1048576 1048576
[ -d gpurun_out/${TAG}_c5/pmc ] && python3 tools/pmc_report.py ${TAG}_c5 f64_C5_1048576 1048576
echo "collected $S -> $DEST"
