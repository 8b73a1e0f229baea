#!/bin/bash
# Copy one tools/gpu_session.sh session (gpurun_out/TAG) into profiles/DEST, every file named by the
# library source hash it ran (SRC, from its bench lines): the GPU suite log, bench lines, rocprofv3
# kernel statistics and chain timelines, and the PMC passes merged into profiles/pmc_traffic.json.
# usage (CPU side, after the gpurun call): bash tools/collect.sh TAG DEST
set -e
TAG=$1; DEST=profiles/${2:-r06}
S=gpurun_out/$TAG
mkdir -p $DEST
SRC=$(python3 -c "
import glob, json, sys
for p in sorted(glob.glob('$S/*.json')) + sorted(glob.glob('$S/pmc_*/p1.json')):
    for l in open(p):
        if l.startswith('{') and '\"lib\"' in l:
            print(json.loads(l)['lib'].rsplit('src ', 1)[-1].strip()); sys.exit()
")
echo "source hash: $SRC"
[ -f $S/pytest_gpu.log ] && cp $S/pytest_gpu.log $DEST/pytest_gpu_src$SRC.log
[ -f $S/bench_default.json ] && cp $S/bench_default.json $DEST/bench_src$SRC.json
for c in C2 C4 C5; do
  lc=$(echo $c | tr C c)
  [ -f $S/bench_$c.json ] && cp $S/bench_$c.json $DEST/bench_${c}_src$SRC.json
  if [ -f $S/prof_$c/run_kernel_stats.csv ]; then
    cp $S/prof_$c/run_kernel_stats.csv $DEST/rocprof_${lc}_kernel_stats_src$SRC.csv
    python3 tools/trace_chain.py $S/prof_$c/run_kernel_trace.csv > $DEST/chain_${c}_src$SRC.txt
  fi
  if [ -d $S/pmc_$c ]; then
    n=$(python3 -c "import sys; sys.path.insert(0, '.'); from bench import CONFIGS; print(CONFIGS['$c'][3])")
    python3 tools/pmc_report.py $S/pmc_$c f64_${c}_$n $n | tee $DEST/pmc_${lc}_src$SRC.log
  fi
done
for t in 1 16; do [ -f $S/callpattern_$t.txt ] && cp $S/callpattern_$t.txt $DEST/callpattern_${t}_src$SRC.txt; done
[ -f $S/c5_fp32_sweep.json ] && cp $S/c5_fp32_sweep.json $DEST/c5_fp32_sweep_src$SRC.json
[ -f $S/svc_concurrent.json ] && cp $S/svc_concurrent.json $DEST/svc_concurrent_src$SRC.json
[ -f $S/bench_2rank_gloo.json ] && cp $S/bench_2rank_gloo.json $DEST/bench_2rank_gloo_src$SRC.json
[ -f $S/svc_probe.txt ] && cp $S/svc_probe.txt $DEST/svc_probe_src$SRC.txt
echo "collected $S -> $DEST"
