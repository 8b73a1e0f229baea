#!/bin/bash
# PMC passes (each counter group in its own rocprofv3 run, --pmc with --kernel-trace only).
set -o pipefail
TAG=${1:-r01}
shift
EXTRA="$@"
OUT=gpurun_out/$TAG/pmc
mkdir -p $OUT
export TMPDIR=/tmp
rocprofv3 -L > $OUT/counters_list.txt 2>&1 || true
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE" "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES" "SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_INSTS_VMEM_RD SQ_INSTS_SMEM" "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE GRBM_COUNT"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc $grp -d $OUT/p$i -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu --no-f32-leg --no-warm-leg --legs none --launch-timing off $EXTRA > $OUT/p$i.json 2> $OUT/p$i.err || { echo "pass $i ($grp) failed"; tail -5 $OUT/p$i.err; exit 1; }
  echo "pass $i ok: $grp"
done
