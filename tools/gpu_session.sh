#!/bin/bash
# One GPU-box session of named steps on the in-tree build (run from the repo root via gpurun):
#   bash tools/gpu_session.sh TAG step [step ...]
# Steps (each under its own time limit; the session stops at the first failure):
#   tests[=EXPR]   -m gpu suite (pytest -k EXPR when given)
#   smoke          __graft_entry__.smoke()
#   bench          the default bench.py line, as the driver runs it
#   lines          bench.py --config C2 / C4 / C5 lines (10 steps)
#   prof           rocprofv3 --kernel-trace --stats of C2 / C4 / C5 bench commands
#   pmc            PMC passes (one counter group per rocprofv3 run) for C2 / C4 / C5
#   ab=R:CFGS:V1,V2  A/B of library variants (tools/build_variant.sh) against the in-tree build,
#                  R interleaved rounds over configs CFGS (comma list), e.g. ab=2:C2,C5:e0x
#   envab=R:CFGS:VAR=v1,v2  A/B of a run-time environment knob of the in-tree build (e.g. GJKEPA_EPA0_FIRST)
#   callpattern    Fortran OpenMP loop of single GJKEPA calls vs GJKEPA_BATCH (1 / 16 threads)
#   stamps=CFGS    per-phase stamps from the diagnostic build (build/diag/stamps)
#   gloo2          two-rank bench rehearsal over gloo on the one GPU
#   hull           convex-hull module: its GPU tests, H1-H3 bench lines, rocprofv3 of H1
#   scene          broad phase + narrow phase scene bench and its rocprofv3 kernel statistics
#   svc            resident query service: concurrent-batch cost (tools/svc_concurrent.py)
#   c5sweep        config C5's fp64 / fp32 sweep with the >= 64-face subset (tools/c5_sweep.py)
#   svcprobe       lone-caller latency (tools/svc_probe.py) of the product build and, from the stamps
#                  build (build/diag/stamps), the serving wave's time per phase
# Results land in gpurun_out/TAG; tools/collect.sh copies them into profiles/.
set -o pipefail
TAG=$1; shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
D=collision-detect-gjk-epa_amd/build
BQ="--no-cpu --no-f32-leg --no-warm-leg"

step_tests() {
  local k=()
  [ -n "$1" ] && k=(-k "$1")
  timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread "${k[@]}" > $OUT/pytest_gpu.log 2>&1
  local rc=$?; tail -3 $OUT/pytest_gpu.log; return $rc
}
step_smoke() { timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 && cat $OUT/smoke.log; }
step_bench() { timeout -k 10 500 python bench.py > $OUT/bench_default.json 2> $OUT/bench_default.err && cat $OUT/bench_default.json; }
step_lines() {
  for c in C2 C4 C5; do
    timeout -k 10 400 python bench.py --config $c --steps 10 --warmup 3 --legs none > $OUT/bench_$c.json 2> $OUT/bench_$c.err || { tail -5 $OUT/bench_$c.err; return 1; }
    python3 -c "import json;d=json.load(open('$OUT/bench_$c.json'));print('$c',d['value'],d['ms_per_step'],d['roofline'].get('traffic'),d.get('parity_sample',{}).get('all_equal'))"
  done
}
step_prof() {
  for c in C2 C4 C5; do
    local s=5; [ $c != C2 ] && s=3
    timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/prof_$c -o run --output-format csv -- python3 bench.py --config $c --steps $s --warmup 1 --legs none $BQ > $OUT/prof_$c.json 2> $OUT/prof_$c.err || { echo "prof $c failed"; tail -5 $OUT/prof_$c.err; return 1; }
    echo "prof $c ok"
  done
}
step_pmc() {
  for c in C2 C4 C5; do
    mkdir -p $OUT/pmc_$c
    local i=0
    for grp in "FETCH_SIZE" "WRITE_SIZE" "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES" "SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_INSTS_VMEM_RD SQ_INSTS_SMEM" "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE GRBM_COUNT"; do
      i=$((i+1))
      timeout -s KILL 300 rocprofv3 --kernel-trace --pmc $grp -d $OUT/pmc_$c/p$i -o run --output-format csv -- python3 bench.py --config $c --steps 2 --warmup 1 $BQ --legs none --launch-timing off > $OUT/pmc_$c/p$i.json 2> $OUT/pmc_$c/p$i.err || { echo "pmc $c pass $i ($grp) failed"; tail -5 $OUT/pmc_$c/p$i.err; return 1; }
    done
    echo "pmc $c ok"
  done
}
step_ab() {
  local rounds=${1%%:*} rest=${1#*:}
  local cfgs=${rest%%:*} vars=${rest#*:}
  for r in $(seq 1 $rounds); do
    for v in main ${vars//,/ }; do
      local lib=$D/libgjkepa_hip.so
      [ "$v" != main ] && lib=$D/variants/$v/libgjkepa_hip.so
      for c in ${cfgs//,/ }; do
        GJKEPA_LIB=$lib timeout -k 10 240 python bench.py --config $c --legs none --cpu-sample 65536 --no-f32-leg --no-warm-leg --launch-timing off \
          > $OUT/ab_${v}_${c}_$r.json 2>> $OUT/ab.err || { echo "FAIL $v $c"; tail -5 $OUT/ab.err; return 1; }
        echo "$r $v $c $(python3 -c "import json;d=json.loads(open('$OUT/ab_${v}_${c}_$r.json').read().splitlines()[-1]);print(d['value'], d['ms_per_step'], d.get('parity_sample',{}).get('all_equal'))")"
      done
    done
  done
}
step_envab() {
  local rounds=${1%%:*} rest=${1#*:}
  local cfgs=${rest%%:*} kv=${rest#*:}
  local var=${kv%%=*} vals=${kv#*=}
  for r in $(seq 1 $rounds); do
    for v in ${vals//,/ }; do
      for c in ${cfgs//,/ }; do
        env $var=$v timeout -k 10 240 python bench.py --config $c --legs none --cpu-sample 65536 --no-f32-leg --no-warm-leg --launch-timing off \
          > $OUT/envab_${v}_${c}_$r.json 2>> $OUT/envab.err || { echo "FAIL $var=$v $c"; tail -5 $OUT/envab.err; return 1; }
        echo "$r $var=$v $c $(python3 -c "import json;d=json.loads(open('$OUT/envab_${v}_${c}_$r.json').read().splitlines()[-1]);print(d['value'], d['ms_per_step'], d.get('parity_sample',{}).get('all_equal'))")"
      done
    done
  done
}
step_callpattern() {
  for t in 1 16; do
    OMP_NUM_THREADS=$t GJKEPA_QUERY_STATS=1 timeout -k 10 300 tests/fortran/build/bench_callpattern $([ $t = 1 ] && echo 5000 || echo 100000) > $OUT/callpattern_$t.txt 2>&1 || { tail -5 $OUT/callpattern_$t.txt; return 1; }
    tail -4 $OUT/callpattern_$t.txt
  done
}
step_stamps() {
  for c in ${1//,/ }; do
    GJKEPA_LIB=$D/diag/stamps/libgjkepa_hip.so timeout -k 10 200 python tools/stamps.py $c > $OUT/stamps_$c.txt 2>&1 || { tail -5 $OUT/stamps_$c.txt; return 1; }
    cat $OUT/stamps_$c.txt
  done
}
step_gloo2() {
  timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --backend gloo --steps 3 --warmup 1 --pairs-per-gpu 262144 > $OUT/bench_2rank_gloo.json 2> $OUT/bench_2rank_gloo.err && cat $OUT/bench_2rank_gloo.json
}
step_hull() {
  timeout -k 10 300 python -u -m pytest tests/test_hull.py -x -v -m gpu --timeout 120 --timeout-method thread > $OUT/hull_pytest.log 2>&1 || { tail -5 $OUT/hull_pytest.log; return 1; }
  for c in H1 H2 H3; do timeout -k 10 300 python tools/bench_hull.py --config $c > $OUT/hull_$c.json 2> $OUT/hull_$c.err || return 1; cat $OUT/hull_$c.json; done
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_hull -o run --output-format csv -- python3 tools/bench_hull.py --config H1 --no-cpu > $OUT/prof_hull.json 2> $OUT/prof_hull.err
}
step_scene() {
  timeout -k 10 300 python tools/bench_scene.py > $OUT/scene.json 2> $OUT/scene.err && cat $OUT/scene.json && \
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_scene -o run --output-format csv -- python3 tools/bench_scene.py --no-cpu > $OUT/prof_scene.json 2> $OUT/prof_scene.err
}
step_c5sweep() { timeout -k 10 500 python tools/c5_sweep.py $((1 << 20)) $OUT/c5_fp32_sweep.json > $OUT/c5_sweep.log 2>&1 && tail -n 3 $OUT/c5_sweep.log; }
step_svcprobe() {
  GJKEPA_QUERY_STATS=1 timeout -k 10 300 python tools/svc_probe.py 3000 > $OUT/svc_probe.txt 2>&1 && cat $OUT/svc_probe.txt && \
  GJKEPA_LIB=$D/diag/stamps/libgjkepa_hip.so timeout -k 10 300 python tools/svc_probe.py 3000 > $OUT/svc_probe_stamps.txt 2>&1 && cat $OUT/svc_probe_stamps.txt
}
step_svc() { timeout -k 10 400 python tools/svc_concurrent.py > $OUT/svc_concurrent.json 2> $OUT/svc_concurrent.err && cat $OUT/svc_concurrent.json; }

for s in "$@"; do
  name=${s%%=*}; arg=""
  [ "$name" != "$s" ] && arg=${s#*=}
  echo "== $s $(date +%T)"
  step_$name "$arg" || { echo "== step $s failed"; exit 1; }
done
echo "== done $(date +%T)"
