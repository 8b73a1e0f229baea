#!/bin/bash
# Round-5 session d: GPU suite + smoke on the in-tree build, resident-service A/B (lean vs full one-wave
# path: lone-call latency, 16-thread calls, cost to a concurrent batch), the default bench line, rocprof
# kernel traces of C2 / C4 / C5.  usage (via gpurun): bash tools/gpu_r5d.sh <tag>
set -o pipefail
TAG=${1:-r5d}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
D=collision-detect-gjk-epa_amd/build
echo "== tests $(date)"
timeout -k 10 900 python -u -m pytest tests -v -m gpu --timeout 420 --timeout-method thread > $OUT/pytest_gpu.log 2>&1; rc=$?
tail -3 $OUT/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
echo "== smoke" && timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 && tail -1 $OUT/smoke.log || exit 1
echo "== service A/B $(date)"
for r in 1 2; do
  for v in main svcfull; do
    lib=$D/libgjkepa_hip.so; [ $v != main ] && lib=$D/variants/$v/libgjkepa_hip.so
    GJKEPA_LIB=$lib GJKEPA_QUERY_STATS=1 timeout -k 10 200 python tools/svc_lone.py 3000 > $OUT/svc_lone_${v}_$r.json 2> $OUT/svc_lone_${v}_$r.err || exit 1
    echo "$r $v lone $(tail -1 $OUT/svc_lone_${v}_$r.json) $(tail -1 $OUT/svc_lone_${v}_$r.err)"
    GJKEPA_LIB=$lib timeout -k 10 300 python tools/svc_concurrent.py 4 16 > $OUT/svc_conc_${v}_$r.json 2>> $OUT/svc.err || exit 1
    echo "$r $v concurrent $(tail -1 $OUT/svc_conc_${v}_$r.json)"
  done
done
echo "== ab EPA tier 0 at 8 lanes $(date)" && bash tools/gpu_r5_ab.sh $TAG 2 "C2" e0g8 e0g8w3 || exit 1
echo "== bench default $(date)"
timeout -k 10 500 python bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail -5 $OUT/bench.err; exit 1; }
python3 tools/r5_summary.py $OUT/bench.json
for c in C2 C4 C5; do
  echo "== rocprof $c $(date)"
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/prof_$c -o run --output-format csv -- python3 bench.py --config $c --steps 5 --warmup 1 --no-cpu --no-f32-leg --no-warm-leg --legs none > $OUT/prof_$c.json 2> $OUT/prof_$c.err || exit 1
done
echo "== done $(date)"
