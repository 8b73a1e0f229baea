#!/bin/bash
# Round-5 session ae: the single-pair call path at the shipped source: lone and 16-thread gjkepa_query
# latency (tools/svc_lone.py) and what the resident service costs a concurrent C2 batch
# (tools/svc_concurrent.py), two rounds each.  usage (via gpurun): bash tools/gpu_r5ae.sh <tag>
set -o pipefail
TAG=${1:-r5ae}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
for r in 1 2; do
  echo "== lone $r $(date)"
  GJKEPA_QUERY_STATS=1 timeout -k 10 200 python tools/svc_lone.py 3000 > $OUT/svc_lone_$r.json 2> $OUT/svc_lone_$r.err || { tail -5 $OUT/svc_lone_$r.err; exit 1; }
  tail -1 $OUT/svc_lone_$r.json
  echo "== concurrent $r $(date)"
  timeout -k 10 300 python tools/svc_concurrent.py 1 4 16 > $OUT/svc_conc_$r.json 2> $OUT/svc_conc_$r.err || { tail -5 $OUT/svc_conc_$r.err; exit 1; }
  tail -1 $OUT/svc_conc_$r.json
done
echo "== done $(date)"
