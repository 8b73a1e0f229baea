#!/bin/bash
# Service checks: query tests (both paths), concurrency cost, call pattern; then the route tallies and the variant A/B.
set -o pipefail
OUT=gpurun_out/${1:-r4svc}; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_query_service.py tests/test_query_combine.py tests/test_fortran_dropin.py -q -x --timeout 200 --timeout-method thread > $OUT/pytest_svc.log 2>&1; rc=$?
tail -3 $OUT/pytest_svc.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/svc_concurrent.py 1 4 16 > $OUT/svc_concurrent.json 2>&1 && cat $OUT/svc_concurrent.json || exit 1
timeout -k 10 700 bash tools/callpattern_probe.sh ${1:-r4svc}/callpattern 5000 100000 || exit 1
timeout -k 10 120 python tools/tally.py C2 C4 C5 > $OUT/tally.log 2>&1; cat $OUT/tally.log
