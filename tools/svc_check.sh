set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/svc1
timeout -k 10 300 python -u -m pytest tests/test_query_service.py tests/test_query_combine.py -x -v --timeout 120 --timeout-method thread > gpurun_out/svc1/pytest.log 2>&1; rc=$?
tail -15 gpurun_out/svc1/pytest.log; [ $rc -eq 0 ] || exit $rc
bash tools/callpattern_probe.sh svc1
