set -o pipefail
mkdir -p gpurun_out/hull
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_hull.py -x -v -m gpu --timeout 120 --timeout-method thread > gpurun_out/hull/pytest.log 2>&1; rc=$?; tail -3 gpurun_out/hull/pytest.log; [ $rc -eq 0 ] || exit $rc
for c in H1 H2 H3; do timeout -k 10 300 python tools/bench_hull.py --config $c > gpurun_out/hull/bench_$c.json 2> gpurun_out/hull/bench_$c.err || exit 1; cat gpurun_out/hull/bench_$c.json; done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/hull/prof -o run --output-format csv -- python3 tools/bench_hull.py --config H1 --no-cpu > gpurun_out/hull/prof.json 2> gpurun_out/hull/prof.err || exit 1
echo done
