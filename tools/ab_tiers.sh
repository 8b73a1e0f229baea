set -o pipefail
export TMPDIR=/tmp
bash tools/ab_c4.sh abt6 || exit 1
TAG=abt6_c5 ROUNDS=2 EXTRA="--config C5" timeout -k 10 900 bash tools/variants.sh || exit 1
TAG=abt6_c2 ROUNDS=2 timeout -k 10 900 bash tools/variants.sh || exit 1
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/abt6/pytest_gpu.log 2>&1; rc=$?
tail -5 gpurun_out/abt6/pytest_gpu.log; exit $rc
