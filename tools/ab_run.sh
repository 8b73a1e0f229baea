#!/bin/bash
# A/B session: every variant under build/variants (interleaved bench rounds + parity spot check),
# per-kernel times of each, phase stamps from build/diag/stamps, then the -m gpu suite on the main build.
set -o pipefail
export TMPDIR=/tmp
T=${1:-ab}
TAG=$T ROUNDS=${ROUNDS:-2} timeout -k 10 600 bash tools/variants.sh && \
TAG=${T}_prof timeout -k 10 400 bash tools/variant_prof.sh && \
if [ -f collision-detect-gjk-epa_amd/build/diag/stamps/libgjkepa_hip.so ]; then
  GJKEPA_LIB=collision-detect-gjk-epa_amd/build/diag/stamps/libgjkepa_hip.so timeout -k 10 200 python tools/stamps.py ${STAMPCFG:-C2} > gpurun_out/$T/stamps.txt 2>&1 && cat gpurun_out/$T/stamps.txt
fi && \
if [ -n "$TESTS" ]; then
  timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/$T/pytest_gpu.log 2>&1; rc=$?; tail -3 gpurun_out/$T/pytest_gpu.log; exit $rc
fi
