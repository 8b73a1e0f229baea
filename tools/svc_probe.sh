#!/bin/bash
# Resident query service latency probe (GPU box): product library with round-trip / device-time
# statistics, then the phase stamps of the serving wave.  usage (via gpurun): bash tools/svc_probe.sh TAG [n]
set -o pipefail
export TMPDIR=/tmp
T=${1:-svcp}; N=${2:-3000}; OUT=gpurun_out/$T; mkdir -p $OUT
GJKEPA_QUERY_STATS=1 timeout -k 10 200 python3 tools/svc_probe.py $N > $OUT/probe.txt 2>&1 && cat $OUT/probe.txt && \
GJKEPA_LIB=collision-detect-gjk-epa_amd/build/variants/stamps/libgjkepa_hip.so timeout -k 10 200 python3 tools/svc_probe.py $N > $OUT/stamps.txt 2>&1 && cat $OUT/stamps.txt
