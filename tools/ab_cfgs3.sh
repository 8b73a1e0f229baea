#!/bin/bash
# A/B of the built variants on C2, C5 and C4 (2 interleaved rounds each).  usage: bash tools/ab_cfgs3.sh TAG
set -o pipefail
export TMPDIR=/tmp
T=${1:-ab3}
TAG=${T}_c2 ROUNDS=2 timeout -k 10 600 bash tools/variants.sh && \
TAG=${T}_c5 ROUNDS=2 EXTRA="--config C5" timeout -k 10 900 bash tools/variants.sh && \
TAG=${T}_c4 ROUNDS=2 EXTRA="--config C4" timeout -k 10 900 bash tools/variants.sh
