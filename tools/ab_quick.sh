#!/bin/bash
# A/B of the built variants on one config (default C2): interleaved bench rounds + parity spot check.
# usage (via gpurun): bash tools/ab_quick.sh TAG [ROUNDS] [extra bench args]
set -o pipefail
export TMPDIR=/tmp
T=${1:-abq}; R=${2:-2}; shift; shift
TAG=$T ROUNDS=$R EXTRA="$*" timeout -k 10 900 bash tools/variants.sh
