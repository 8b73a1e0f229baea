#!/bin/bash
# Round-5 session k: contact case_04 over LDS (and the contact type taken before the contact point):
# parity of each variant on the fixtures that reach every case_04 branch, then A/B on C2 / C4 / C5.
# usage (via gpurun): bash tools/gpu_r5k.sh <tag> <variant>...
set -o pipefail
TAG=$1; shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
D=collision-detect-gjk-epa_amd/build
for v in "$@"; do
  echo "== parity $v $(date)"
  GJKEPA_LIB=$D/variants/$v/libgjkepa_hip.so timeout -k 10 400 python -u -m pytest tests/test_branch_cov.py tests/test_gpu_parity.py tests/test_contacts.py -q -m gpu --timeout 300 --timeout-method thread > $OUT/parity_$v.log 2>&1 || { tail -20 $OUT/parity_$v.log; exit 1; }
  tail -1 $OUT/parity_$v.log
done
echo "== ab $(date)" && bash tools/gpu_r5_ab.sh $TAG 2 "C2 C4 C5" "$@" || exit 1
echo "== done $(date)"
