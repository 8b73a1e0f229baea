#!/bin/bash
# Round-5 session r: A/B of library variants (build/variants/NAME) and of environment settings of the
# in-tree build (NAME=ENV=VALUE), two interleaved rounds on C2 / C4 / C5 after a parity pass per variant.
# usage (via gpurun): [SUITE=1] bash tools/gpu_r5r.sh <tag> <variant | name=ENV=value>...  (SUITE=1: the GPU suite first)
set -o pipefail
TAG=$1; shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
D=collision-detect-gjk-epa_amd/build
if [ "${SUITE:-0}" = 1 ]; then
  echo "== tests $(date)"
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -30 $OUT/pytest_gpu.log; exit 1; }
  tail -1 $OUT/pytest_gpu.log
fi
for v in "$@"; do
  case "$v" in *=*) continue ;; esac
  echo "== parity $v $(date)"
  GJKEPA_LIB=$D/variants/$v/libgjkepa_hip.so timeout -k 10 400 python -u -m pytest tests/test_branch_cov.py tests/test_gpu_parity.py tests/test_contacts.py -q -m gpu --timeout 300 --timeout-method thread > $OUT/parity_$v.log 2>&1 || { tail -20 $OUT/parity_$v.log; exit 1; }
  tail -1 $OUT/parity_$v.log
done
for r in 1 2; do
  for v in main "$@"; do
    name=${v%%=*}; lib=$D/libgjkepa_hip.so; envset=""
    case "$v" in
      main) ;;
      *=*) envset=${v#*=} ;;
      *) lib=$D/variants/$v/libgjkepa_hip.so ;;
    esac
    for c in C2 C4 C5; do
      env GJKEPA_LIB=$lib $envset timeout -k 10 240 python bench.py --config $c --legs none --no-cpu --no-f32-leg --no-warm-leg --launch-timing off \
        > $OUT/ab_${name}_${c}_$r.json 2>> $OUT/ab.err || { echo "FAIL $v $c"; tail -5 $OUT/ab.err; exit 1; }
      echo "$r $name $c $(python3 -c "import json;d=json.loads(open('$OUT/ab_${name}_${c}_$r.json').read().splitlines()[-1]);print(d['value'], d['ms_per_step'])")"
    done
  done
done
echo "== done $(date)"
