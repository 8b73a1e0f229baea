set -o pipefail
export TMPDIR=/tmp
TAG=abscan ROUNDS=2 timeout -k 10 600 bash tools/variants.sh && bash tools/callpattern_probe.sh abscan_cp 5000 50000
