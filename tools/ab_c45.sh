set -o pipefail
export TMPDIR=/tmp
TAG=abprio5 ROUNDS=2 EXTRA="--config C5" timeout -k 10 900 bash tools/variants.sh && TAG=abprio4 ROUNDS=2 EXTRA="--config C4" timeout -k 10 900 bash tools/variants.sh
