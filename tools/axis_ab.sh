set -o pipefail
mkdir -p gpurun_out/axis
TAG=axis ROUNDS=2 bash tools/variants.sh || exit 1
for v in base axis; do
  GJKEPA_LIB=collision-detect-gjk-epa_amd/build/variants/$v/libgjkepa_hip.so timeout -k 10 300 python tools/bench_scene.py --no-cpu > gpurun_out/axis/scene_$v.json 2> gpurun_out/axis/scene_$v.err || exit 1
  echo "$v scene: $(tail -1 gpurun_out/axis/scene_$v.json | cut -c1-200)"
done
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/axis/pytest.log 2>&1; rc=$?; tail -5 gpurun_out/axis/pytest.log; exit $rc
