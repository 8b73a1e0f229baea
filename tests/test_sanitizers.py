"""Host code under AddressSanitizer + UndefinedBehaviorSanitizer: the product's
workload generators (csrc/synth.cpp) and the oracle restatement, driven over pair pools, point
clouds and a scene by tests/asan/driver.c.  GPU sanitizers are not available on this pool; the
device code is covered by the bit-exact parity tests instead."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(shutil.which("gcc") is None or shutil.which("g++") is None, reason="needs gcc/g++")
def test_host_code_is_sanitizer_clean(tmp_path):
    san = ["-fsanitize=address,undefined", "-fno-sanitize-recover=all", "-fno-omit-frame-pointer", "-O1", "-g",
           "-fopenmp", "-ffp-contract=off"]
    objs = []
    for src, cc, std in [("oracle/gjkepa_oracle.c", "gcc", "-std=c11"),
                         ("collision-detect-gjk-epa_amd/csrc/synth.cpp", "g++", "-std=c++17"),
                         ("tests/asan/driver.c", "gcc", "-std=c11")]:
        obj = str(tmp_path / (os.path.basename(src) + ".o"))
        subprocess.run([cc, std, *san, "-c", os.path.join(ROOT, src), "-o", obj], check=True, cwd=ROOT)
        objs.append(obj)
    exe = str(tmp_path / "driver")
    subprocess.run(["g++", *san, *objs, "-o", exe, "-lm"], check=True)
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=1", OMP_NUM_THREADS="2",
               UBSAN_OPTIONS="print_stacktrace=1")
    out = subprocess.run([exe], capture_output=True, text=True, timeout=300, env=env)
    assert out.returncode == 0, out.stdout[-2000:] + out.stderr[-4000:]
    assert "sanitizers clean" in out.stdout
