"""SURVEY §5 sanitizers: the CPU restatement (oracle/) and the C++ host code that needs no GPU,
built with AddressSanitizer + UBSan (-fno-sanitize-recover: any report fails the run) and run on
the reference's clouds and degenerate inputs.  Host-only (GPU ASan is not available on the pool)."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SAN = ["-O1", "-g", "-fno-omit-frame-pointer", "-fsanitize=address,undefined", "-fno-sanitize-recover=all"]


@pytest.fixture(scope="module")
def asan_driver(tmp_path_factory):
    if not shutil.which("g++"):
        pytest.skip("g++ not available")
    out = str(tmp_path_factory.mktemp("asan") / "oracle_asan")
    srcs = [os.path.join(ROOT, "oracle", f) for f in sorted(os.listdir(os.path.join(ROOT, "oracle")))
            if f.endswith(".cpp")]
    cmd = (["g++", "-std=c++14", "-ffp-contract=off", "-fopenmp"] + SAN +
           [os.path.join(ROOT, "tests", "cpp", "oracle_asan_driver.cpp")] + srcs + ["-o", out])
    subprocess.run(cmd, check=True, capture_output=True, text=True)
    return out


@pytest.mark.parametrize("cloud", ["indoor_source", "underwater_target"])
def test_oracle_under_asan_ubsan(asan_driver, cloud):
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0:halt_on_error=1",
               UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1", OMP_NUM_THREADS="2")
    p = subprocess.run([asan_driver, os.path.join(ROOT, "tests", "golden", "clouds", cloud + ".pcd"), "12"],
                       capture_output=True, text=True, env=env, timeout=600)
    assert p.returncode == 0, p.stdout[-2000:] + p.stderr[-4000:]
    assert "oracle sanitizer run clean" in p.stdout
    assert "runtime error" not in p.stderr and "AddressSanitizer" not in p.stderr
