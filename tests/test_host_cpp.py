"""The C++ host layer (curve_amd/host: chunkserver surfaces over the C ABI)
through its own test binary, whose cases follow the reference's gtest cases.
CPU: every non-GPU case must pass (GPU cases report SKIP).  GPU: all cases."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HOST = os.path.join(ROOT, "curve_amd", "host")
BIN = os.path.join(HOST, "host_test")


@pytest.fixture(scope="module")
def host_test():
    if not os.path.exists(os.path.join(ROOT, "curve_amd", "libcurvecrc.so")):
        subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "curve_amd", "csrc")], check=True)
    # only the test binary: relinking the shared harnesses here (make's `all`, after a
    # libcurvecrc rebuild) raced the xdist workers that dlopen them at the same time
    subprocess.run(["make", "-s", "-C", HOST, "host_test"], check=True)
    return BIN


def run(binary, *args, timeout=300):
    p = subprocess.run([binary, *args], capture_output=True, text=True, timeout=timeout)
    return p.returncode, p.stdout + p.stderr


def test_host_layer_cpu_cases(host_test):
    import torch
    if torch.cuda.device_count() > 0:  # counting devices does not initialise HIP here
        pytest.skip("GPU present: covered by test_host_layer_all_cases")
    rc, out = run(host_test)
    assert rc == 0, out
    assert "6 ran, 0 failed, 8 skipped" in out, out


@pytest.mark.gpu
def test_host_layer_all_cases(host_test):
    rc, out = run(host_test, "--gpu")
    assert rc == 0, out
    assert "14 ran, 0 failed, 0 skipped" in out, out
