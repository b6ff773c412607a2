"""Plain-C consumer of the ABI (examples/abi_demo.c): builds with gcc against
include/curve_crc.h + libcurvecrc.so and runs -- CPU checks here, all checks
(device page CRCs, slices, host paths, verify) on a GPU."""
import os
import subprocess

import pytest

from conftest import ROOT


def build_demo(tmp_path):
    exe = str(tmp_path / "abi_demo")
    cmd = ["gcc", "-O2", "-std=c11", "-D__HIP_PLATFORM_AMD__", "-I/opt/rocm/include", f"-I{ROOT}/include",
           f"{ROOT}/examples/abi_demo.c", f"-L{ROOT}/curve_amd", "-lcurvecrc", "-L/opt/rocm/lib", "-lamdhip64",
           f"-Wl,-rpath,{ROOT}/curve_amd", "-Wl,-rpath,/opt/rocm/lib", "-o", exe]
    subprocess.run(cmd, check=True, capture_output=True)
    return exe


def test_abi_demo_cpu(tmp_path):
    r = subprocess.run([build_demo(tmp_path)], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr


@pytest.mark.gpu
def test_abi_demo_gpu(tmp_path):
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    r = subprocess.run([build_demo(tmp_path)], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0 and "all checks passed" in r.stdout, r.stdout + r.stderr
