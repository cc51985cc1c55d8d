"""The C ABI driven from plain C (examples/qlin_c_demo.c): compiled with gcc against
include/qlin_gfx950.h and the in-tree library.  CPU: ABI version and argument validation;
GPU: quantize + pack + fused GEMV checked against the exact dequantized weight."""
import os
import shutil
import subprocess

import pytest

from conftest import ROOT

LIBDIR = os.path.join(ROOT, "llama3-quantization_amd", "csrc")


@pytest.fixture(scope="module")
def demo(tmp_path_factory):
    if not shutil.which("gcc"):
        pytest.skip("gcc not available")
    out = str(tmp_path_factory.mktemp("cdemo") / "qlin_c_demo")
    cmd = ["gcc", "-O2", "-I", os.path.join(ROOT, "include"), "-I", "/opt/rocm/include",
           "-D__HIP_PLATFORM_AMD__", os.path.join(ROOT, "examples", "qlin_c_demo.c"),
           "-L", LIBDIR, "-lqlin_gfx950", "-L", "/opt/rocm/lib", "-lamdhip64", "-lm",
           "-Wl,-rpath," + LIBDIR + ":/opt/rocm/lib", "-o", out]
    subprocess.run(cmd, check=True, capture_output=True, text=True)
    return out


def test_c_abi_version_and_validation(demo):
    r = subprocess.run([demo, "--abi"], capture_output=True, text=True, timeout=60)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "argument validation ok" in r.stdout


@pytest.mark.gpu
def test_c_abi_quantize_gemv(demo):
    r = subprocess.run([demo], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
