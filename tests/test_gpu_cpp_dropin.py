"""Build tests/cpp/test_dropin.cc against include/RandBLAS.hh (the drop-in C++ header) with g++ and
run it on the GPU: a reference-style client using host arrays and the reference's overloads."""
import os
import subprocess

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_cpp_dropin_client(tmp_path):
    exe = str(tmp_path / "test_dropin")
    libdir = os.path.join(ROOT, "randblas_amd")
    subprocess.run(["g++", "-std=c++17", "-O2", "-Wall", "-I", os.path.join(ROOT, "include"), "-I", "/opt/rocm/include",
                    "-D__HIP_PLATFORM_AMD__",
                    os.path.join(ROOT, "tests", "cpp", "test_dropin.cc"), "-L", libdir, "-lrandblas_hip", "-L/opt/rocm/lib", "-lamdhip64",
                    f"-Wl,-rpath,{libdir}", "-o", exe], check=True)
    out = subprocess.run([exe], capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stdout + out.stderr
    assert "ALL PASSED" in out.stdout
