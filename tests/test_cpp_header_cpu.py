"""The drop-in C++ header compiles with g++ (C++17 and C++20) against the C ABI (no GPU needed)."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.parametrize("std", ["c++17", "c++20"])
def test_header_compiles_and_links(tmp_path, std):
    exe = str(tmp_path / "t")
    libdir = os.path.join(ROOT, "randblas_amd")
    r = subprocess.run(["g++", f"-std={std}", "-O1", "-Wall", "-Werror", "-I", os.path.join(ROOT, "include"), "-I", "/opt/rocm/include",
                    "-D__HIP_PLATFORM_AMD__",
                        os.path.join(ROOT, "tests", "cpp", "test_dropin.cc"), "-L", libdir, "-lrandblas_hip", "-L/opt/rocm/lib", "-lamdhip64",
                        f"-Wl,-rpath,{libdir}", "-o", exe], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
