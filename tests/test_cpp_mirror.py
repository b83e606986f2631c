"""The C++ host mirror (include/dcf.hpp) and its port of the reference's own
tests (tests/cpp/test_dcf.cpp): compiled here, run on the GPU."""
import json
import os
import subprocess

import pytest

from tests.conftest import GOLDEN, ROOT

BIN = os.path.join(ROOT, "tests", "cpp", "build", "test_dcf")


def build_cpp(hip_lib_path):
    os.makedirs(os.path.dirname(BIN), exist_ok=True)
    libdir = os.path.dirname(hip_lib_path)
    subprocess.check_call(["g++", "-std=c++17", "-O2", "-Wall", "-Wextra", "-I", os.path.join(ROOT, "include"),
                           os.path.join(ROOT, "tests", "cpp", "test_dcf.cpp"), "-o", BIN, "-L", libdir, "-ldcf_hip",
                           f"-Wl,-rpath,{libdir}"])
    return BIN


def test_cpp_mirror_compiles(hip_lib):
    assert os.path.exists(build_cpp(hip_lib._name))


@pytest.mark.gpu
def test_cpp_mirror_reference_tests_on_gpu(hip_lib):
    exe = build_cpp(hip_lib._name)
    row0 = json.load(open(os.path.join(GOLDEN, "prg16.json")))["rows"][0]
    env = dict(os.environ, DCF_PRG16_ROW0_SL=row0["sl"])
    r = subprocess.run([exe], env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "cpp mirror ok" in r.stdout
