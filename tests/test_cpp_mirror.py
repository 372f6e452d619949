"""The C++ host mirror (include/turtle_kv_amd/filter_builder.hpp): compiled against
libtkv_amq.so; on CPU it must fail loudly (Unavailable), on the GPU it must reproduce the
golden filter pages byte for byte."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def build_mirror_test(tmp_path):
    from turtle_kv_amd import _build
    _build.build()
    exe = str(tmp_path / "test_mirror")
    subprocess.run(["/opt/rocm/bin/hipcc", "-O2", "-std=c++17", "-I" + os.path.join(ROOT, "include"),
                    "-o", exe, os.path.join(ROOT, "tests", "cpp", "test_mirror.cpp"),
                    "-L" + os.path.join(ROOT, "turtle_kv_amd"), "-ltkv_amq",
                    "-Wl,-rpath," + os.path.join(ROOT, "turtle_kv_amd")], check=True,
                   capture_output=True)
    return exe


def test_cpp_mirror_compiles_and_fails_loudly_without_gpu(tmp_path):
    exe = build_mirror_test(tmp_path)
    r = subprocess.run([exe, os.path.join(ROOT, "tests", "golden")], capture_output=True, text=True)
    if "NODEVICE" not in r.stdout:
        pytest.skip("a GPU is visible; covered by the gpu test")
    assert r.returncode == 0, r.stdout + r.stderr


@pytest.mark.gpu
def test_cpp_mirror_gpu(tmp_path):
    exe = build_mirror_test(tmp_path)
    r = subprocess.run([exe, os.path.join(ROOT, "tests", "golden")], capture_output=True, text=True,
                       timeout=300)
    assert r.returncode == 0 and r.stdout.startswith("OK"), r.stdout + r.stderr
