"""In-tree build of libtkv_amq.so (hipcc, gfx950).  No JIT cache: the .so lives next to
this file so it travels to the GPU box with the repo snapshot."""
from __future__ import annotations

import os
import subprocess

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
LIB = os.path.join(HERE, "libtkv_amq.so")
SOURCES = [os.path.join(HERE, "csrc", "tkv_amq_kernels.hip"),
           os.path.join(HERE, "csrc", "tkv_amq_stage.cpp")]
DEPS = SOURCES + [os.path.join(HERE, "csrc", "tkv_amq_device.h"),
                  os.path.join(ROOT, "include", "tkv_amq.h")]
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
FLAGS = ["-O3", "--offload-arch=gfx950", "-std=c++17", "-shared", "-fPIC",
         "-Wall", "-Wno-unused-function", "-I" + os.path.join(ROOT, "include")]


def stale() -> bool:
    if not os.path.exists(LIB):
        return True
    t = os.path.getmtime(LIB)
    return any(os.path.getmtime(d) > t for d in DEPS)


def build(force: bool = False) -> str:
    if force or stale():
        tmp = LIB + ".tmp"
        subprocess.run([HIPCC, *FLAGS, "-o", tmp, *SOURCES], check=True)
        os.replace(tmp, LIB)
    return LIB


if __name__ == "__main__":
    print(build(force=True))
