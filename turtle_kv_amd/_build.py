"""In-tree build of libtkv_amq.so (hipcc, gfx950).  No JIT cache: the .so lives next to
this file so it travels to the GPU box with the repo snapshot.

Several processes may ask for the library at once (bench.py's rank processes, pytest-xdist
workers): the stale check, the compile and the stamp run under an exclusive flock, the
check is repeated once the lock is held, and each process compiles into its own temp file
before the atomic rename."""
from __future__ import annotations

import fcntl
import hashlib
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


STAMP = LIB + ".src"  # sha256 of the sources and flags the library was built from
LOCK = LIB + ".lock"


def source_digest() -> str:
    h = hashlib.sha256(" ".join([HIPCC, *FLAGS]).encode())
    for d in DEPS:
        with open(d, "rb") as f:
            h.update(f.read())
    return h.hexdigest()


def stale() -> bool:
    """By content, not mtime: a checkout that restores an older source must rebuild."""
    if not (os.path.exists(LIB) and os.path.exists(STAMP)):
        return True
    with open(STAMP) as f:
        return f.read().strip() != source_digest()


def build(force: bool = False) -> str:
    if not force and not stale():
        return LIB
    with open(LOCK, "a") as lk:
        fcntl.flock(lk, fcntl.LOCK_EX)
        try:
            if force or stale():  # another process may have built it while we waited
                tmp = f"{LIB}.{os.getpid()}.tmp"
                digest = source_digest()
                try:
                    subprocess.run([HIPCC, *FLAGS, "-o", tmp, *SOURCES], check=True)
                    os.replace(tmp, LIB)
                finally:
                    if os.path.exists(tmp):
                        os.remove(tmp)
                with open(STAMP, "w") as f:
                    f.write(digest + "\n")
        finally:
            fcntl.flock(lk, fcntl.LOCK_UN)
    return LIB


if __name__ == "__main__":
    print(build(force=True))
