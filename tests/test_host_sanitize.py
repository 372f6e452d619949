"""CPU: the host code under AddressSanitizer + UndefinedBehaviorSanitizer, and ThreadSanitizer.

tests/cpp/test_host_sanitize.cpp links the host part of tkv_amq_kernels.hip (the plan and
TreeOptions sizing entry points), tkv_amq_stage.cpp and the C oracle, all built with
`-fsanitize=address,undefined` (hipcc: host side only, `-Xarch_host`; the oracle with the same
clang).  The driver runs cases from stdin; every result line must equal the same call through
the unsanitized libraries (ctypes), and any sanitizer report fails the run.  The threaded
paths (key staging, the oracle's checkpoint-level build) also run under ThreadSanitizer.
No device."""
import ctypes
import os
import subprocess

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
CLANG = "/opt/rocm/llvm/bin/clang"
SAN = ["-fsanitize=address", "-fsanitize=undefined", "-fno-sanitize-recover=all"]


def fnv(b: bytes) -> int:
    h = 1469598103934665603
    for x in b:
        h = ((h ^ x) * 1099511628211) & 0xFFFFFFFFFFFFFFFF
    return h


def build_driver(d, san):
    if not (os.path.exists(HIPCC) and os.path.exists(CLANG)):
        pytest.skip("ROCm clang / hipcc not installed")
    SAN = san
    inc = ["-I" + os.path.join(ROOT, "include")]
    host_san = [f for s in SAN for f in ("-Xarch_host", s)]
    steps = [
        [CLANG, "-O1", "-g", "-fno-omit-frame-pointer", "-std=gnu11", *SAN, "-c",
         os.path.join(ROOT, "oracle", "tkv_amq_oracle.c"), "-o", str(d / "oracle.o")],
        # device code too (the host object registers the gfx950 code object); device code is
        # not sanitized
        [HIPCC, "--offload-arch=gfx950", "-O1", "-g", "-std=c++17", *inc, *host_san, "-c",
         os.path.join(ROOT, "turtle_kv_amd", "csrc", "tkv_amq_kernels.hip"), "-o", str(d / "kernels.o")],
        [HIPCC, "-O1", "-g", "-std=c++17", *inc, *host_san, "-c",
         os.path.join(ROOT, "turtle_kv_amd", "csrc", "tkv_amq_stage.cpp"), "-o", str(d / "stage.o")],
        [HIPCC, "-O1", "-g", "-std=c++17", *inc, *host_san, "-c",
         os.path.join(ROOT, "tests", "cpp", "test_host_sanitize.cpp"), "-o", str(d / "main.o")],
        [HIPCC, *host_san, "-o", str(d / "test_host_sanitize"), str(d / "main.o"), str(d / "kernels.o"),
         str(d / "stage.o"), str(d / "oracle.o"), "-lpthread", "-lm"],
    ]
    for cmd in steps:
        r = subprocess.run(cmd, capture_output=True, text=True, timeout=300)
        assert r.returncode == 0, f"{' '.join(cmd)}\n{r.stderr[-3000:]}"
    return str(d / "test_host_sanitize")


@pytest.fixture(scope="module")
def driver(tmp_path_factory):
    return build_driver(tmp_path_factory.mktemp("asan"), SAN)


@pytest.fixture(scope="module")
def tsan_driver(tmp_path_factory):
    return build_driver(tmp_path_factory.mktemp("tsan"), ["-fsanitize=thread"])


def run(driver, lines):
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0:halt_on_error=1",
               UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1",
               TSAN_OPTIONS="halt_on_error=1")
    r = subprocess.run([driver], input="\n".join(lines) + "\n", capture_output=True, text=True,
                       timeout=300, env=env)
    assert r.returncode == 0 and "Sanitizer" not in r.stderr, r.stderr[-4000:]
    out = r.stdout.strip().splitlines()
    assert len(out) == len(lines)
    return [ln.split() for ln in out]


def plan_cases():
    rng = np.random.default_rng(5)
    cases = []
    for kind, bpks in ((0, [0, 1, 10, 33, 64, 65]), (1, [0, 11, 12, 16, 22, 40])):
        for bpk in bpks:
            for n in (0, 1, 7, 300):
                counts = [int(c) for c in rng.integers(0, 70000, n)]
                if n > 2:
                    counts[0], counts[1] = 0, 1 << 20
                for cap, stride, pl in ((32704, 0, 0), (65472, 0, 0), (8128, 65536, 0), (0, 0, 15),
                                        (0, 0, 20), (64, 0, 0)):
                    cases.append((kind, bpk, cap, stride, pl, counts))
    return cases


def test_plan_and_sizing_sanitized(driver, amq):
    L = amq.abi.lib()
    cases = plan_cases()
    lines = [f"plan {k} {b} {c} {s} {p} {len(cnt)} " + " ".join(map(str, cnt))
             for k, b, c, s, p, cnt in cases]
    sizes = [(k, leaf, key, val, bpk) for k in (0, 1) for leaf in (0, 104, 4096, 2 << 20, 32 << 20)
             for key, val in ((24, 100), (16, 0), (200, 1000)) for bpk in (0, 10, 12, 24)]
    lines += ["size %d %d %d %d %d" % s for s in sizes]
    got = run(driver, lines)
    for (k, b, c, s, p, cnt), g in zip(cases, got):
        n = len(cnt)
        counts = np.asarray(cnt, dtype=np.uint64)
        segs = np.zeros(max(n, 1) * 64, np.uint8)
        total, ws, mb = ctypes.c_uint64(), ctypes.c_uint64(), ctypes.c_uint32()
        cp = ctypes.c_void_p(counts.ctypes.data) if n else None
        sp = ctypes.c_void_p(segs.ctypes.data) if n else None
        if p:
            st = L.tkv_amq_plan_pages(k, cp, None, n, b, p, sp, ctypes.byref(total), ctypes.byref(ws),
                                      ctypes.byref(mb))
        else:
            st = L.tkv_amq_plan(k, cp, None, n, b, c, s, sp, ctypes.byref(total), ctypes.byref(ws),
                                ctypes.byref(mb))
        h = fnv(segs[:64 * n].tobytes()) if st == 0 and n else 0
        assert g == ["plan", str(st), str(total.value), str(ws.value), str(mb.value), str(h)], (k, b, c, s, p, n)
    for s, g in zip(sizes, got[len(cases):]):
        k, leaf, key, val, bpk = s
        want = ["size", str(L.tkv_amq_filter_page_size_log2(k, leaf, key, val, bpk)),
                str(L.tkv_amq_expected_items_per_leaf(leaf, key, val)), str(L.tkv_amq_leaf_data_size(leaf))]
        assert g == want, s


def test_oracle_sanitized(driver, oracle):
    blooms = [(n, bpk, 40 + n) for n in (0, 1, 63, 4096, 16384) for bpk in (0, 1, 10, 33)]
    vqfs = [(n, bpk, cap, 50 + n) for n in (0, 1, 777, 16384, 40000) for bpk in (12, 22)
            for cap in (8128, 32704)]
    got = run(driver, ["bloom %d %d %d" % c for c in blooms] + ["vqf %d %d %d %d" % c for c in vqfs])
    for (n, bpk, seed), g in zip(blooms, got):
        keys = oracle.gen_keys16(seed, 0, n)
        st, pl = oracle.bloom_build(keys, n, bpk, src_page_id=7)
        assert g == ["bloom", str(st), str(fnv(pl.tobytes())), "0"], (n, bpk)
    for (n, bpk, cap, seed), g in zip(vqfs, got[len(blooms):]):
        keys = oracle.gen_keys16(seed, 0, n)
        oracle.sort_segments(keys, np.array([0, n], np.uint64), 1)
        st, pl, p = oracle.vqf_build(keys, n, bpk, cap, src_page_id=9)
        used = p.payload_used if st == 0 else 0
        assert g[:4] == ["vqf", str(st), str(fnv(pl[:used].tobytes())), str(used)], (n, bpk, cap)
        assert g[4] == "0", f"false negatives {(n, bpk, cap)}"


def test_stage_sanitized(driver):
    cases = [(16, 1, 0), (16, 40000, 0), (24, 5000, 3), (0, 0, 0), (0, 1, 1), (0, 70000, 0),
             (0, 300000, 7)]
    got = run(driver, ["stage %d %d %d %d" % (f, n, t, 100 + i) for i, (f, n, t) in enumerate(cases)])
    for c, g in zip(cases, got):
        assert g == ["stage", "0", "1"], c


def oracle_build_expect(oracle, kind, n_segs, per, bpk, threads, seed):
    n = per * n_segs
    keys = oracle.gen_keys16(seed, 0, n)
    begin = np.arange(n_segs + 1, dtype=np.uint64) * per
    if kind == 1:
        oracle.sort_segments(keys, begin, threads)
    cap = oracle.lib().tkvo_bloom_payload_size(per, bpk) if kind == 0 else 32704
    off = np.arange(n_segs, dtype=np.uint64) * cap
    capv = np.full(n_segs, cap, np.uint64)
    out = np.zeros(int(cap) * n_segs + 1, np.uint8)
    P = oracle._p
    st = oracle.lib().tkvo_build_segments(kind, P(keys), P(begin), n_segs, bpk, None, P(out), P(off),
                                          P(capv), threads)
    return ["obuild", str(st), str(fnv(out[:int(cap) * n_segs].tobytes()))]


@pytest.mark.parametrize("which", ["asan", "tsan"])
def test_threaded_paths_sanitized(driver, tsan_driver, oracle, which):
    d = driver if which == "asan" else tsan_driver
    builds = [(0, 16, 3000, 10, 4, 61), (1, 16, 3000, 12, 4, 62), (0, 5, 700, 33, 8, 63)]
    stages = [(16, 200000, 6), (0, 150000, 5)]
    got = run(d, ["obuild %d %d %d %d %d %d" % c for c in builds] +
              ["stage %d %d %d %d" % (f, n, t, 200 + i) for i, (f, n, t) in enumerate(stages)])
    for c, g in zip(builds, got):
        assert g == oracle_build_expect(oracle, *c), c
    for c, g in zip(stages, got[len(builds):]):
        assert g == ["stage", "0", "1"], c
