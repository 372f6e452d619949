"""Build rate of single Bloom filters past four LDS windows (the tiled monolithic build) and of
batches holding leaves past 16 windows (tkv_amq_build_ex: those leaves built together through
the tiled build, the others batched), @10 bits/key, HIP events, 20 reps.  --shape var / k20:
variable-length keys of 8-31 bytes, or 20-byte keys (random bytes made on the device), whose
leaves past 16 windows take bloom_part_any (round 5: device atomics)."""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def make_keys(torch, amq, shape, n):
    if shape == "k16":
        return amq.KeyBatch.fixed(amq.gen_keys16(5, 0, n))
    g = torch.Generator(device="cuda")
    g.manual_seed(5)
    if shape == "var":
        lens = torch.randint(8, 32, (n,), generator=g, device="cuda", dtype=torch.int64)
        offs = torch.zeros(n + 1, dtype=torch.int64, device="cuda")
        offs[1:] = torch.cumsum(lens, 0)
        data = torch.randint(0, 256, (int(offs[-1]),), generator=g, device="cuda", dtype=torch.uint8)
        return amq.KeyBatch.variable(data, offs)
    stride = int(shape[1:])
    return amq.KeyBatch.fixed(torch.randint(0, 256, (n, stride), generator=g, device="cuda",
                                            dtype=torch.uint8))


def main():
    import argparse

    import torch

    import turtle_kv_amd as amq
    ap = argparse.ArgumentParser()
    ap.add_argument("--shape", default="k16", help="k16, var, or kN (N-byte keys)")
    ap.add_argument("--only", default=None, help="run the cases whose name contains this")
    args = ap.parse_args()
    cases = [("one filter of 1M", [1_000_000]),
             ("one filter of 3M", [3_000_000]),
             ("one filter of 12M", [12_000_000]),
             ("test batch [3M, 500, 16384]", [3_000_000, 500, 16384]),
             ("8 x 3M + 200 x 16K", [3_000_000] * 8 + [16384] * 200),
             ("64 x 3M", [3_000_000] * 64)]
    if args.shape != "k16":  # (single filters of 1M keys take the window path, not the tiled build)
        cases = [c for c in cases if c[1] != [1_000_000]]
    if args.only:
        cases = [c for c in cases if args.only in c[0]]
    for name, counts in cases:
        n = sum(counts)
        kb = make_keys(torch, amq, args.shape, n)
        plan = amq.plan_filters(amq.BLOOM, counts, 10)
        out = torch.empty(plan.total_out_bytes, dtype=torch.uint8, device="cuda")
        ws = torch.empty(max(1, plan.workspace_bytes), dtype=torch.uint8, device="cuda")
        for _ in range(3):
            amq.build_all_filters(plan, kb, out=out, workspace=ws, check=False)
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(20)]
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for a, b in ev:
            a.record()
            amq.build_all_filters(plan, kb, out=out, workspace=ws, check=False)
            b.record()
        host_us = (time.perf_counter() - t0) / len(ev) * 1e6
        torch.cuda.synchronize()
        ms = float(np.median([a.elapsed_time(b) for a, b in ev]))
        # (host_us: the enqueue time per call; when it is above the events' time, the host and
        # not the device sets the rate of back-to-back calls)
        print(f"{args.shape} {name}: {n} keys, {ms * 1e3:.1f} us, {n / ms / 1e6:.1f} Gkeys/s "
              f"(host enqueue {host_us:.1f} us per call)", flush=True)
        del kb, out, ws
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
