"""Build rate of single Bloom filters past four LDS windows (the tiled monolithic build) and of
batches holding leaves past 16 windows (tkv_amq_build_ex: those leaves built together through
the tiled build, the others batched), @10 bits/key, HIP events, 20 reps."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch

    import turtle_kv_amd as amq
    for name, counts in [("one filter of 1M", [1_000_000]),
                         ("one filter of 3M", [3_000_000]),
                         ("one filter of 12M", [12_000_000]),
                         ("test batch [3M, 500, 16384]", [3_000_000, 500, 16384]),
                         ("8 x 3M + 200 x 16K", [3_000_000] * 8 + [16384] * 200),
                         ("64 x 3M", [3_000_000] * 64)]:
        n = sum(counts)
        keys = amq.gen_keys16(5, 0, n)
        kb = amq.KeyBatch.fixed(keys)
        plan = amq.plan_filters(amq.BLOOM, counts, 10)
        out = torch.empty(plan.total_out_bytes, dtype=torch.uint8, device="cuda")
        ws = torch.empty(max(1, plan.workspace_bytes), dtype=torch.uint8, device="cuda")
        for _ in range(3):
            amq.build_all_filters(plan, kb, out=out, workspace=ws, check=False)
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(20)]
        for a, b in ev:
            a.record()
            amq.build_all_filters(plan, kb, out=out, workspace=ws, check=False)
            b.record()
        torch.cuda.synchronize()
        ms = float(np.median([a.elapsed_time(b) for a, b in ev]))
        print(f"{name}: {n} keys, {ms * 1e3:.1f} us, {n / ms / 1e6:.1f} Gkeys/s", flush=True)


if __name__ == "__main__":
    main()
