"""Build rate of Bloom batches of window-sized leaves (5-16 LDS windows each), 16-byte keys
@10 bits/key, HIP events, 10 reps: the window path, or (an experiment build with a lower
oversize threshold, TKV_AMQ_LIB) the multi-leaf tiled build."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch

    import turtle_kv_amd as amq
    for name, counts in [("128 x 650K (5 windows)", [650_000] * 128),
                         ("64 x 1M (8 windows)", [1_000_000] * 64),
                         ("48 x 1.5M (12 windows)", [1_500_000] * 48),
                         ("32 x 2M (16 windows)", [2_000_000] * 32),
                         ("8 x 1M + 500 x 16K", [1_000_000] * 8 + [16384] * 500)]:
        n = sum(counts)
        keys = amq.gen_keys16(5, 0, n)
        kb = amq.KeyBatch.fixed(keys)
        plan = amq.plan_filters(amq.BLOOM, counts, 10)
        out = torch.empty(plan.total_out_bytes, dtype=torch.uint8, device="cuda")
        ws = torch.empty(max(1, plan.workspace_bytes), dtype=torch.uint8, device="cuda")
        for _ in range(3):
            amq.build_all_filters(plan, kb, out=out, workspace=ws, check=False)
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(10)]
        for a, b in ev:
            a.record()
            amq.build_all_filters(plan, kb, out=out, workspace=ws, check=False)
            b.record()
        torch.cuda.synchronize()
        ms = float(np.median([a.elapsed_time(b) for a, b in ev]))
        print(f"{name}: {n} keys, {ms * 1e3:.1f} us, {n / ms / 1e6:.1f} Gkeys/s", flush=True)
        del out, ws, keys, kb


if __name__ == "__main__":
    main()
