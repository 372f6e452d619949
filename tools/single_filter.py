"""Build time of one Bloom filter per batch at sizes around the window path / tiled build
threshold (kWinMonoMax): 16-byte keys, HIP events, 20 reps.  With TKV_AMQ_LIB (and
TKV_AMQ_EXPERIMENT=1) an experiment build of the library is timed instead."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch

    import turtle_kv_amd as amq
    for bpk in (10, 12):
        for n in (150_000, 200_000, 300_000, 400_000, 500_000, 650_000, 800_000, 1_000_000, 1_500_000):
            keys = amq.gen_keys16(7, 0, n)
            kb = amq.KeyBatch.fixed(keys)
            plan = amq.plan_filters(amq.BLOOM, [n], bpk)
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
            win = -(-plan.max_seg_blocks * 64 // (160 * 1024))
            print(f"bpk {bpk} n {n}: {win} windows, {ms * 1e3:.1f} us, {n / ms / 1e6:.1f} Gkeys/s", flush=True)


if __name__ == "__main__":
    main()
