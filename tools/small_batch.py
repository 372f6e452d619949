"""Time builds of the first L leaves of the bench layout (16,384-key leaves, 16-byte keys) for
several L: the small-batch curve (a checkpoint's build_all_pages queue holds tens to
thousands of leaves).  Run under rocprofv3 --kernel-trace --stats for per-kernel times.

  python tools/small_batch.py [--kind 0|1] [--leaves 1,8,64,256,512,1024] [--reps 50]
"""
import argparse
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import turtle_kv_amd as amq  # noqa: E402
from bench import sort_segments_device  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--kind", type=int, default=0)
    ap.add_argument("--bpk", type=int, default=0)
    ap.add_argument("--leaves", default="1,8,64,256,512,1024")
    ap.add_argument("--reps", type=int, default=50)
    ap.add_argument("--leaf-keys", type=int, default=16384)
    ap.add_argument("--key-bytes", type=int, default=16,
                    help="16 (splitmix keys, sorted per leaf for VQF), 24 (random 24-byte keys) or "
                         "0 (variable length, 8-31 bytes through an offsets array); the last two "
                         "in generation order")
    ap.add_argument("--var-lens", default="8,32",
                    help="variable-length keys: lengths uniform in [lo, hi) (e.g. 24,25: all 24 bytes "
                         "through an offsets array, the reference's KeyView form of TurtleKV keys)")
    ap.add_argument("--cap", type=int, default=0,
                    help="VQF payload capacity (default: the TreeOptions filter page at --bpk)")
    ap.add_argument("--no-ws", action="store_true",
                    help="call the ABI without a workspace (Bloom: the unsplit paths)")
    ap.add_argument("--ws-bytes", type=int, default=-1,
                    help="call the ABI with exactly this much workspace (Bloom window path: "
                         "one part per leaf when short of the partial images)")

    a = ap.parse_args()
    bpk = a.bpk or (10 if a.kind == 0 else 12)
    cap = a.cap or (amq.TreeOptions(a.kind).set_filter_bits_per_key(bpk).filter_page_payload_size()
                    if a.kind else 0)
    S = a.leaf_keys
    for L in [int(x) for x in a.leaves.split(",")]:
        counts = [S] * L
        if a.key_bytes == 16:
            keys = amq.gen_keys16(42, 0, S * L)
            if a.kind == 1:
                keys = sort_segments_device(torch, keys, counts)
            kb = amq.KeyBatch.fixed(keys)
        elif a.key_bytes == 0:
            g = torch.Generator(device="cuda")
            g.manual_seed(42)
            lo, hi = (int(x) for x in a.var_lens.split(","))
            lens = torch.randint(lo, hi, (S * L,), dtype=torch.int64, device="cuda", generator=g)
            offs = torch.zeros(S * L + 1, dtype=torch.int64, device="cuda")
            torch.cumsum(lens, 0, out=offs[1:])
            blob = torch.randint(0, 256, (int(offs[-1].item()),), dtype=torch.uint8, device="cuda",
                                 generator=g)
            kb = amq.KeyBatch.variable(blob, offs)
        else:
            g = torch.Generator(device="cuda")
            g.manual_seed(42)
            kb = amq.KeyBatch.fixed(torch.randint(0, 256, (S * L, a.key_bytes), dtype=torch.uint8,
                                                  device="cuda", generator=g))
        plan = amq.plan_filters(a.kind, counts, bpk, payload_capacity=cap)
        out = torch.empty(plan.total_out_bytes, dtype=torch.uint8, device="cuda")
        ws = torch.empty(max(plan.workspace_bytes, 1), dtype=torch.uint8, device="cuda")
        lib, F = amq.abi.lib(), amq.filters
        segs = plan.device_segs()

        ws_bytes = a.ws_bytes

        def build():
            if ws_bytes >= 0:
                amq.abi.check(lib.tkv_amq_build(a.kind, F._ptr(kb.data), F._ptr(kb.offsets), kb.stride,
                                              kb.n, F._ptr(segs), plan.n_segs, plan.max_seg_blocks,
                                              F._ptr(out), F._ptr(ws) if ws_bytes else None, ws_bytes,
                                              F._stream_handle()), "build")
            elif a.no_ws:
                amq.abi.check(lib.tkv_amq_build(a.kind, F._ptr(kb.data), None, 16, kb.n, F._ptr(segs),
                                              plan.n_segs, plan.max_seg_blocks, F._ptr(out), None, 0,
                                              F._stream_handle()), "build")
            else:
                amq.build_all_filters(plan, kb, out=out, workspace=ws, check=False)
        for _ in range(5):
            build()
        torch.cuda.synchronize()
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
              for _ in range(a.reps)]
        for e0, e1 in ev:
            e0.record()
            build()
            e1.record()
        torch.cuda.synchronize()
        ms = float(np.median([e0.elapsed_time(e1) for e0, e1 in ev]))
        print(f"kind {a.kind} kb {a.key_bytes:2d} leaves {L:5d} keys {S * L:9d} median {ms * 1e3:8.1f} us "
              f"{S * L / ms / 1e3:9.1f} Mkeys/s ws {plan.workspace_bytes}", flush=True)


if __name__ == "__main__":
    main()
