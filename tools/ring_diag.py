"""Per-step cycle stamps of vqf_decide_ring's decider wave for one lone leaf (diagnostic build:
hipcc -O3 --offload-arch=gfx950 -std=c++17 -shared -fPIC -Iinclude -DTKV_DIAG_RING
-DTKV_AMQ_EXPERIMENT_BUILD -o tools/diag/libtkv_amq_diag.so turtle_kv_amd/csrc/*.hip *.cpp,
run with TKV_AMQ_EXPERIMENT=1 TKV_AMQ_LIB=tools/diag/libtkv_amq_diag.so: tools/gpu/plans/
ring_diag.txt; tools/diag/ travels to the GPU box, tools/exp/ does not).
Prints, over the leaf's 64-key steps: the wait for the slot, the count read (one LDS round trip
after the previous step's count update), the decision, and the whole step (stamp to stamp)."""
import ctypes
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import turtle_kv_amd as amq  # noqa: E402
from bench import sort_segments_device  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 16384
    keys = sort_segments_device(torch, amq.gen_keys16(42, 0, n), [n])
    cap = amq.TreeOptions(1).set_filter_bits_per_key(12).filter_page_payload_size()
    plan = amq.plan_filters(1, [n], 12, payload_capacity=cap)
    kb = amq.KeyBatch.fixed(keys)
    out = torch.empty(plan.total_out_bytes, dtype=torch.uint8, device="cuda")
    ws = torch.empty(plan.workspace_bytes, dtype=torch.uint8, device="cuda")
    for _ in range(200):
        amq.build_all_filters(plan, kb, out=out, workspace=ws, check=False)
    torch.cuda.synchronize()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(50)]
    for a, b in ev:
        a.record()
        amq.build_all_filters(plan, kb, out=out, workspace=ws, check=False)
        b.record()
    torch.cuda.synchronize()
    us = float(np.median([a.elapsed_time(b) for a, b in ev])) * 1e3
    L = amq.abi.lib()
    buf = np.zeros(4 * 4096 + 8, np.uint64)
    L.tkv_amq_diag_read.argtypes = [ctypes.c_void_p]
    assert L.tkv_amq_diag_read(buf.ctypes.data) == 0
    steps = (n + 63) // 64
    d = buf[:4 * steps].reshape(steps, 4)
    wait, cntr, dec = d[:, 0].astype(float), d[:, 1].astype(float), d[:, 2].astype(float)
    spins = (d[:, 3] & 0xffffffff).astype(int)
    alts = (d[:, 3] >> 32).astype(int)  # 1: a lane reached the threshold (the slow path)
    print(f"leaf {n} keys, {steps} steps, build median {us:.1f} us")
    for name, v in (("wait", wait), ("count read", cntr), ("decision", dec)):
        print(f"  {name:10s} mean {v.mean():7.1f}  median {np.median(v):7.1f}  p90 {np.percentile(v, 90):7.1f} cycles")
    alt = alts > 0
    print(f"  slow steps {alt.mean():.2f}: decision {dec[alt].mean():.0f} vs {dec[~alt].mean():.0f} cycles; "
          f"step total {(wait + cntr + dec)[alt].mean():.0f} vs {(wait + cntr + dec)[~alt].mean():.0f}")
    print(f"  steps that waited for a slot: {(spins > 0).mean():.2f}")
    tot = wait + cntr + dec
    print(f"  sum per step {tot.mean():.0f} cycles = {tot.sum() / 2.4e3:.1f} us at 2.4 GHz")
    k = buf[4 * 4096:4 * 4096 + 3].astype(np.int64)
    if k[2] > 0:
        print(f"  ring_place kernel (leaf 0): decide {(k[1] - k[0]) / 2.4e3:.1f} us, "
              f"place sort {(k[2] - k[1]) / 2.4e3:.1f} us at 2.4 GHz (s_memtime)")


if __name__ == "__main__":
    main()
