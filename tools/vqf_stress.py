"""Repeatability stress for the VQF build (one 2-rank gloo run of
bench --chunks 3 --workload vqf12 gathered an array that differed from a one-GPU build).

Run one or several copies at once on the same GPU (the failing run had two processes sharing
the device):  python tools/vqf_stress.py --iters 40 --procs 2

Each process, per iteration:
  * regenerates the keys on the device (gen_keys16) and sorts each leaf with the bench's torch
    sort (sort_segments_device), and compares the sorted keys with the oracle's sort;
  * builds the bench's block-cyclic round plans (PipelinedLeafGather's, 2 ranks x 3 rounds of the
    4M-key layout) one after another on ONE workspace first filled with 0xFF, and the
    whole-batch plan on a fresh workspace;
  * compares every leaf's bytes with the first iteration's (and, on iteration 0, with the
    oracle).
Any difference is printed with its leaf and the iteration; exit 1."""
from __future__ import annotations

import argparse
import os
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def child(args, tag):
    import torch

    import bench
    import turtle_kv_amd as amq
    from oracle import oracle as O
    from turtle_kv_amd import dist as tdist
    O.build_oracle()
    dev = torch.device("cuda", 0)
    kind, bpk = 1, 12
    cap = amq.TreeOptions(kind).set_filter_bits_per_key(bpk).filter_page_payload_size()
    counts = bench.segment_counts(args.keys, 16384)
    W = 2
    per_rank = -(-len(counts) // W)
    q = -(-per_rank // 3)
    stride = tdist.leaf_stride(kind, bpk, max(counts), cap)
    sb = np.concatenate([[0], np.cumsum(counts)]).astype(np.uint64)
    host = O.gen_keys16(42, 0, int(sb[-1]))
    O.sort_segments(host, sb, n_threads=8)
    ref_keys = torch.from_numpy(host).to(dev)
    # plans: the whole batch, and every rank's rounds
    full_plan = amq.plan_filters(kind, counts, bpk, payload_capacity=cap, out_stride=stride)
    rounds = []
    for r in range(W):
        for b, e in tdist.cyclic_rounds(len(counts), W, r, q):
            if b < e:
                rounds.append((b, e, amq.plan_filters(kind, np.asarray(counts[b:e], np.uint64), bpk,
                                                      payload_capacity=cap, out_stride=stride,
                                                      src_page_ids=np.arange(b, e, dtype=np.uint64))))
    ws_bytes = max(p.workspace_bytes for _, _, p in rounds)
    ws = torch.empty(ws_bytes, dtype=torch.uint8, device=dev)
    first = None
    bad = 0
    t0 = time.time()
    for it in range(args.iters):
        keys = amq.gen_keys16(42, 0, int(sb[-1]), device=dev)
        keys = bench.sort_segments_device(torch, keys, counts)
        if not torch.equal(keys, ref_keys):
            rows = torch.nonzero((keys != ref_keys).any(1)).flatten()
            print(f"[{tag}] iter {it}: torch-sorted keys differ from the oracle's in "
                  f"{rows.numel()} rows, first {rows[:8].tolist()}", flush=True)
            bad += 1
        full = torch.zeros(full_plan.total_out_bytes, dtype=torch.uint8, device=dev)
        amq.build_all_filters(full_plan, amq.KeyBatch.fixed(ref_keys), out=full)
        piece = torch.zeros(full_plan.total_out_bytes, dtype=torch.uint8, device=dev)
        ws.fill_(0xFF)
        for b, e, p in rounds:
            amq.build_all_filters(p, amq.KeyBatch.fixed(ref_keys[int(sb[b]):int(sb[e])]),
                                  out=piece[b * stride:e * stride], workspace=ws)
        torch.cuda.synchronize()
        if first is None:
            first = full.clone()
            o = full.cpu().numpy()
            for s in (0, 1, len(counts) // 2, len(counts) - 1):
                st, ref, pl = O.vqf_build(host[int(sb[s]):], counts[s], bpk, cap, src_page_id=s)
                if o[s * stride:s * stride + pl.payload_used].tobytes() != ref[:pl.payload_used].tobytes():
                    print(f"[{tag}] iter 0: leaf {s} differs from the oracle", flush=True)
                    bad += 1
        for name, arr in (("whole-batch build", full), ("round builds on a 0xFF workspace", piece)):
            if not torch.equal(arr, first):
                d = torch.nonzero(arr != first).flatten()
                leaves = sorted({int(x) // stride for x in d[:100000].tolist()})
                print(f"[{tag}] iter {it}: {name} differs from iteration 0 in {d.numel()} bytes, "
                      f"leaves {leaves[:20]}", flush=True)
                bad += 1
        if it % 10 == 0:
            print(f"[{tag}] iter {it} ok so far (bad={bad}, {time.time() - t0:.1f} s)", flush=True)
    print(f"[{tag}] done: {args.iters} iterations, {bad} differences", flush=True)
    return 1 if bad else 0


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=30)
    ap.add_argument("--procs", type=int, default=1)
    ap.add_argument("--keys", type=int, default=4_000_000)
    ap.add_argument("--child", default=None)
    args = ap.parse_args()
    if args.child is not None:
        sys.exit(child(args, args.child))
    ps = [subprocess.Popen([sys.executable, os.path.abspath(__file__), "--iters", str(args.iters),
                            "--keys", str(args.keys), "--child", str(i)]) for i in range(args.procs)]
    rc = 0
    for p in ps:
        rc = rc or p.wait()
    sys.exit(rc)


if __name__ == "__main__":
    main()
