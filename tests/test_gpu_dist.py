"""GPU, world_size 2 on one device (gloo, host-staged all-gather): each rank builds its leaf
range with the HIP kernels into a fixed-stride slice; the gathered array must equal a
single-process GPU build and the oracle."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def worker(rank, world, port, kind, q):
    import sys
    sys.path.insert(0, ROOT)
    import turtle_kv_amd as amq
    from turtle_kv_amd import dist as tdist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.cuda.set_device(0)
    counts = [16384] * 7 + [5000]
    bpk, cap = (10, 0) if kind == 0 else (12, 32704)
    stride = tdist.leaf_stride(kind, bpk, max(counts), cap)
    sh = tdist.shard_leaves(counts, world, rank)
    plan = tdist.plan_shard(kind, counts, bpk, sh, stride, payload_capacity=cap)
    keys = amq.gen_keys16(42, sh.key_begin, sh.key_end - sh.key_begin)
    if kind == 1:
        from bench import sort_segments_device
        keys = sort_segments_device(torch, keys, counts[sh.leaf_begin:sh.leaf_end])
    out = torch.zeros(plan.total_out_bytes, dtype=torch.uint8, device="cuda")
    amq.build_all_filters(plan, amq.KeyBatch.fixed(keys), out=out)
    g = tdist.allgather_filters(out)
    if rank == 0:
        full_plan = amq.plan_filters(kind, counts, bpk, payload_capacity=cap, out_stride=stride)
        allk = amq.gen_keys16(42, 0, sum(counts))
        if kind == 1:
            from bench import sort_segments_device
            allk = sort_segments_device(torch, allk, counts)
        full = torch.zeros(sh.leaves_per_rank * world * stride, dtype=torch.uint8, device="cuda")
        amq.build_all_filters(full_plan, amq.KeyBatch.fixed(allk), out=full[:full_plan.total_out_bytes])
        q.put(bool(torch.equal(g, full)))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("kind", [0, 1])
def test_sharded_build_allgather_on_gpu(kind):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    ps = [ctx.Process(target=worker, args=(r, 2, port, kind, q)) for r in range(2)]
    for p in ps:
        p.start()
    for p in ps:
        p.join(300)
    assert all(p.exitcode == 0 for p in ps), [p.exitcode for p in ps]
    assert q.get(timeout=5) is True
