"""The RCCL (torch.distributed "nccl") branches of turtle_kv_amd.dist, executed on the one-GPU
box before any 8-GPU run: a child process creates a world-size-1 "nccl" group bound to
device 0 and runs

  - allgather_filters on device tensors (dist.all_gather_into_tensor, dist.py nccl branch),
  - ExactHashShardedBloom.route -> exchange (device all_to_all_single of the counts and the
    records) -> range builds -> allgather, and the pipelined HashShardedBloom step (route blocks
    -> part builds -> in-place all_gather_into_tensor of every round), which take the
    collective path whenever a process group exists,
  - the float64 MAX / int32 MIN all-reduces on device tensors that bench.py uses,

and compares each result with the single-process build (and the oracle).  RCCL cannot put
two ranks on one GPU, so world size 1 is the most this box can run; bench.py's multi-rank
logic is covered by the gloo tests."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def child():
    import numpy as np
    import torch
    import torch.distributed as dist
    sys.path.insert(0, ROOT)
    import turtle_kv_amd as amq
    from turtle_kv_amd import dist as tdist
    from oracle import oracle as O

    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", device_id=dev, rank=0, world_size=1)
    assert dist.get_backend() == "nccl"
    res = {}

    # 1. leaf-sharded build + all_gather_into_tensor on the device
    counts = [16384] * 7 + [5000]
    for kind, bpk, cap in ((0, 10, 0), (1, 12, 32704)):
        stride = tdist.leaf_stride(kind, bpk, max(counts), cap)
        sh = tdist.shard_leaves(counts, 1, 0)
        plan = tdist.plan_shard(kind, counts, bpk, sh, stride, payload_capacity=cap)
        keys = amq.gen_keys16(42, 0, sum(counts))
        if kind == 1:
            from bench import sort_segments_device
            keys = sort_segments_device(torch, keys, counts)
        out = torch.zeros(plan.total_out_bytes, dtype=torch.uint8, device=dev)
        amq.build_all_filters(plan, amq.KeyBatch.fixed(keys), out=out)
        g = tdist.allgather_filters(out)
        torch.cuda.synchronize()
        res[f"allgather_kind{kind}"] = bool(g.is_cuda and torch.equal(g, out))

    # 2. hash-range sharding through route -> all_to_all_single -> range build -> all-gather
    n = 1_500_000
    keys = amq.gen_keys16(7, 0, n)
    ex = tdist.ExactHashShardedBloom(n, 12, 1, 0, dev)
    routed, sc = ex.route(keys)
    owned, sub = ex.exchange(routed, sc)
    # one rank: the all-to-all of the 12-byte bit records (k = 8 at 12 bits/key) is a copy
    res["exchange_identity"] = bool(ex.records and owned.shape == (n, 12) and torch.equal(owned, routed)
                                    and tuple(sub.shape) == (1, ex.g) and int(sub.sum()) == n)
    res["exact_equal_one_gpu"] = bool(torch.equal(ex.build(keys), amq.build_all_filters(
        amq.plan_filters(0, [n], 12), amq.KeyBatch.fixed(keys))[:ex.payload_bytes]))
    # the pipelined step: route blocks -> part builds -> in-place all_gather_into_tensor per round
    hs = tdist.HashShardedBloom(n, 12, 1, 0, dev, chunks=2)
    filt = hs.build(keys)
    torch.cuda.synchronize()
    whole = amq.build_all_filters(amq.plan_filters(0, [n], 12), amq.KeyBatch.fixed(keys))
    res["hash_sharded_equal_one_gpu"] = bool(torch.equal(filt, whole[:filt.numel()]))
    O.build_oracle()
    st, ref = O.bloom_build(keys.cpu().numpy(), n, 12, src_page_id=0)
    res["hash_sharded_equal_oracle"] = bool(st == 0 and filt.cpu().numpy().tobytes() == ref.tobytes())

    # 3. the bench's device all-reduces
    t = torch.tensor([1.25], dtype=torch.float64, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    f = torch.tensor([1], dtype=torch.int32, device=dev)
    dist.all_reduce(f, op=dist.ReduceOp.MIN)
    res["allreduce"] = bool(float(t.item()) == 1.25 and int(f.item()) == 1)
    dist.barrier()
    dist.destroy_process_group()
    print("RESULT " + json.dumps(res), flush=True)


def test_rccl_paths_world1():
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK"):
        env.pop(k, None)
    r = subprocess.run([sys.executable, os.path.abspath(__file__)], capture_output=True, text=True,
                       timeout=300, env=env, cwd=ROOT)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    line = [ln for ln in r.stdout.splitlines() if ln.startswith("RESULT ")]
    assert line, r.stdout[-2000:]
    res = json.loads(line[-1][len("RESULT "):])
    assert all(res.values()), res


if __name__ == "__main__":
    child()
