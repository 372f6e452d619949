"""GPU: the build and probe launch entry points are graph-capturable (no allocation, host
copy or synchronisation inside a launch call, include/tkv_amq.h).  Captured into a HIP graph
(torch.cuda.CUDAGraph) and replayed, they write the same bytes as eager calls -- how a caller
amortises launches for small, launch-bound leaf batches."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("kind,bpk,cap,counts", [(0, 10, 0, [16384] * 3 + [999, 0, 5]),
                                                (1, 12, 32704, [16384] * 3 + [999, 0, 5]),
                                                (0, 10, 0, [300_000])])   # monolithic: record path
def test_build_and_probe_replay_in_graph(oracle, amq, kind, bpk, cap, counts):
    import torch
    keys = oracle.gen_keys16(91, 0, sum(counts))
    if kind == 1:
        oracle.sort_segments(keys, np.concatenate([[0], np.cumsum(counts)]).astype(np.uint64))
    kb = amq.KeyBatch.fixed(torch.from_numpy(keys).cuda())
    plan = amq.plan_filters(kind, counts, bpk, payload_capacity=cap)
    eager = amq.build_all_filters(plan, kb).clone()
    out = torch.zeros_like(eager)
    ws = torch.empty(max(plan.workspace_bytes, 1), dtype=torch.uint8, device="cuda")
    qseg = torch.repeat_interleave(torch.arange(len(counts), dtype=torch.int32, device="cuda"),
                                   torch.tensor(counts, device="cuda"))
    res = torch.empty(len(keys), dtype=torch.uint8, device="cuda")
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):  # warm-up on the capture stream (first-call kernel attributes)
        amq.build_all_filters(plan, kb, out=out, workspace=ws, stream=s, check=False)
        amq.probe_filters(plan, out, kb, qseg, out=res, stream=s)
    s.synchronize()
    out.zero_()
    res.zero_()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        amq.build_all_filters(plan, kb, out=out, workspace=ws, stream=s, check=False)
        amq.probe_filters(plan, out, kb, qseg, out=res, stream=s)
    for _ in range(3):
        g.replay()
    torch.cuda.synchronize()
    o, e = out.cpu().numpy(), eager.cpu().numpy()
    for seg in plan.segs:
        a, b = int(seg["out_offset"]), int(seg["payload_bytes"])
        assert np.array_equal(o[a:a + b], e[a:a + b])
    assert bool(res.all()), "false negative after graph replay"
    amq.abi.check(amq.abi.lib().tkv_amq_build_check(kind, amq.filters._ptr(ws), plan.workspace_bytes,
                                                    amq.filters._stream_handle(s)), "build check")
