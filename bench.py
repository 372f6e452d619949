"""Filter-build benchmark (BASELINE.json metric: filter-build Mkeys/s, device-resident,
16-byte keys @ 10 bits/key, bit-exact).

  python bench.py [--gpus N] [--steps K] [--warmup W]
                  [--workload bloom10|bloom12|vqf12|probe10|probe_vqf12|bloom10k24|vqf12k24|
                              bloom10var|vqf12var|bloom12big|bloom10mono|bloom10monok24|bloom12hash]
                  [--total-keys T]

One step = one pass of the hot path over one batch: build every leaf filter of
`--keys-per-gpu` (default 100M, BASELINE config 2) 16-byte keys held in HBM, S = 16,384 keys
per leaf (6,103 full leaves + 8,448), into one device filter array.  Multi-GPU: one process
per GPU (torch.distributed, RCCL); each rank builds its own contiguous range of leaves (weak
scaling, no data-path collective).  `--gpus N` without a launcher starts the N rank
processes itself (before anything touches a GPU); under torch.distributed.run the world size
must equal --gpus.  The RCCL all-gather of the filter array (north star) is timed separately
after the timed region and reported as `allgather_ms` (`--allgather` puts it inside the
timed step instead); rank 0 then checks the gathered array against a single-process build.

After the timed region every rank byte-compares ALL of its leaves with the CPU oracle built
from independently generated keys ("verified"; "verify": leaves_checked == of_leaves); probe
workloads compare all 200M answers with the oracle's ("fpr_oracle"); the hash-range sharded
filter (config 5) is compared whole with a multithreaded oracle build of all keys.

The printed JSON line carries `roofline` (dominant kernel, HIP events on the build stream,
algorithmic bytes), `valu_roofline` (the bound the build kernels sit on: PMC VALU instructions
per key against the measured integer VALU issue rate, profiles/traffic_<workload>.json) and
`cpu_baseline` (the C oracle -- a restatement of the reference's CPU path, -O3 -march=native
-mbmi2 -mavx2 on this host -- timed on this host's cores by rank 0 after the other ranks have
exited).  Every rank also runs the end-to-end leg (pinned host keys in, filter pages back to
pinned host memory over its own PCIe link) at the same time: `e2e_pcie_inclusive`.
"""
from __future__ import annotations

import argparse
import json
import os
import socket
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

SEG_KEYS = 16384
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s peak (spec)
FABRIC_LINES_G_PER_S = 61.7  # MI355X_MICROARCH.md: random rows of a 151 MB table, 7.9 TB/s / 128 B

WORKLOADS = {
    # name: (kind, bits_per_key, metric label); VQF payload capacity comes from TreeOptions
    "bloom10": (0, 10, "Bloom @10 bits/key"),
    "bloom12": (0, 12, "Bloom @12 bits/key"),
    "vqf12": (1, 12, "VQF @12 bits/key (reference clamp of 10 -> 12)"),
    "probe10": (0, 10, "Bloom @10 probe, 50% hits"),
    "probe_vqf12": (1, 12, "VQF @12 probe, 50% hits"),
    "bloom10k24": (0, 10, "Bloom @10 bits/key, 24-byte keys (TurtleKV default key size)"),
    "vqf12k24": (1, 12, "VQF @12 bits/key, 24-byte keys (TurtleKV default key size) in generation order"),
    "bloom10mono": (0, 10, "Bloom @10 bits/key, one monolithic filter per GPU"),
    "bloom10monok24": (0, 10, "Bloom @10 bits/key, 24-byte keys, one monolithic filter per GPU"),
    "bloom10var": (0, 10, "Bloom @10 bits/key, variable-length keys (8-31 B)"),
    "bloom12hash": (0, 12, "Bloom @12 bits/key, one filter over all GPUs' keys, hash-range sharded"),
    "vqf12var": (1, 12, "VQF @12 bits/key, variable-length keys (8-31 B) in generation order"),
    "bloom12big": (0, 12, "Bloom @12 bits/key, 200K-key leaves (images past one CU's LDS: the window path)"),
}
# BASELINE config 5 read literally: one monolithic filter whose bitmap byte ranges are owned by
# the ranks (route -> RCCL all-to-all of the keys -> range build; turtle_kv_amd.dist)
HASH_SHARDED = {"bloom12hash"}
# workloads whose one filter spans every key of the GPU (the monolithic
# single-filter Bloom variant)
MONOLITHIC = {"bloom10mono", "bloom10monok24"}
KEY_BYTES = {"bloom10k24": 24, "vqf12k24": 24, "bloom10var": 0, "vqf12var": 0, "bloom10monok24": 24}  # 0: variable length
LEAF_KEYS = {"bloom12big": 200_000}  # default keys per leaf where it is not SEG_KEYS
SWEEP_LEAVES = (64, 256, 1024)                   # + the whole batch


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--workload", default="bloom10", choices=sorted(WORKLOADS))
    ap.add_argument("--keys-per-gpu", type=int, default=100_000_000)
    ap.add_argument("--leaf-keys", type=int, default=None,
                    help=f"keys per leaf filter (default {SEG_KEYS}; monolithic workloads: all "
                         "keys of the GPU)")
    ap.add_argument("--total-keys", type=int, default=None,
                    help="strong scaling: one checkpoint of this many keys split over the "
                         "ranks by leaf range (BASELINE config 5: --workload bloom12 "
                         "--total-keys 1000000000)")
    ap.add_argument("--allgather", action="store_true", help="time the RCCL all-gather in-step")
    ap.add_argument("--no-step-allgather", action="store_true",
                    help="bloom12hash: time the all-gather of the filter's rounds after the "
                         "step instead of pipelined inside it")
    ap.add_argument("--chunks", type=int, default=1,
                    help="with a process group: build each rank's leaves in this many rounds of "
                         "block-cyclic leaf chunks and all-gather round c on a communication "
                         "stream while round c+1 builds (the gather inside the timed step; "
                         "turtle_kv_amd.dist.PipelinedLeafGather)")
    ap.add_argument("--pipeline-rounds", type=int, default=4,
                    help="N > 1 leaf lines: rounds per rank of the pipelined build + all-gather "
                         "figure (build_plus_allgather_pipelined)")
    ap.add_argument("--backend", default="nccl", choices=["nccl", "gloo"],
                    help="process-group backend for N > 1 (nccl = RCCL; gloo only to rehearse "
                         "the multi-rank logic on one GPU)")
    ap.add_argument("--ramp-ms", type=float, default=500.0,
                    help="untimed clock ramp before the warmup steps: repeat the step for at "
                         "least this long (the GPU needs ~0.1-0.3 s of load to reach its "
                         "steady clock; 0 disables)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-e2e", action="store_true")
    ap.add_argument("--no-verify", action="store_true",
                    help="skip the post-timing oracle comparison (kernel experiments only)")
    ap.add_argument("--sweep", action="store_true",
                    help="also time the build over the first 64 / 256 / 1024 leaves (batch-size "
                         "curve; off by default so that a kernel-trace profile of the default "
                         "command averages the timed launches only)")
    ap.add_argument("--experiment-lib", action="store_true",
                    help="allow TKV_AMQ_LIB (an experiment build of the library) for kernel A/B "
                         "timing")
    ap.add_argument("--cpu-threads", type=int, default=0,
                    help="CPU baseline threads (0: every core this process may use)")
    return ap.parse_args()


# ---------------------------------------------------------------------------------------
# --gpus N without a launcher: start the ranks (this process never touches a GPU)
# ---------------------------------------------------------------------------------------
def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def launch_ranks(n: int) -> int:
    """One child process per rank, as torch.distributed.run would start them; rank 0's
    stdout carries the JSON line.  Returns the first non-zero exit code, else 0."""
    # build the library once here (hipcc only, no GPU), not in N ranks at once
    from turtle_kv_amd import _build
    _build.build()
    port = _free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n),
                   LOCAL_WORLD_SIZE=str(n), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__), *sys.argv[1:]],
                                      env=env))
    rc = 0
    pending = list(procs)
    while pending:
        for p in list(pending):
            code = p.poll()
            if code is None:
                continue
            pending.remove(p)
            if code != 0 and rc == 0:
                rc = code
                for q in pending:  # a failed rank leaves the others waiting in a collective
                    q.terminate()
        time.sleep(0.05)
    return rc


# ---------------------------------------------------------------------------------------
# host CPU share (the CPU baseline's core count)
# ---------------------------------------------------------------------------------------
def host_cpu_share():
    """CPUs this process may use: the affinity mask, capped by a cgroup CPU quota if one is
    set (the GPU box runs each job with a 16-CPU quota on a 256-thread host)."""
    aff = len(os.sched_getaffinity(0))
    quota = None
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()
        if q != "max":
            quota = int(q) / int(per)
    except (OSError, ValueError):
        pass
    cores = aff if quota is None else max(1, min(aff, int(quota)))
    return cores, {"affinity_cpus": aff, "cgroup_cpu_quota": quota,
                   "host_cpus": os.cpu_count()}


def segment_counts(n_keys, leaf_keys=SEG_KEYS):
    full, rem = divmod(n_keys, leaf_keys)
    return [leaf_keys] * full + ([rem] if rem else [])


def _oracle_libs():
    """(native-march oracle or None, portable oracle) -- loaded only for the baseline leg"""
    from oracle import oracle as O
    O.build_oracle()
    return O, O.native_lib(), O.lib()


def cpu_baseline(kind, bpk, cap, keys_host, counts, threads, leaf_keys=SEG_KEYS):
    """The C oracle (one filter per thread at a time, leaves spread over `threads` workers
    like TreeSerializeContext::build_all_pages) over the same keys, bounded to ~10 s."""
    O, native, portable = _oracle_libs()
    n_segs = len(counts)
    cores, share = host_cpu_share()

    def run(L, ns, nthr):
        c = counts[:ns]
        sb = np.concatenate([[0], np.cumsum(c)]).astype(np.uint64)
        if kind == 0:
            sizes = np.array([O.lib().tkvo_bloom_payload_size(int(x), bpk) for x in c], np.uint64)
        else:
            sizes = np.full(ns, cap, np.uint64)
        offs = np.concatenate([[0], np.cumsum(sizes)[:-1]]).astype(np.uint64)
        out = np.empty(int(sizes.sum()), np.uint8)
        t0 = time.perf_counter()
        st, _ = O.build_segments(kind, keys_host, sb, bpk, offs, sizes, 0, n_threads=nthr,
                                 out=out, L=L, baseline=kind == 1)
        dt = time.perf_counter() - t0
        assert st == 0, st
        return int(sb[-1]), dt

    def timed(L, nthr):
        probe_segs = min(n_segs, 4 * nthr)
        n0, t0 = run(L, probe_segs, nthr)
        rate = n0 / max(t0, 1e-9)
        target = min(int(sum(counts)), int(rate * 8.0))
        ns = n_segs if target >= sum(counts) else max(probe_segs, target // leaf_keys)
        nk, dt = (n0, t0) if ns == probe_segs else run(L, ns, nthr)
        return ns, nk, dt

    L = native or portable
    ns, nk, dt = timed(L, threads)
    used = min(threads, ns)  # one filter per thread at a time
    res = {"value": round(nk / dt / 1e6, 2), "unit": "Mkeys/s", "cores": used,
           "kind": "port",
           "sample": f"{ns} leaves x {leaf_keys} keys ({nk} keys) of the same workload, "
                     + ("BMI2 VQF build (oracle/tkv_amq_baseline.c: pdep/tzcnt select, POPCNT, "
                        "unrolled XXH64; byte-equal to the oracle) " if kind == 1 else "C oracle ")
                     + f"(oracle/tkv_amq_oracle.c, "
                     f"{'-O3 -march=native -mbmi2 -mavx2' if native else '-O3 -march=x86-64-v3 (native build failed)'}), "
                     f"{used} threads, {dt:.2f} s wall",
           "host": share,
           "per_core_mkeys_s": round(nk / dt / 1e6 / used, 2)}
    if native:
        ns2, nk2, dt2 = timed(portable, threads)
        res["portable_x86_64_v3"] = {"value": round(nk2 / dt2 / 1e6, 2), "threads": min(threads, ns2)}
    return res


# ---------------------------------------------------------------------------------------
# main
# ---------------------------------------------------------------------------------------
def main():
    args = parse()
    if os.environ.get("TKV_AMQ_LIB") and not args.experiment_lib:
        raise SystemExit("bench.py: TKV_AMQ_LIB names an experiment library; pass "
                         "--experiment-lib to time it (its line is not the shipped library's)")
    if args.experiment_lib:
        os.environ["TKV_AMQ_EXPERIMENT"] = "1"
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch_ranks(args.gpus))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world != args.gpus:
        raise SystemExit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}; launch with "
                         f"torch.distributed.run --nproc-per-node {args.gpus}, or without a "
                         "launcher (bench.py starts the ranks itself)")
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))

    import torch
    import torch.distributed as dist

    import turtle_kv_amd as amq

    n_dev = torch.cuda.device_count()
    if world > 1 and args.backend == "nccl" and world > n_dev:
        raise SystemExit(f"bench.py: {world} ranks over RCCL need {world} GPUs, {n_dev} visible "
                         "(--backend gloo rehearses the multi-rank logic with shared devices)")
    # one process per GPU (gloo rehearsals with more ranks than GPUs share devices round-robin)
    local = local % max(1, n_dev)
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    # a process group whenever ranks exist: N > 1, or one rank under a launcher
    # (torch.distributed.run --nproc-per-node 1: the RCCL code path at world size 1)
    pg = world > 1 or "LOCAL_RANK" in os.environ
    if pg:
        if args.backend == "nccl":
            # the communicator is bound to this rank's device (RCCL over xGMI)
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(args.backend)
    kind, bpk, label = WORKLOADS[args.workload]
    if args.workload in HASH_SHARDED:
        return bench_hash_sharded(args, torch, dist, amq, world, rank, dev, bpk, label, pg)
    if args.chunks > 1:
        return bench_pipelined_gather(args, torch, dist, amq, world, rank, dev, kind, bpk, label,
                                      pg)
    # the VQF payload capacity is the default TreeOptions' filter page at this bits/key
    # (tree/tree_options.hpp:177-220): 32 KiB pages, 32,704 payload bytes at 12 bits/key
    cap = (amq.TreeOptions(kind).set_filter_bits_per_key(bpk).filter_page_payload_size()
           if kind == amq.VQF else 0)
    from turtle_kv_amd import dist as tdist

    t_start = time.perf_counter()

    def progress(msg):  # multi-rank runs report their stages on stderr (rank 0)
        if world > 1 and rank == 0:
            print(f"bench.py {args.workload} x{world} +{time.perf_counter() - t_start:.1f}s: {msg}",
                  file=sys.stderr, flush=True)

    strong = args.total_keys is not None
    leaf_keys = args.leaf_keys or LEAF_KEYS.get(args.workload, SEG_KEYS)
    if args.workload in MONOLITHIC and args.leaf_keys is None:
        leaf_keys = args.total_keys // world if strong else args.keys_per_gpu
    if strong:
        # strong scaling: one checkpoint of --total-keys keys; rank r builds its leaf range
        all_counts = segment_counts(args.total_keys, leaf_keys)
    else:
        # weak scaling: the checkpoint has `world` x (this GPU's leaves)
        all_counts = segment_counts(args.keys_per_gpu, leaf_keys) * world
    # rank r builds the contiguous leaf range turtle_kv_amd.dist.shard_leaves gives it, at a
    # fixed per-leaf stride so leaf s sits at s * stride in the all-gathered array
    shard = tdist.shard_leaves(all_counts, world, rank)
    stride = tdist.leaf_stride(kind, bpk, max(all_counts), cap)
    plan = tdist.plan_shard(kind, all_counts, bpk, shard, stride, payload_capacity=cap)
    counts = all_counts[shard.leaf_begin:shard.leaf_end]
    n = shard.key_end - shard.key_begin
    total_keys = sum(all_counts)
    key_bytes = KEY_BYTES.get(args.workload, 16)
    offsets = None
    if key_bytes == 16:
        keys = amq.gen_keys16(42, shard.key_begin, n, device=dev)
    elif key_bytes == 0:
        # variable-length keys (the reference's KeyView ranges): lengths uniform in [8, 32)
        g = torch.Generator(device=dev)
        g.manual_seed(42 + rank)
        var_lens = torch.randint(8, 32, (n,), dtype=torch.int64, device=dev, generator=g)
        offsets = torch.zeros(n + 1, dtype=torch.int64, device=dev)
        torch.cumsum(var_lens, 0, out=offsets[1:])
        keys = torch.randint(0, 256, (int(offsets[-1].item()),), dtype=torch.uint8, device=dev,
                             generator=g)
        del var_lens
    else:
        g = torch.Generator(device=dev)
        g.manual_seed(42 + rank)
        keys = torch.randint(0, 256, (n, key_bytes), dtype=torch.uint8, device=dev, generator=g)
    if kind == 1 and key_bytes == 16:
        # VQF inserts in leaf key order: sort each leaf's keys (memcmp order) on the device
        # (other key shapes are inserted in generation order: the same work, and the oracle
        # check below inserts them in the same order)
        progress("keys generated; sorting each leaf")
        keys = one_rank_at_a_time(torch, dist, world, rank,
                                  lambda: sort_segments_device(torch, keys, counts))
    kb = amq.KeyBatch.variable(keys, offsets) if offsets is not None else amq.KeyBatch.fixed(keys)
    progress(f"{n} keys per rank generated")
    # zeroed once: the build never writes past a leaf's payload, so the slack bytes of every
    # fixed-stride slot stay 0 and the gathered array is comparable byte for byte
    out = torch.zeros(plan.total_out_bytes, dtype=torch.uint8, device=dev)
    ws = torch.empty(max(plan.workspace_bytes, 1), dtype=torch.uint8, device=dev)
    gathered = (torch.empty(plan.total_out_bytes * world, dtype=torch.uint8, device=dev)
                if pg else None)

    probe = args.workload.startswith("probe")
    if probe:
        amq.build_all_filters(plan, kb, out=out, workspace=ws)
        q, qseg, is_hit = make_probe_queries(torch, amq, n, counts, dev, shard.key_begin)
        qb = amq.KeyBatch.fixed(q)
        res = torch.empty(q.shape[0], dtype=torch.uint8, device=dev)

    stream = torch.cuda.current_stream()

    def step():
        if probe:
            amq.probe_filters(plan, out, qb, qseg, out=res)
        else:
            amq.build_all_filters(plan, kb, out=out, workspace=ws, check=False)
        if args.allgather and pg:
            tdist.allgather_filters(out, gathered)

    # clock ramp (untimed): a 1 ms step from an idle GPU runs ~15% below the steady clock
    ramp0 = time.perf_counter()
    n_ramp = 0
    while (time.perf_counter() - ramp0) * 1e3 < args.ramp_ms:
        for _ in range(8):
            step()
        n_ramp += 8
        torch.cuda.synchronize()
    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    if not probe and kind == 1:
        amq.abi.check(amq.abi.lib().tkv_amq_build_check(kind, amq.filters._ptr(ws),
                                                        ws.numel(),
                                                        amq.filters._stream_handle()), "vqf build")

    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
          for _ in range(args.steps)]
    coll_dev = dev if args.backend == "nccl" else "cpu"
    if pg:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(args.steps):
        ev[i][0].record(stream)
        step()
        ev[i][1].record(stream)
    torch.cuda.synchronize()
    if pg:
        dist.barrier()
    wall = time.perf_counter() - t0
    if pg:
        wall = reduce_max(torch, dist, wall, coll_dev)
    kernel_ms = float(np.mean([a.elapsed_time(b) for a, b in ev]))
    progress(f"{args.steps} timed steps: {wall / args.steps * 1e3:.3f} ms per step; verifying")

    units = 2 * total_keys if probe else total_keys
    ms_per_step = wall / args.steps * 1e3
    value = units * args.steps / wall / 1e6

    # ---- the timed output, checked (untimed) ----
    verified = None
    probe_check = None
    if not args.no_verify:
        if probe:
            probe_check = verify_probe(torch, kind, plan, out, q, qseg, is_hit, res,
                                       baseline=(rank == 0 and world == 1
                                                 and not args.no_cpu_baseline))
            ok = True
        else:
            verified = verify_all_leaves(torch, kind, bpk, cap, plan, keys, offsets, out,
                                         key_bytes, shard, host_cpu_share()[0])
            ok = verified["ok"]
        if pg:
            flag = torch.tensor([1 if ok else 0], dtype=torch.int32, device=coll_dev)
            dist.all_reduce(flag, op=dist.ReduceOp.MIN)
            ok = bool(flag.item())
            if verified is not None:
                verified["all_ranks_ok"] = ok
        if not ok:
            raise SystemExit(f"bench.py: timed output differs from the oracle: {verified}")

    # algorithmic bytes per launch: build = 16 B/key in + filter payload out;
    # probe = 16 B key + 4 B leaf id + 1 B result per lookup
    fpr = None
    if probe:
        alg_bytes = q.shape[0] * (16 + 4 + 1)
        hit_res = res[is_hit]
        if not bool(hit_res.all()):
            bad = torch.nonzero(hit_res == 0).flatten()
            raise SystemExit(f"false negatives in the probe: {bad.numel()} of {hit_res.numel()} "
                             f"hits, first indices {bad[:8].tolist()}")
        fpr = float(res[~is_hit].float().mean())
    else:
        key_in = n * key_bytes if offsets is None else keys.numel() + 8 * (n + 1)
        alg_bytes = key_in + int(plan.segs["payload_bytes"].astype(np.int64).sum())
    achieved = alg_bytes / (kernel_ms * 1e-3) / 1e9
    prof = load_profile(args.workload)
    traffic = prof.get("hbm_bytes_per_launch")
    valu_roof = valu_roofline(prof, n, kernel_ms) if not probe else None

    fabric_roof = None
    if probe and prof.get("TCC_EA0_RDREQ_per_launch"):
        # the bound a random-gather probe sits on: L2 -> fabric read requests (one 128-B line
        # each) per second, against the random-row gather rate MI355X_MICROARCH.md measures
        # for a 151 MB table (7.4-7.9 TB/s = 58-62 G lines/s)
        req = prof["TCC_EA0_RDREQ_per_launch"] / (kernel_ms * 1e-3) / 1e9
        fabric_roof = {"achieved": round(req, 2), "peak": FABRIC_LINES_G_PER_S,
                       "unit": "G fabric read requests/s", "frac": round(req / FABRIC_LINES_G_PER_S, 4),
                       "requests_per_lookup": prof.get("ea_read_requests_per_unit"),
                       "note": "PMC TCC_EA0_RDREQ per launch (profiles/traffic_*.json); peak = "
                               "7.9 TB/s / 128 B, the guide's random-row gather rate"}

    allgather_ms = None
    gather_ok = None
    if pg:
        progress("verified; timing the all-gather")
        if not args.allgather:
            torch.cuda.synchronize()
            dist.barrier()
            g0 = time.perf_counter()
            for _ in range(3):
                tdist.allgather_filters(out, gathered)
            torch.cuda.synchronize()
            allgather_ms = reduce_max(torch, dist, (time.perf_counter() - g0) / 3 * 1e3, coll_dev)
        else:
            tdist.allgather_filters(out, gathered)
        if rank == 0 and not args.no_verify and not probe:
            progress("checking the gathered array against a one-process build")
            gather_ok = verify_gather(torch, amq, kind, bpk, cap, all_counts, stride, gathered,
                                      key_bytes, dev)
        if world > n_dev:
            dist.barrier()  # (ranks sharing rank 0's device wait for its check and sort)
        progress("all-gather done; the pipelined figure")

    # the north star's whole step with the all-gather overlapped (untimed by `value`): the same
    # leaves dealt in block-cyclic rounds, round c gathered on a communication stream while
    # round c + 1 builds (turtle_kv_amd.dist.PipelinedLeafGather; bench --chunks K times it alone)
    pipelined = None
    if (pg and world > 1 and not probe and key_bytes == 16 and args.workload not in MONOLITHIC
            and not args.allgather):
        del gathered
        torch.cuda.empty_cache()
        try:
            pipelined = pipelined_figure(torch, dist, amq, tdist, kind, bpk, cap, all_counts,
                                         world, rank, stride, dev, coll_dev, args.pipeline_rounds)
        except Exception as e:  # an extra figure: it must not cost the timed line
            pipelined = {"error": f"{type(e).__name__}: {e}"[:400]}
            torch.cuda.synchronize()
            dist.barrier()

    progress("pipelined figure done; host legs")
    sweep = None
    if rank == 0 and world == 1 and not probe and args.sweep and \
            args.workload not in MONOLITHIC and len(counts) > SWEEP_LEAVES[0]:
        sweep = batch_sweep(torch, amq, kind, bpk, cap, counts, kb, ws, plan, kernel_ms)

    # the north star's host leg on EVERY rank at once: each GPU's pages go back to host page
    # memory over its own PCIe link (tree/tree_serialize_context.cpp:62-115); the aggregate is
    # all ranks' keys over the slowest rank's time
    e2e = None
    if (not args.no_e2e and not probe and key_bytes == 16 and n <= 200_000_000
            and args.workload not in MONOLITHIC):
        sync = (lambda: dist.barrier()) if pg else (lambda: None)
        red = (lambda x: reduce_max(torch, dist, x, coll_dev)) if pg else (lambda x: x)
        e2e = end_to_end(torch, amq, kind, bpk, cap, counts, keys, sync=sync, reduce_max=red,
                         total_keys=total_keys, world=world)

    comm = comm_info(torch, dist, dev) if pg else None
    if pg:
        dist.barrier()
    if rank != 0:
        dist.destroy_process_group()
        return
    if pg:
        # every other rank has left its last collective: the CPU baseline below runs on a host
        # whose other ranks are gone (no rank spinning in a barrier beside it)
        dist.destroy_process_group()

    base = None
    cores, _ = host_cpu_share()
    threads = args.cpu_threads or cores
    if not args.no_cpu_baseline:
        if probe:
            base = probe_check.get("cpu_baseline") if probe_check else None
        elif key_bytes == 16:
            # the CPU sample is bounded (~8 s); copy at most the first 100M keys to the host
            lim = max(1, 100_000_000 // leaf_keys)
            nk_host = sum(counts[:lim]) if n > 100_000_000 else n
            base = cpu_baseline(kind, bpk, cap, keys[:nk_host].cpu().numpy(),
                                counts[:lim] if n > 100_000_000 else counts,
                                threads, leaf_keys)
            if world > 1:
                base["note"] = (f"rank 0's keys (the same leaves every rank builds), timed on rank "
                                f"0's host after the other {world - 1} ranks exited")

    kdesc = f"{key_bytes}B" if key_bytes else "8-31B (mean %.1f B)" % (keys.numel() / max(n, 1))
    line = {
        "metric": f"filter-build Mkeys/s (device-resident), 16B keys @10 bits/key; bit-exact"
        if args.workload == "bloom10" else f"{label} Mkeys/s (device-resident)",
        "value": round(value, 2),
        "unit": "Mkeys/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ramp_steps": n_ramp,
        "ms_per_step": round(ms_per_step, 4),
        "higher_is_better": True,
        "scaling": "strong" if strong else "weak",
        "vs_baseline": None,
        "dtype": "u64",
        "data": "synthetic (splitmix64 seed 42 keys generated on the device)",
        "config": {"workload": (f"{label}: {total_keys} x {kdesc} keys over {world} GPU(s)"
                                if strong else f"{label}: {n} x {kdesc} keys per GPU")
                               + f", {leaf_keys}-key leaves ({len(counts)} filters on rank 0)",
                   "keys_per_gpu": n, "total_keys": total_keys, "key_bytes": key_bytes,
                   "leaf_keys": leaf_keys, "bits_per_key": bpk,
                   "filter": "bloom-blocked512" if kind == 0 else "vqf",
                   "payload_capacity": cap or None,
                   "parallelism": f"leaf-sharded x{world}",
                   "backend": args.backend if pg else None},
        "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS,
                     "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4),
                     "traffic": traffic, "kernel_ms": round(kernel_ms, 4),
                     "alg_bytes_per_launch": alg_bytes},
        "cpu_baseline": base,
    }
    if comm is not None:
        line["comm"] = comm
    if verified is not None:
        line["verified"] = verified["ok"] and verified.get("all_ranks_ok", True)
        line["verify"] = verified
    if valu_roof is not None:
        line["valu_roofline"] = valu_roof
    if fabric_roof is not None:
        line["fabric_roofline"] = fabric_roof
    if allgather_ms is not None:
        line["allgather_ms"] = round(allgather_ms, 3)
        line["allgather_bytes_in_per_gpu"] = (world - 1) * plan.total_out_bytes
        line["build_plus_allgather_mkeys_s"] = round(units / ((ms_per_step + allgather_ms) * 1e-3) / 1e6, 2)
    if gather_ok is not None:
        line["gather_verified"] = gather_ok
    if pipelined is not None and "ms_per_step" in pipelined:
        pipelined["mkeys_s"] = round(units / (pipelined["ms_per_step"] * 1e-3) / 1e6, 2)
    if pipelined is not None:
        line["build_plus_allgather_pipelined"] = pipelined
    if sweep is not None:
        line["batch_sweep"] = sweep
    if e2e is not None:
        line["e2e_pcie_inclusive"] = e2e
    if fpr is not None:
        line["probe"] = {"lookups": int(q.shape[0]), "hits_all_true": True,
                         "false_positive_rate": round(fpr, 6)}
        if probe_check is not None:
            line["probe"].update({k: v for k, v in probe_check.items() if k != "cpu_baseline"})
            line["verified"] = probe_check["results_equal_oracle"]
    print(json.dumps(line), flush=True)


def reduce_max(torch, dist, x, device):
    """max over ranks of one float (a tensor on the rank's device for RCCL, host for gloo)"""
    t = torch.tensor([float(x)], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def valu_roofline(prof, n_keys, kernel_ms):
    """The bound a build kernel actually sits on: integer VALU issue,
    from the PMC counters of profiles/traffic_<workload>.json."""
    if not prof.get("valu_instr_per_key"):
        return None
    wave_instr = prof["valu_instr_per_key"] * n_keys / 64
    ach = wave_instr / (kernel_ms * 1e-3) / 1e9
    peak = prof.get("valu_peak_ginstr_s", prof.get("valu_peak_ginstr_s_at_2.4GHz", 614.4))
    r = {"achieved": round(ach, 1), "peak": peak, "unit": "G wave64-VALU-instr/s",
         "frac": round(ach / peak, 4), "instr_per_key": prof["valu_instr_per_key"],
         "note": prof.get("valu_peak_note", "PMC SQ_INSTS_VALU per key (profiles/traffic_*.json); "
                                            "peak = 1024 SIMDs x 2.4 GHz / 4 cycles")}
    if prof.get("valu_busy_frac") is not None:
        r["valu_busy_frac_pmc"] = prof["valu_busy_frac"]
    return r


def pipelined_figure(torch, dist, amq, tdist, kind, bpk, cap, all_counts, world, rank, stride, dev,
                     coll_dev, rounds, reps=5):
    """Max over ranks of the pipelined build + all-gather step time (PipelinedLeafGather,
    `rounds` rounds per rank) after one untimed step.  (bench --chunks K runs the same step as
    its timed step and checks the array it gathers.)"""
    per_rank = -(-len(all_counts) // world)
    q = -(-per_rank // max(1, rounds))
    pl = tdist.PipelinedLeafGather(kind, all_counts, bpk, world, rank, stride, q, dev,
                                   payload_capacity=cap)
    def make_batches():
        bs = []
        for (b, e), (k0, k1) in zip(pl.rounds, pl.key_ranges()):
            if k1 == k0:
                bs.append(None)
                continue
            keys = amq.gen_keys16(42, k0, k1 - k0, device=dev)
            if kind == 1:
                keys = sort_segments_device(torch, keys, all_counts[b:e])
            bs.append(amq.KeyBatch.fixed(keys))
        return bs

    batches = one_rank_at_a_time(torch, dist, world, rank, make_batches)
    pl.step(batches)
    torch.cuda.synchronize()
    dist.barrier()
    t0 = time.perf_counter()
    for _ in range(reps):
        pl.step(batches)
    torch.cuda.synchronize()
    dist.barrier()
    ms = reduce_max(torch, dist, (time.perf_counter() - t0) / reps * 1e3, coll_dev)
    out = {"ms_per_step": round(ms, 4), "rounds": len(pl.rounds), "chunk_leaves": q,
           "reps": reps, "note": "block-cyclic rounds, round c all-gathered on a communication "
                                 "stream while round c+1 builds; every rank ends the step with "
                                 "the whole array (bench --chunks verifies it)"}
    del pl, batches
    torch.cuda.empty_cache()
    return out


# ---------------------------------------------------------------------------------------
# leaf build with the all-gather pipelined into the step (--chunks K)
# ---------------------------------------------------------------------------------------
def bench_pipelined_gather(args, torch, dist, amq, world, rank, dev, kind, bpk, label, pg):
    """The north star's multi-GPU step with the all-gather inside it: the checkpoint's leaves
    are dealt to the ranks in block-cyclic chunks of Q leaves (round c of rank r = leaves
    [(c*W + r)*Q, (c*W + r + 1)*Q)), each rank builds its K rounds one after the other on the
    compute stream and all-gathers round c on a communication stream while round c + 1 builds,
    so every rank ends the step holding the whole leaf-ordered filter array.  The step costs
    about max(build, gather) + one round's gather; `breakdown_ms` times build-only and
    gather-only steps beside it.  Rank 0 checks the gathered array against a one-GPU build of
    every leaf (itself checked against the oracle by the plain leaf line)."""
    from turtle_kv_amd import dist as tdist
    if not pg:
        raise SystemExit("bench.py: --chunks needs a process group (a launcher, or --gpus N > 1)")
    if args.workload.startswith("probe") or args.workload in MONOLITHIC or \
            KEY_BYTES.get(args.workload, 16) != 16:
        raise SystemExit("bench.py: --chunks pipelines the leaf build of 16-byte keys "
                         "(bloom10, bloom12, vqf12, bloom12big)")
    cap = (amq.TreeOptions(kind).set_filter_bits_per_key(bpk).filter_page_payload_size()
           if kind == amq.VQF else 0)
    strong = args.total_keys is not None
    leaf_keys = args.leaf_keys or LEAF_KEYS.get(args.workload, SEG_KEYS)
    all_counts = (segment_counts(args.total_keys, leaf_keys) if strong
                  else segment_counts(args.keys_per_gpu, leaf_keys) * world)
    n_leaves = len(all_counts)
    per_rank = -(-n_leaves // world)
    q = -(-per_rank // args.chunks)
    stride = tdist.leaf_stride(kind, bpk, max(all_counts), cap)
    pl = tdist.PipelinedLeafGather(kind, all_counts, bpk, world, rank, stride, q, dev,
                                   payload_capacity=cap)
    def make_batches():
        bs = []
        for (b, e), (k0, k1) in zip(pl.rounds, pl.key_ranges()):
            if k1 == k0:
                bs.append(None)
                continue
            keys = amq.gen_keys16(42, k0, k1 - k0, device=dev)
            if kind == 1:
                keys = sort_segments_device(torch, keys, all_counts[b:e])
            bs.append(amq.KeyBatch.fixed(keys))
        return bs

    batches = one_rank_at_a_time(torch, dist, world, rank, make_batches)
    n = sum(k1 - k0 for k0, k1 in pl.key_ranges())
    total_keys = sum(all_counts)
    coll_dev = dev if args.backend == "nccl" else "cpu"

    def timed(steps, **kw):
        dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(steps):
            pl.step(batches, **kw)
        torch.cuda.synchronize()
        dist.barrier()
        return reduce_max(torch, dist, time.perf_counter() - t0, coll_dev)

    ramp0 = time.perf_counter()
    n_ramp = 0
    while (time.perf_counter() - ramp0) * 1e3 < args.ramp_ms:
        pl.step(batches)
        n_ramp += 1
        torch.cuda.synchronize()
    for _ in range(args.warmup):
        pl.step(batches)
    torch.cuda.synchronize()
    wall = timed(args.steps)
    ms_per_step = wall / args.steps * 1e3
    reps = max(1, min(5, args.steps))
    build_ms = timed(reps, gather=False) / reps * 1e3
    gather_ms = timed(reps, build=False) / reps * 1e3

    pl.step(batches)  # the checked array: one more full step
    torch.cuda.synchronize()
    gather_ok = None
    if rank == 0 and not args.no_verify:
        gather_ok = verify_gather(torch, amq, kind, bpk, cap, all_counts, stride, pl.filters(), 16,
                                  dev, layout=(world, q), batches=batches)
    flag = torch.tensor([0 if gather_ok is False else 1], dtype=torch.int32, device=coll_dev)
    dist.all_reduce(flag, op=dist.ReduceOp.MIN)
    if not bool(flag.item()):
        raise SystemExit("bench.py: the pipelined all-gather's array differs from a one-GPU build")
    comm = comm_info(torch, dist, dev)
    dist.barrier()
    dist.destroy_process_group()
    if rank != 0:
        return
    line = {
        "metric": f"{label} Mkeys/s incl. all-gather (device-resident)",
        "value": round(total_keys * args.steps / wall / 1e6, 2), "unit": "Mkeys/s",
        "n_gpus": world, "steps": args.steps, "warmup": args.warmup, "ramp_steps": n_ramp,
        "ms_per_step": round(ms_per_step, 4), "higher_is_better": True,
        "scaling": "strong" if strong else "weak", "vs_baseline": None, "dtype": "u64",
        "data": "synthetic (splitmix64 seed 42 keys generated on the device)",
        "config": {"workload": f"{label}: {total_keys} x 16B keys in {n_leaves} {leaf_keys}-key "
                               f"leaves, block-cyclic chunks of {q} leaves, {len(pl.rounds)} "
                               f"rounds per rank, every rank gathers the whole array",
                   "keys_per_gpu": n, "total_keys": total_keys, "key_bytes": 16,
                   "leaf_keys": leaf_keys, "bits_per_key": bpk,
                   "filter": "bloom-blocked512" if kind == 0 else "vqf",
                   "payload_capacity": cap or None, "parallelism": f"leaf-sharded x{world}",
                   "backend": args.backend, "chunk_leaves": q, "rounds": len(pl.rounds)},
        "roofline": None,
        "cpu_baseline": None,
        "breakdown_ms": {"build_only": round(build_ms, 4), "gather_only": round(gather_ms, 4),
                         "pipelined": round(ms_per_step, 4),
                         "sum_of_parts": round(build_ms + gather_ms, 4),
                         "max_of_parts": round(max(build_ms, gather_ms), 4)},
        "allgather_bytes_in_per_gpu": (world - 1) * len(pl.rounds) * pl.round_bytes,
        "gather_verified": gather_ok,
        "comm": comm,
        "note": "roofline and cpu_baseline are the plain leaf line's (same build kernels); this "
                "line measures the gather overlap",
    }
    print(json.dumps(line), flush=True)


# ---------------------------------------------------------------------------------------
# hash-range sharded monolithic Bloom (BASELINE config 5 read literally)
# ---------------------------------------------------------------------------------------
def bench_hash_sharded(args, torch, dist, amq, world, rank, dev, bpk, label, pg=False):
    """One Bloom filter over every rank's keys; rank r owns parts r, r + N, r + 2N, ... of its
    bitmap (turtle_kv_amd.dist.HashShardedBloom).  A step, pipelined over a compute and a
    communication stream: route the rank's keys in K chunks (every key hashed once into its
    12-byte bit record, counting-sorted by part into fixed-capacity blocks) -> all-to-all of
    chunk c's blocks while chunk c + 1 routes (RCCL, equal splits, no host synchronisation) ->
    build each owned part from the blocks received -> all-gather round j (part j of every
    rank, one contiguous range) in place while part j + 1 builds.  With --no-step-allgather the
    gather is timed separately.  Without a process group (one GPU, no launcher) the step is the
    route and the part builds.  Rank 0 checks the whole gathered filter against the CPU oracle
    (every key hashed on every host thread) after the timed region."""
    from turtle_kv_amd import dist as tdist
    strong = args.total_keys is not None
    n_local = args.total_keys // world if strong else args.keys_per_gpu
    total = n_local * world
    chunks = args.chunks if args.chunks > 1 else (4 if world > 1 else 1)
    keys = amq.gen_keys16(42, rank * n_local, n_local, device=dev)
    hs = tdist.HashShardedBloom(total, bpk, world, rank, dev, chunks=chunks)
    gather_in_step = pg and not args.no_step_allgather

    def progress(msg):  # long runs (1B keys) report their stages on stderr
        if rank == 0:
            print(f"bench.py bloom12hash: {msg}", file=sys.stderr, flush=True)

    progress(f"{n_local} keys per rank generated; ramp")

    def step():
        hs.step(keys, gather=gather_in_step)

    ramp0 = time.perf_counter()
    n_ramp = 0
    while (time.perf_counter() - ramp0) * 1e3 < args.ramp_ms:
        step()
        n_ramp += 1
        torch.cuda.synchronize()
    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    progress(f"ramp ({n_ramp} steps) and warmup done")
    coll_dev = dev if args.backend == "nccl" else "cpu"
    if pg:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    if pg:
        dist.barrier()
    wall = time.perf_counter() - t0
    if pg:
        wall = reduce_max(torch, dist, wall, coll_dev)
    progress(f"{args.steps} timed steps: {wall / args.steps * 1e3:.3f} ms per step")
    lost = hs.lost()  # blocks that needed more overflow room than they have (not for hashed keys)

    # untimed breakdown: the stages one after another on rank 0 (HIP events on the current
    # stream; each stage's collectives on the current stream, not overlapped)
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(5)]
    if pg:
        dist.barrier()
    torch.cuda.synchronize()
    ev[0].record()
    if not hs.records:
        hs.step(keys, gather=False)
        ev[1].record()
        ev[2].record()
        ev[3].record()
    else:
        for c in range(hs.chunks):
            hs.route_chunk(keys, c)
        ev[1].record()
        if pg and world > 1:
            for c in range(hs.chunks):
                hs.exchange_chunk(c)
        ev[2].record()
        for j in range(hs.g):
            hs.build_part(j)
        ev[3].record()
    if pg:
        if hs.records:
            for j in range(hs.g):
                hs.gather_round(j)
        else:
            hs.allgather()
    ev[4].record()
    torch.cuda.synchronize()
    route_ms, a2a_ms, build_ms, gather_ms = (ev[i].elapsed_time(ev[i + 1]) for i in range(4))
    # one more pipelined step with an event at every stage boundary: when each chunk's route,
    # each round's exchange, each part build and each round's gather ended on its stream
    timeline = None
    if hs.records:
        if pg:
            dist.barrier()
        hs.step(keys, gather=gather_in_step, timeline=True)
        torch.cuda.synchronize()
        timeline = hs.timeline_ms()

    allgather_ms = None
    if pg and not gather_in_step:
        dist.barrier()
        g0 = time.perf_counter()
        for _ in range(3):
            hs.allgather()
        torch.cuda.synchronize()
        allgather_ms = reduce_max(torch, dist, (time.perf_counter() - g0) / 3 * 1e3, coll_dev)
    filt = hs.filter() if hs.records else hs.allgather()
    torch.cuda.synchronize()
    progress("breakdown and all-gather done; verifying")
    comm = comm_info(torch, dist, dev) if pg else None

    check = None
    if rank == 0 and not args.no_verify:
        check = verify_hash_sharded(torch, amq, filt, total, bpk, dev)
    if pg:
        flag = torch.tensor([1 if (check is None or check["ok"]) and not lost else 0],
                            dtype=torch.int32, device=coll_dev)
        dist.all_reduce(flag, op=dist.ReduceOp.MIN)
        ok = bool(flag.item())
    else:
        ok = (check is None or check["ok"]) and not lost
    if not ok:
        raise SystemExit(f"bench.py: hash-sharded filter differs (or its blocks lost overflow "
                         f"entries: {lost}): {check}")
    if pg:
        dist.barrier()
    if rank != 0:
        dist.destroy_process_group()
        return
    if pg:
        dist.destroy_process_group()
    base = None
    if not args.no_cpu_baseline:
        base = cpu_baseline_monolithic(bpk, min(total, 20_000_000))
    ms_per_step = wall / args.steps * 1e3
    value = total * args.steps / wall / 1e6
    alg = n_local * 16 + (int(hs.payload_bytes) - 64) // world  # keys in, this rank's bitmap out
    if gather_in_step:
        path = f"route ({chunks} chunks) -> all-to-all -> part builds -> all-gather, pipelined"
    elif pg:
        path = f"route ({chunks} chunks) -> all-to-all -> part builds, pipelined"
    elif hs._direct:
        path = "one range build from the keys (one GPU, <= 6,400 tiles: no route)"
    else:
        path = f"route ({chunks} chunk(s)) -> part builds"
    rp = getattr(hs, "rp", None)
    line = {
        "metric": f"{label} Mkeys/s (device-resident)",
        "value": round(value, 2), "unit": "Mkeys/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ramp_steps": n_ramp, "ms_per_step": round(ms_per_step, 4),
        "higher_is_better": True, "scaling": "strong" if strong else "weak", "vs_baseline": None,
        "dtype": "u64", "data": "synthetic (splitmix64 seed 42 keys generated on the device)",
        "config": {"workload": f"{label}: {total} x 16B keys, {n_local} per GPU, one filter of "
                               f"{hs.n_blocks} blocks ({hs.T} tiles) in {world * hs.g} parts of "
                               f"{hs.q} tiles; rank r owns parts r, r + {world}, ...",
                   "keys_per_gpu": n_local, "total_keys": total, "key_bytes": 16,
                   "bits_per_key": bpk, "filter": "bloom-blocked512, monolithic",
                   "parallelism": f"hash-range-sharded x{world}",
                   "backend": args.backend if pg else None, "chunks": chunks,
                   "allgather_in_step": bool(gather_in_step),
                   "path": path, "units": "12-byte bit records" if hs.records else "16-byte keys"},
        "roofline": {"bound": "hbm", "achieved": round(alg / (ms_per_step * 1e-3) / 1e9, 1),
                     "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": round(alg / (ms_per_step * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
                     "traffic": (None if hs._direct else
                                 load_profile(f"bloom12hash{'1B' if total >= 1_000_000_000 else ''}")
                                 .get("hbm_bytes_per_launch")),
                     "alg_bytes_per_launch": alg,
                     "note": "whole step on rank 0; traffic: PMC bytes of the step's kernels"},
        "cpu_baseline": base,
        "step_breakdown_rank0_ms": {"route": round(route_ms, 4), "all_to_all": round(a2a_ms, 4),
                                    "part_builds": round(build_ms, 4),
                                    "allgather": round(gather_ms, 4),
                                    "note": "the routed form's stages one after another (untimed "
                                            "by value" + ("; the timed step is the direct range "
                                                          "build)" if hs._direct else ")")},
        "step_timeline_rank0_ms": timeline,
        "verified": check["ok"] if check else None, "verify": check,
    }
    if rp is not None:
        line["route_plan"] = {"route_wgs": rp.route_wgs, "region_cap": rp.region_cap,
                              "block_bytes": rp.block_bytes, "ovf_cap": rp.ovf_cap,
                              "parts_per_rank": hs.g,
                              "exchanged_bytes_per_rank": (world - 1) * chunks * hs.g * rp.block_bytes,
                              "record_bytes_per_rank": 12 * n_local * (world - 1) // world,
                              "overflow_lost": lost}
    if comm is not None:
        line["comm"] = comm
    if allgather_ms is not None:
        line["allgather_ms"] = round(allgather_ms, 3)
        line["build_plus_allgather_mkeys_s"] = round(total / ((ms_per_step + allgather_ms) * 1e-3) / 1e6, 2)
    print(json.dumps(line), flush=True)


def verify_hash_sharded(torch, amq, filt, total, bpk, dev):
    """The gathered hash-range sharded filter against the CPU oracle, WHOLE: the oracle generates
    all `total` keys, hashes each one and sets its bits in one host bitmap on every host thread
    (oracle.bloom_sample_blocks with the single window [0, block_count); ~10 s for config 5's
    1B keys on 16 threads), and the header is checked field by field."""
    from oracle import oracle as O
    O.build_oracle()
    nb = int(O.lib().tkvo_bloom_block_count(total, bpk))
    cores, _ = host_cpu_share()
    t0 = time.perf_counter()
    st, got = O.bloom_sample_blocks(42, 0, total, bpk, [(0, nb)], n_threads=cores)
    dt = time.perf_counter() - t0
    host = filt.cpu().numpy()
    ref = got[(0, nb)]
    body_ok = st == 0 and host.size == 64 + ref.size and np.array_equal(host[64:], ref)
    k = int(O.lib().tkvo_bloom_hash_count(bpk))
    hdr = np.frombuffer(host[:64].tobytes(), dtype="<u8")
    hdr_ok = (int(hdr[0]) == 0xCA6F49A0F3F8A4B0 and int(hdr[1]) == 512 * nb and int(hdr[2]) == 0
              and int(hdr[3]) == 0 and int(hdr[4]) == 8 * nb
              and int(hdr[5]) == nb | (k << 32) | (2 << 48) and int(hdr[6]) == total)
    check = {"equal_to_oracle": bool(body_ok and hdr_ok), "header_ok": bool(hdr_ok),
             "oracle_whole_filter": {"blocks": nb, "bytes": 64 + 64 * nb, "keys_hashed": total,
                                     "threads": cores, "seconds": round(dt, 2)}}
    if not body_ok and st == 0 and host.size == 64 + ref.size:
        d = np.nonzero(host[64:] != ref)[0]
        check["differing_tiles"] = sorted({int(x) // (64 * 2048) for x in d[:100000]})[:16]
        check["bytes_differing"] = int(d.size)
    check["ok"] = check["equal_to_oracle"]
    return check


def comm_info(torch, dist, dev):
    """The process group as the ranks see it: the communicator's world size and backend and
    every rank's bound device, gathered from the ranks themselves (an N-rank line shows that
    RCCL saw N ranks on N devices)."""
    p = torch.cuda.get_device_properties(dev)
    mine = {"rank": dist.get_rank(), "device": dev.index, "uuid": str(getattr(p, "uuid", "")),
            "pci_bus_id": getattr(p, "pci_bus_id", None), "host": socket.gethostname()}
    everyone = [None] * dist.get_world_size()
    dist.all_gather_object(everyone, mine)
    return {"world_size": dist.get_world_size(), "backend": dist.get_backend(), "ranks": everyone,
            "distinct_devices": len({(e["host"], e["uuid"], e["pci_bus_id"]) for e in everyone})}


def cpu_baseline_monolithic(bpk, n):
    """One Bloom filter over n keys on one host thread: the reference builds each filter on
    one thread (filter_builder.hpp:127, WorkerPool::null_pool()), so a single filter gets one
    core whatever the host has."""
    O, native, portable = _oracle_libs()
    keys = O.gen_keys16(42, 0, n)
    L = native or portable
    t0 = time.perf_counter()
    st, _ = O.bloom_build(keys, n, bpk, src_page_id=0, L=L)
    dt = time.perf_counter() - t0
    assert st == 0, st
    return {"value": round(n / dt / 1e6, 2), "unit": "Mkeys/s", "cores": 1, "kind": "port",
            "sample": f"one {n}-key Bloom filter @{bpk} bits/key, C oracle "
                      f"({'-O3 -march=native -mbmi2 -mavx2' if native else '-O3 -march=x86-64-v3'}),"
                      f" 1 thread (one filter per thread, as the reference), {dt:.2f} s wall"}


# ---------------------------------------------------------------------------------------
# verification of the timed output (untimed, oracle = the checker)
# ---------------------------------------------------------------------------------------
def verify_all_leaves(torch, kind, bpk, cap, plan, keys, offsets, out, key_bytes, shard, threads):
    """Byte-compare EVERY leaf of this rank's timed output with the CPU oracle (SURVEY.md 8(c):
    whole-output parity at the bench's own size).  16-byte keys are regenerated on the host by
    the oracle and, for VQF, sorted there (so the device key generator and the device sort are
    checked too: `keys_equal_oracle`); other key shapes are copied from the device.  The
    oracle builds all leaves on `threads` host threads (tkvo_build_segments_ex) into an array
    laid out like the device's, and the two arrays are compared whole: every payload byte and
    the never-written slack between payloads."""
    from oracle import oracle as O
    O.build_oracle()
    t0 = time.perf_counter()
    segs = plan.segs
    counts = segs["n_keys"].astype(np.uint64)
    sb = np.concatenate([[0], np.cumsum(counts)]).astype(np.uint64)
    n = int(sb[-1])
    res = {"against": ("CPU oracle (oracle/tkv_amq_oracle.c) on oracle-generated keys"
                       if key_bytes == 16 else "CPU oracle on the device keys")}
    offs = None
    if key_bytes == 16:
        kh = O.gen_keys16(42, shard.key_begin, n)
        if kind == 1:
            O.sort_segments(kh, sb, n_threads=threads)
        res["keys_equal_oracle"] = bool(np.array_equal(kh, keys[:n].cpu().numpy()))
        stride = 16
    elif key_bytes == 0:
        kh = keys.cpu().numpy()
        offs = offsets.cpu().numpy().astype(np.uint64)
        stride = 0
    else:
        kh = keys.cpu().numpy()
        stride = key_bytes
    got = out.cpu().numpy()
    caps = (np.full(len(counts), cap, np.uint64) if kind == 1
            else segs["payload_bytes"].astype(np.uint64))
    ref = np.zeros(len(got) + int(cap or 0), np.uint8)
    st = O.build_segments_ex(kind, kh if len(kh) else np.zeros(16, np.uint8), offs, stride, sb, bpk,
                             segs["out_offset"], caps, ref, src_page_id=segs["src_page_id"],
                             n_threads=threads)
    del kh
    bad = []
    if st != 0:
        bad.append(f"oracle status {st}")
    else:
        ref = ref[:len(got)]
        if not np.array_equal(got, ref):
            diff = np.nonzero(got != ref)[0]
            ends = (segs["out_offset"] + segs["payload_bytes"]).astype(np.int64)
            leaves = np.unique(np.searchsorted(ends, diff[:1_000_000], side="right"))
            bad = [int(x) for x in leaves[:16]]
            res["bytes_differing"] = int(diff.size)
    res.update({"ok": not bad and res.get("keys_equal_oracle", True),
                "leaves_checked": int(len(counts)), "of_leaves": int(len(counts)), "keys": n,
                "mismatched_leaves": bad, "threads": threads,
                "seconds": round(time.perf_counter() - t0, 2)})
    return res


def verify_gather(torch, amq, kind, bpk, cap, all_counts, stride, gathered, key_bytes, dev,
                  layout=None, batches=None):
    """Rank 0: the all-gathered array equals a single-process build of every leaf at the same
    stride (16-byte keys; other key shapes are generated per rank and are not regenerable).
    layout = (world, chunk_leaves) for the block-cyclic pipelined array (None: contiguous leaf
    ranges of ceil(n_leaves / world) leaves; world then from the process group).  On a mismatch
    `diagnose_gather` names every differing leaf with its owning rank and round, decides from
    the oracle which side is wrong, and keeps the bytes (gpurun_out/verify_gather_fail/)."""
    if key_bytes != 16 or sum(all_counts) > 1_200_000_000:
        return None
    full_plan = amq.plan_filters(kind, all_counts, bpk, payload_capacity=cap, out_stride=stride)
    allk = amq.gen_keys16(42, 0, sum(all_counts), device=dev)
    if kind == 1:
        allk = sort_segments_device(torch, allk, all_counts)
    full = torch.zeros(max(gathered.numel(), full_plan.total_out_bytes), dtype=torch.uint8,
                       device=dev)
    amq.build_all_filters(full_plan, amq.KeyBatch.fixed(allk), out=full[:full_plan.total_out_bytes])
    ok = bool(torch.equal(full[:gathered.numel()], gathered))
    if not ok and stride:
        bad = torch.nonzero(full[:gathered.numel()] != gathered).flatten()
        leaves = sorted({int(x) // stride for x in bad.tolist()})
        print(f"verify_gather: {bad.numel()} bytes differ, in {len(leaves)} leaves {leaves[:16]} "
              f"(first byte {int(bad[0])})", file=sys.stderr, flush=True)
        try:
            diagnose_gather(torch, amq, kind, bpk, cap, all_counts, stride, gathered, full, allk,
                            leaves, layout, batches)
        except Exception as e:  # (the diagnosis must not hide the failure itself)
            print(f"verify_gather: diagnosis failed: {e!r}", file=sys.stderr, flush=True)
    del full, allk
    return ok


def diagnose_gather(torch, amq, kind, bpk, cap, all_counts, stride, gathered, full, allk, leaves,
                    layout, batches, max_leaves=32):
    """For each differing leaf (up to max_leaves): its owner rank and round, whether the keys
    each side built from are the oracle's (for VQF: sorted as the oracle sorts them), which
    side's bytes equal the oracle's filter, and whether a rebuild of the leaf alone on this GPU
    reproduces either side.  Writes summary.json plus the leaves' bytes from both sides and the
    oracle under gpurun_out/verify_gather_fail/ and prints the summary on stderr."""
    import torch.distributed as dist
    from oracle import oracle as O
    O.build_oracle()
    world = layout[0] if layout else dist.get_world_size()
    n = len(all_counts)
    begin = np.concatenate([[0], np.cumsum(np.asarray(all_counts, dtype=np.int64))])
    out_dir = os.path.join(ROOT, "gpurun_out", "verify_gather_fail")
    os.makedirs(out_dir, exist_ok=True)
    rows, keep = [], {}
    for s_ in leaves[:max_leaves]:
        if layout:
            q = layout[1]
            rnd, rank = s_ // (world * q), (s_ // q) % world
        else:
            per = -(-n // world)
            rnd, rank = 0, s_ // per
        k0, k1 = int(begin[s_]), int(begin[s_ + 1])
        kh = O.gen_keys16(42, k0, k1 - k0)
        if kind == 1:
            O.sort_segments(kh, np.array([0, k1 - k0], dtype=np.uint64))
            st, ref, pl = O.vqf_build(kh, k1 - k0, bpk, cap, src_page_id=s_)
            ref = ref[:pl.payload_used]
        else:
            st, ref = O.bloom_build(kh, k1 - k0, bpk, src_page_id=s_)
        ref = ref.tobytes()
        g = gathered[s_ * stride:s_ * stride + len(ref)].cpu().numpy().tobytes()
        f = full[s_ * stride:s_ * stride + len(ref)].cpu().numpy().tobytes()
        row = {"leaf": int(s_), "rank": int(rank), "round": int(rnd), "keys": k1 - k0,
               "gathered_equals_oracle": g == ref, "single_build_equals_oracle": f == ref,
               "single_build_keys_equal_oracle": bool(np.array_equal(allk[k0:k1].cpu().numpy(), kh)),
               "bytes_differing": int(sum(a != b for a, b in zip(g, f)))}
        if batches is not None and layout and rank == 0 and rnd < len(batches) and batches[rnd] is not None:
            # this rank's own round batch: the keys its build actually read
            rb = rnd * world * q  # the round's first leaf; rank 0's leaves come first in it
            off = int(begin[s_] - begin[rb])
            row["round_batch_keys_equal_oracle"] = bool(np.array_equal(
                batches[rnd].data[off:off + k1 - k0].cpu().numpy(), kh))
        # the leaf alone, twice, on this GPU
        sp = amq.plan_filters(kind, [k1 - k0], bpk, payload_capacity=cap, src_page_ids=[s_])
        again = []
        for _ in range(2):
            o = amq.build_all_filters(sp, amq.KeyBatch.fixed(torch.from_numpy(kh).to(allk.device)))
            again.append(o[:len(ref)].cpu().numpy().tobytes() == ref)
        row["alone_equals_oracle"] = again
        rows.append(row)
        keep[f"leaf{s_}_gathered"] = np.frombuffer(g, np.uint8)
        keep[f"leaf{s_}_single"] = np.frombuffer(f, np.uint8)
        keep[f"leaf{s_}_oracle"] = np.frombuffer(ref, np.uint8)
    summary = {"kind": kind, "bpk": bpk, "world": world, "layout": layout, "n_leaves": n,
               "differing_leaves": len(leaves), "leaves": rows}
    with open(os.path.join(out_dir, "summary.json"), "w") as fh:
        json.dump(summary, fh, indent=1)
    np.savez(os.path.join(out_dir, "leaves.npz"), **keep)
    print("verify_gather diagnosis: " + json.dumps(summary), file=sys.stderr, flush=True)


def verify_probe(torch, kind, plan, filters, q, qseg, is_hit, res, baseline):
    """All lookups of the timed probe through the CPU oracle over the GPU-built filter bytes:
    the answers (and so the FPR) must be identical.  Timed, this is also the probe's CPU
    baseline (the oracle's reject_page loop over `cores` host threads)."""
    from oracle import oracle as O
    O.build_oracle()
    native = O.native_lib() if baseline else None
    cores, share = host_cpu_share()
    f = filters.cpu().numpy()
    qh = q.cpu().numpy()
    qs = qseg.cpu().numpy().astype(np.uint32)
    got = res.cpu().numpy()
    hit = is_hit.cpu().numpy()
    offs = plan.segs["out_offset"]
    t0 = time.perf_counter()
    st, ref = O.probe_segments(kind, f, offs, qh, qs, n_threads=cores, L=native)
    dt = time.perf_counter() - t0
    if st != 0:
        raise SystemExit(f"bench.py: oracle probe failed ({st})")
    equal = bool(np.array_equal(got, ref))
    if not equal:
        raise SystemExit(f"bench.py: probe answers differ from the oracle's at "
                         f"{np.nonzero(got != ref)[0][:8].tolist()}")
    out = {"results_equal_oracle": equal,
           "fpr_oracle": round(float(ref[~hit].mean()), 6),
           "false_positives": int(ref[~hit].sum())}
    if baseline:
        out["cpu_baseline"] = {
            "value": round(len(qs) / dt / 1e6, 2), "unit": "Mkeys/s", "cores": cores,
            "kind": "port",
            "sample": f"all {len(qs)} lookups of the timed probe, C oracle probe "
                      f"(tkvo_probe_segments: hash + {'Bloom query' if kind == 0 else 'vqf_is_present'}"
                      f" per lookup, {'-O3 -march=native -mbmi2 -mavx2' if native else '-O3 -march=x86-64-v3'}), "
                      f"{cores} threads, {dt:.2f} s wall",
            "host": share, "per_core_mkeys_s": round(len(qs) / dt / 1e6 / cores, 2)}
    return out


def batch_sweep(torch, amq, kind, bpk, cap, counts, kb, ws, plan_all, kernel_ms_all, steps=20):
    """Build rate against the number of leaves per batch (a checkpoint's build_all_pages
    queue holds tens to thousands of leaves): the first L leaves of the same keys."""
    rows = []
    stream = torch.cuda.current_stream()
    for L in SWEEP_LEAVES:
        if L >= len(counts):
            continue
        c = counts[:L]
        nk = sum(c)
        p = amq.plan_filters(kind, c, bpk, payload_capacity=cap)
        sub = (amq.KeyBatch.fixed(kb.data[:nk]) if kb.offsets is None else
               amq.KeyBatch.variable(kb.data, kb.offsets[:nk + 1]))
        o = torch.empty(max(p.total_out_bytes, 1), dtype=torch.uint8, device=kb.data.device)
        if p.workspace_bytes > ws.numel():  # (small Bloom batches split leaves over workgroups)
            ws = torch.empty(p.workspace_bytes, dtype=torch.uint8, device=kb.data.device)
        for _ in range(5):
            amq.build_all_filters(p, sub, out=o, workspace=ws, check=False)
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
              for _ in range(steps)]
        for a, b in ev:
            a.record(stream)
            amq.build_all_filters(p, sub, out=o, workspace=ws, check=False)
            b.record(stream)
        torch.cuda.synchronize()
        ms = float(np.mean([a.elapsed_time(b) for a, b in ev]))
        rows.append({"leaves": L, "keys": nk, "ms": round(ms, 4), "mkeys_s": round(nk / ms / 1e3, 1)})
    rows.append({"leaves": len(counts), "keys": int(sum(counts)), "ms": round(kernel_ms_all, 4),
                 "mkeys_s": round(sum(counts) / kernel_ms_all / 1e3, 1)})
    return rows


def one_rank_at_a_time(torch, dist, world, rank, fn):
    """fn() on every rank.  Ranks sharing one device (gloo rehearsals with more ranks than
    GPUs) run it one after another: torch's device sort, run from several processes on one GPU
    at once, stalled for minutes (4 and 8 ranks, round 6) while each alone takes ~0.2 s."""
    import torch.distributed as tdist_
    if not (tdist_.is_available() and tdist_.is_initialized()) or world <= torch.cuda.device_count():
        return fn()
    res = None
    for r in range(world):
        if r == rank:
            res = fn()
            torch.cuda.synchronize()
        dist.barrier()
    return res


def sort_segments_device(torch, keys, counts, chunk_keys=1 << 23):
    """memcmp order within each leaf: lexicographic on the big-endian view of the two
    8-byte words, via two stable sorts (low word, then high word) and a stable leaf sort.
    Runs over groups of whole leaves of at most `chunk_keys` keys: the same torch sequence
    applied to all 100M keys at once returned rows that were not a permutation of the input
    past leaf ~2007 on this ROCm build (argsort and repeat_interleave alone check out at
    100M, tools/gpu/diag_torch_sort.py; the failing op was not isolated).  Chunked, the
    result equals the oracle's sort at full size (tests/test_gpu_scale.py), and the bench
    re-checks every leaf against oracle-generated keys after every run (verify_all_leaves)."""
    out = torch.empty_like(keys)
    b = 0
    i = 0
    while i < len(counts):
        j, nk = i, 0
        while j < len(counts) and (nk == 0 or nk + counts[j] <= chunk_keys):
            nk += counts[j]
            j += 1
        out[b:b + nk] = _sort_leaves(torch, keys[b:b + nk], counts[i:j])
        b += nk
        i = j
    return out


def _sort_leaves(torch, keys, counts):
    n = keys.shape[0]
    if n == 0:
        return keys
    w = keys.reshape(n, 16).view(torch.int64).reshape(n, 2)
    def be(x):  # byte-swap to big-endian order, map unsigned -> signed order
        b = x.view(torch.uint8).reshape(-1, 8).flip(1).contiguous().view(torch.int64).reshape(-1)
        return b ^ torch.iinfo(torch.int64).min
    hi, lo = be(w[:, 0].contiguous()), be(w[:, 1].contiguous())
    seg = torch.repeat_interleave(torch.arange(len(counts), device=keys.device),
                                  torch.tensor(counts, device=keys.device))
    idx = torch.argsort(lo, stable=True)
    idx = idx[torch.argsort(hi[idx], stable=True)]
    idx = idx[torch.argsort(seg[idx], stable=True)]
    return keys[idx]


def _lsr(x, s):
    """logical right shift of an int64 tensor"""
    return (x >> s) & ((1 << (64 - s)) - 1)


def _s64(c):
    return c - (1 << 64) if c >= 1 << 63 else c


def splitmix_keys16(torch, seed, idx):
    """Key idx[i] of oracle/tkv_amq_oracle.c tkvo_gen_keys16 (== turtle_kv_amd.gen_keys16),
    computed elementwise: (splitmix64_at(seed, 2g+1), splitmix64_at(seed, 2g+2)), little
    endian.  `seed` is an int or an int64 tensor like idx."""
    def at(n):
        z = seed + n * _s64(0x9E3779B97F4A7C15)
        z = (z ^ _lsr(z, 30)) * _s64(0xBF58476D1CE4E5B9)
        z = (z ^ _lsr(z, 27)) * _s64(0x94D049BB133111EB)
        return z ^ _lsr(z, 31)
    w = torch.stack([at(2 * idx + 1), at(2 * idx + 2)], dim=1)
    return w.view(torch.uint8).reshape(idx.shape[0], 16)


def make_probe_queries(torch, amq, n, counts, dev, key_begin):
    """BASELINE config 4: n hits (the inserted keys, each probing its own
    leaf) + n misses (seed 43 keys, each probing a random leaf), shuffled with seed 44.
    The shuffled keys are generated in place (no 3.2 GB row gather: torch's index kernels
    returned wrong rows on multi-GB uint8 tensors on this ROCm build, see
    sort_segments_device)."""
    seg_hit = torch.repeat_interleave(torch.arange(len(counts), device=dev, dtype=torch.int32),
                                      torch.tensor(counts, device=dev))
    g = torch.Generator(device=dev)
    g.manual_seed(44)
    seg_miss = torch.randint(0, len(counts), (n,), device=dev, dtype=torch.int32, generator=g)
    perm = torch.randperm(2 * n, device=dev, generator=g)
    is_hit = perm < n
    gi = torch.where(is_hit, perm, perm - n) + key_begin
    seed = torch.where(is_hit, 42, 43).to(torch.int64)
    q = splitmix_keys16(torch, seed, gi).contiguous()
    qs = torch.cat([seg_hit, seg_miss])[perm].contiguous()
    return q, qs, is_hit


def end_to_end(torch, amq, kind, bpk, cap, counts, keys, iters=3, sync=lambda: None,
               reduce_max=lambda x: x, total_keys=None, world=1):
    """Keys from pinned host memory -> H2D -> build -> D2H into pinned host pages, through
    turtle_kv_amd.filters.HostFilterPipeline (chunked, three streams, overlapped).  With
    several ranks every rank runs its own leg at the same time (`sync` lines them up); the
    rate is all ranks' keys over the slowest rank's time (`reduce_max`)."""
    n = keys.shape[0]
    total_keys = total_keys or n
    h_keys = torch.empty(keys.shape, dtype=torch.uint8, pin_memory=True)
    h_keys.copy_(keys)
    pipe = amq.filters.HostFilterPipeline(kind, counts, bpk, payload_capacity=cap)
    h_out = pipe.run(h_keys)
    torch.cuda.synchronize()
    sync()
    t0 = time.perf_counter()
    for _ in range(iters):
        pipe.run(h_keys, h_out)
    dt_rank = (time.perf_counter() - t0) / iters
    dt = reduce_max(dt_rank)
    gbs = (keys.numel() + h_out.numel()) / dt_rank / 1e9
    res = {"mkeys_s": round(total_keys / dt / 1e6, 2), "ms_per_batch": round(dt * 1e3, 3),
           "pcie_gb_s_rank0": round(gbs, 1), "ranks": world,
           "note": "pinned host keys -> H2D -> build -> D2H filter pages; 8M-key chunks "
                   "pipelined on three streams (HostFilterPipeline)"
                   + ("; every rank at once over its own PCIe link, all ranks' keys / slowest rank"
                      if world > 1 else "")}
    # the reference's input form: keys viewed inside edit records (EditView), gathered on the
    # host chunk by chunk (tkv_amq_stage_keys) ahead of each chunk's H2D copy
    rec = np.empty((n, 32), dtype=np.uint8)          # [16-byte key | 16-byte value] per edit
    rec[:, :16] = h_keys.numpy()
    views = amq.key_views(rec, np.arange(n, dtype=np.uint64) * 32, 16)
    h_out2 = pipe.run_views(views)
    assert torch.equal(h_out2, h_out), "staged-from-views pages differ"
    torch.cuda.synchronize()
    sync()
    t0 = time.perf_counter()
    for _ in range(iters):
        pipe.run_views(views, h_out2)
    dt = reduce_max((time.perf_counter() - t0) / iters)
    res["from_key_views"] = {"mkeys_s": round(total_keys / dt / 1e6, 2), "ms_per_batch": round(dt * 1e3, 3),
                             "note": "keys viewed in 32-byte edit records, gathered by "
                                     "tkv_amq_stage_keys (16 host threads per rank) chunk by "
                                     "chunk, overlapping the previous chunk's copies and build"}
    del rec, views
    return res


def load_profile(workload):
    """profiles/traffic_<workload>.json, written by tools/pmc_summary.py from rocprofv3 --pmc
    passes of this bench (HBM bytes per launch, VALU instructions per key)."""
    p = os.path.join(ROOT, "profiles", f"traffic_{workload}.json")
    if os.path.exists(p):
        with open(p) as f:
            return json.load(f)
    return {}


if __name__ == "__main__":
    main()
