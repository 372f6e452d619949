"""Projected config-5 step at N ranks: HashShardedBloom.step's two streams played out with
stage times from one-GPU measurements and link bytes over xGMI.

Compute stream: route chunk 0..C-1, then part build j (waits for X(C-1, j)).
Communication stream, in issue order: X(c, *) for c < C-1 (each waits for route c), then
X(C-1, 0), X(C-1, 1), and per build j: X(C-1, j + 2), G(j - 1); finally G(g - 1).  G(j) waits
for build j.  X(c, *) moves a chunk's blocks of every round, X(C-1, j) one round's.

  python tools/c5_schedule.py --route-ms-per-1b 11.2 --part-ms 0.192 --link-gbs 153
"""
import argparse


def plan(n_total, bpk, world, chunks):
    """Block and part geometry as tkv_amq_bloom_route_plan sizes it (the C++ is the source)."""
    import math
    n_blocks = -(-n_total * bpk // 512)
    T = -(-n_blocks // 2048)
    per_rank = -(-T // world)
    g = -(-per_rank // 256)
    q = -(-T // (world * g))
    ck = -(-(-(-n_total // world)) // chunks)
    P = min(256, max(1, -(-ck // (32 * 1024))))
    e = -(-ck // P) * min(q * 2048, n_blocks) / n_blocks  # records per region
    cap = (int(e + 2 * math.sqrt(e) + 16) + 15) & ~15
    ovf_cap = 4096 + 4 * P + ck // (world * g * 256)
    a256 = lambda x: (x + 255) & ~255
    block = a256(a256(a256(4 * P) + 256 + 12 * P * cap) + 16 * ovf_cap)
    part_bytes = q * 2048 * 64
    return dict(T=T, g=g, q=q, chunk_keys=ck, block_bytes=block, part_bytes=part_bytes,
                records_per_part=n_total / (world * g))


def simulate(world, chunks, g, route_chunk_ms, part_ms, x_chunk_ms, x_round_ms, g_round_ms):
    t_cur = 0.0
    route_end = []
    for c in range(chunks):
        t_cur += route_chunk_ms
        route_end.append(t_cur)
    t_comm = 0.0
    tl = {}
    for c in range(chunks - 1):
        t_comm = max(t_comm, route_end[c]) + x_chunk_ms
        tl[f"exchange_chunk_{c}"] = t_comm
    t_comm = max(t_comm, route_end[-1])
    x_end = [None] * g
    b_end = [None] * g

    def x_last(j):
        nonlocal t_comm
        t_comm += x_round_ms
        x_end[j] = t_comm
        tl[f"exchange_{j}"] = t_comm

    def gather(j):
        nonlocal t_comm
        t_comm = max(t_comm, b_end[j]) + g_round_ms
        tl[f"gather_{j}"] = t_comm

    for j in range(min(2, g)):
        x_last(j)
    for j in range(g):
        t_cur = max(t_cur, x_end[j]) + part_ms
        b_end[j] = t_cur
        tl[f"build_{j}"] = t_cur
        if j + 2 < g:
            x_last(j + 2)
        if j >= 1:
            gather(j - 1)
    gather(g - 1)
    return max(t_cur, t_comm), tl


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--total-keys", type=int, default=1_000_000_000)
    ap.add_argument("--bpk", type=int, default=12)
    ap.add_argument("--world", type=int, default=8)
    ap.add_argument("--chunks", type=int, default=4)
    ap.add_argument("--route-ms-per-1b", type=float, default=11.2, help="one GPU, 1B keys")
    ap.add_argument("--part-ms", type=float, default=0.192, help="one part build of ~21M records")
    ap.add_argument("--link-gbs", type=float, default=153.0, help="per xGMI link, one direction")
    ap.add_argument("--links", type=int, default=7)
    ap.add_argument("--one-gpu-ms", type=float, default=20.3, help="the measured step at N = 1")
    a = ap.parse_args()
    p = plan(a.total_keys, a.bpk, a.world, a.chunks)
    W, C, g = a.world, a.chunks, p["g"]
    rate = a.links * a.link_gbs * 1e9  # bytes/s into (and out of) one GPU
    x_chunk_bytes = (W - 1) * g * p["block_bytes"]  # one chunk's blocks, every round, out
    x_round_bytes = (W - 1) * p["block_bytes"]
    g_round_bytes = (W - 1) * p["part_bytes"]
    route_chunk_ms = a.route_ms_per_1b * a.total_keys / 1e9 / W / C
    step, tl = simulate(W, C, g, route_chunk_ms, a.part_ms, x_chunk_bytes / rate * 1e3,
                        x_round_bytes / rate * 1e3, g_round_bytes / rate * 1e3)
    xb = C * x_round_bytes * g
    print(f"plan: {p}")
    print(f"per rank over xGMI: exchange {xb / 1e9:.3f} GB (records alone "
          f"{12 * a.total_keys / W * (W - 1) / W / 1e9:.3f}), all-gather {g * g_round_bytes / 1e9:.3f} GB, "
          f"link floor {(xb + g * g_round_bytes) / rate * 1e3:.2f} ms at {rate / 1e9:.0f} GB/s")
    print(f"step {step:.2f} ms -> {a.total_keys / step / 1e6:.0f} Gkeys/s, "
          f"{a.one_gpu_ms / step:.2f}x the one-GPU step of {a.one_gpu_ms} ms")
    for k in sorted(tl, key=tl.get):
        print(f"  {k:20s} {tl[k]:.3f} ms")


if __name__ == "__main__":
    main()
