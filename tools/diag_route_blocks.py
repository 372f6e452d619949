"""GPU diagnostic: the pipelined hash-range form played by hand on one GPU for a few shapes;
per tile, bytes differing from the oracle and whether bits are missing or extra."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def main():
    import torch

    import turtle_kv_amd as amq
    from oracle import oracle as O
    from test_gpu_hash_shard import _pipelined_by_hand
    O.build_oracle()
    for n, bpk, world, chunks in [(900_000, 5, 1, 1), (900_000, 5, 2, 1), (900_000, 12, 2, 1),
                                  (900_000, 8, 2, 1), (900_000, 5, 2, 2), (2_000_000, 5, 2, 1),
                                  (900_000, 6, 2, 1), (900_000, 10, 2, 1)]:
        keys = amq.gen_keys16(31, 0, n)
        per = -(-n // world)
        parts = [keys[r * per:min(n, (r + 1) * per)] for r in range(world)]
        filt, hss = _pipelined_by_hand(amq, torch, parts, bpk, chunks)
        st, ref = O.bloom_build(keys.cpu().numpy(), n, bpk, src_page_id=0)
        got = filt.cpu().numpy()
        h = hss[0]
        msg = f"n={n} bpk={bpk} W={world} K={chunks} T={h.T} q={h.q} parts={h.n_parts} P={h.rp.route_wgs} cap={h.rp.region_cap}"
        if got.tobytes() == ref.tobytes():
            print(msg, "OK", flush=True)
            continue
        g8, r8 = got[64:].view(np.uint8), ref[64:].view(np.uint8)
        tiles = {}
        for t in range(h.T):
            a, b = g8[t * 131072:(t + 1) * 131072], r8[t * 131072:(t + 1) * 131072]
            miss = int(np.unpackbits(b & ~a).sum())
            extra = int(np.unpackbits(a & ~b).sum())
            if miss or extra:
                tiles[t] = (miss, extra, int(np.unpackbits(b).sum()))
        print(msg, "header", got[:64].tobytes() == ref[:64].tobytes(), "tiles (missing, extra, ref bits):", tiles, flush=True)
        # each received part block's region counts and overflow counter ([round][chunk][sender])
        for r, hs in enumerate(hss):
            rp = hs.rp
            blk = hs.recv.cpu().numpy()
            for i in range(hs.g * hs.chunks * hs.world):
                b = blk[i * rp.block_bytes:(i + 1) * rp.block_bytes]
                cnt = b[rp.counts_off:rp.counts_off + 4 * rp.route_wgs].view(np.uint32)
                ovf = int(b[rp.ovf_n_off:rp.ovf_n_off + 4].view(np.uint32)[0])
                print(f"  rank {r} block {i}: records {int(cnt.sum())} max region {int(cnt.max())} "
                      f"(cap {rp.region_cap}) ovf {ovf}")

if __name__ == "__main__":
    main()
