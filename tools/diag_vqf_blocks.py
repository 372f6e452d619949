"""Per-block comparison of one VQF leaf (GPU build vs the oracle): which blocks differ, and
whether their element counts (metadata zeros) or only their entries differ.  Kernel debugging.
  TKV_AMQ_LIB=... python tools/diag_vqf_blocks.py [n_keys] [bpk] [cap]"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import turtle_kv_amd as amq  # noqa: E402
from oracle import oracle as O  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 16384
bpk = int(sys.argv[2]) if len(sys.argv) > 2 else 12
cap = int(sys.argv[3]) if len(sys.argv) > 3 else 32704
O.build_oracle()
keys = O.gen_keys16(42, 0, n)
O.sort_segments(keys, np.array([0, n], np.uint64))
plan = amq.plan_filters(1, [n], bpk, payload_capacity=cap)
out = amq.build_all_filters(plan, amq.KeyBatch.fixed(torch.from_numpy(keys).cuda())).cpu().numpy()
st, ref, p = O.vqf_build(keys, n, bpk, cap, src_page_id=0)
seg = plan.segs[0]
o, nbytes = int(seg["out_offset"]), int(seg["payload_bytes"])
got = out[o:o + nbytes]
ref = ref[:p.payload_used]
T = int(seg["tag_bits"])
nb = int(seg["n_blocks"])
md = 16 if T == 8 else 8
def zeros(b):
    return sum(8 - bin(int(x)).count("1") for x in b[:md])
bad = []
for b in range(nb):
    g = got[80 + 64 * b:80 + 64 * (b + 1)]
    r = ref[80 + 64 * b:80 + 64 * (b + 1)]
    if g.tobytes() != r.tobytes():
        bad.append((b, zeros(g), zeros(r), g[:md].tobytes() == r[:md].tobytes()))
print("header equal", got[:80].tobytes() == ref[:80].tobytes(), "blocks", nb, "bad", len(bad))
for b in bad[:40]:
    print("block %4d zeros gpu %3d oracle %3d metadata equal %s" % b)
