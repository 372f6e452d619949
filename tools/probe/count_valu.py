"""VALU instructions (v_*) per kernel body of an AMDGPU assembly file (hipcc -S), for
tools/probe/xxh_short_count.hip: the runtime-length short XXH64 against one body per length."""
import re
import sys

counts, cur = {}, None
for line in open(sys.argv[1]):
    m = re.match(r"^([A-Za-z_][\w$.]*):\s*(;.*)?$", line)
    if m and not m.group(1).startswith(".L"):
        cur = m.group(1)
        counts.setdefault(cur, 0)
        continue
    s = line.strip()
    if cur and s.startswith("s_endpgm"):
        cur = None
    elif cur and s.startswith("v_"):
        counts[cur] += 1
var = {k: v for k, v in counts.items() if "var" in k}
fixed = {int(re.search(r"ILj(\d+)E", k).group(1)): v for k, v in counts.items() if "len" in k}
for k, v in var.items():
    print(f"runtime length (mixed wave): {v} VALU")
for n in sorted(fixed):
    print(f"length {n:2d}: {fixed[n]} VALU")
if fixed:
    avg = sum(fixed.values()) / len(fixed)
    print(f"mean over lengths 8..31 (uniform): {avg:.1f} VALU; a mixed wave pays "
          f"{list(var.values())[0] - avg:.1f} more per key")
