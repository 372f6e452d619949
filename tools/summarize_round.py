"""Turn one profile_round.sh output directory into profiles/traffic_<workload>.json (through
tools/pmc_summary.py) for every workload with PMC passes, taking the key count and the
algorithmic bytes per launch from that round's bench line of the workload.

  python tools/summarize_round.py gpurun_out/r03_round [--copy profiles/r03/round]
"""
from __future__ import annotations

import argparse
import json
import os
import shutil
import subprocess
import sys

KERNELS = {  # kernel-name substrings of one step (pmc_summary sums them)
    "bloom10": "bloom_build_lds", "bloom12": "bloom_build_lds", "bloom10k24": "bloom_build_lds",
    "bloom10var": "bloom_build_lds", "vqf12": "vqf_decide<,vqf_place_fused",
    "vqf12k24": "vqf_decide<,vqf_place_fused", "vqf12var": "vqf_decide<,vqf_place_fused",
    "bloom10mono": "bloom_part_keys16,bloom_tile,bloom_overflow",
    "bloom10monok24": "bloom_part_keys24,bloom_tile,bloom_overflow",
    "bloom12big": "bloom_build_window,bloom_split_merge",
    "probe10": "bloom_probe", "probe_vqf12": "vqf_probe",
}


def bench_line(d, w):
    p = os.path.join(d, f"bench_{w}.log")
    if not os.path.exists(p):
        return None
    lines = [ln for ln in open(p) if ln.startswith("{")]
    return json.loads(lines[-1]) if lines else None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--copy", default=None, help="copy the pass CSVs and stats here (profiles/...)")
    a = ap.parse_args()
    here = os.path.dirname(os.path.abspath(__file__))
    for w, kern in KERNELS.items():
        fetch = os.path.join(a.dir, f"pmc_{w}_fetch")
        write = os.path.join(a.dir, f"pmc_{w}_write")
        if not (os.path.isdir(fetch) and os.path.isdir(write)):
            continue
        line = bench_line(a.dir, w)
        if line is None:
            print(f"{w}: no bench line, skipped", file=sys.stderr)
            continue
        units = line["probe"]["lookups"] if "probe" in line else line["config"]["keys_per_gpu"]
        alg = line["roofline"]["alg_bytes_per_launch"]
        dst = a.copy or os.path.join(a.dir, "summary")
        os.makedirs(dst, exist_ok=True)
        passes = {}
        for name in ("fetch", "write", "sq", "valu", "tcc"):
            src = os.path.join(a.dir, f"pmc_{w}_{name}")
            if os.path.isdir(src):
                tgt = os.path.join(dst, f"pmc_{w}_{name}")
                os.makedirs(tgt, exist_ok=True)
                # only the rows of the step's kernels (the pass also profiles key generation etc.)
                with open(os.path.join(src, "run_counter_collection.csv")) as fi, \
                        open(os.path.join(tgt, "run_counter_collection.csv"), "w") as fo:
                    head = fi.readline()
                    fo.write(head)
                    for ln in fi:
                        if any(k in ln for k in kern.split(",")):
                            fo.write(ln)
                passes[name] = tgt
        cmd = [sys.executable, os.path.join(here, "pmc_summary.py"), "--workload", w, "--kernel", kern,
               "--fetch", passes["fetch"], "--write", passes["write"], "--keys", str(units),
               "--alg-bytes", str(alg)]
        for name in ("sq", "valu", "tcc"):
            if name in passes:
                cmd += [f"--{name}", passes[name]]
        cmd += ["--ms", str(line["roofline"]["kernel_ms"])]  # the bench's step time (HIP events)
        subprocess.run(cmd, check=True, stdout=subprocess.DEVNULL)
        print(f"{w}: profiles/traffic_{w}.json")
    if a.copy:
        for f in os.listdir(a.dir):
            if f.startswith(("bench_", "gpu_tests", "sweep_", "small_")) and f.endswith(".log"):
                shutil.copy(os.path.join(a.dir, f), a.copy)
            p = os.path.join(a.dir, f)
            if f.startswith("prof_") and os.path.isdir(p):
                for g in os.listdir(p):
                    if g.endswith("kernel_stats.csv"):
                        shutil.copy(os.path.join(p, g), os.path.join(a.copy, f"{f[5:]}_kernel_stats.csv"))


if __name__ == "__main__":
    main()
