"""Summarise rocprofv3 --pmc passes for one kernel into profiles/traffic_<workload>.json
(read by bench.py for roofline.traffic and valu_roofline).

  python tools/pmc_summary.py --workload bloom10 --kernel bloom_build \
      --fetch gpurun_out/pmc_fetch --write gpurun_out/pmc_write --sq gpurun_out/pmc_sq \
      --keys 100000000 --alg-bytes 1725390848

HBM bytes follow MI355X_MICROARCH.md (HBM section): FETCH_SIZE counts half of a 16 B/lane
streaming read on gfx950, so hbm = 2*FETCH_SIZE*1024 + WRITE_SIZE*1024.
"""
from __future__ import annotations

import argparse
import collections
import csv
import json
import os

# gfx950 integer VALU issue, measured by tools/ubench_valu.hip (profiles/r03/ubench_valu.log):
# v_xor_b32 / v_add_u32 streams, 8 independent chains per wave, 8 waves per SIMD, >= 2 s of
# back-to-back launches: 578.8-584.5 G wave64-instructions/s at an in-kernel clock of 2.38-2.39
# GHz, i.e. one wave64 integer instruction per ~4.2 shader cycles per SIMD (v_fma_f32 the same:
# 583 G/s).  The guide's 2-cycle v_fma_f32 figure (MI355X_MICROARCH.md:473) is not reached by
# these streams: 1 wave/SIMD 439, 2 waves 531, 4 waves 560, 8 waves 579 G/s.
SIMDS = 1024
VALU_PEAK_G = 578.8   # measured, G wave64-instructions/s (the v_xor_b32 row at 8 waves/SIMD)
VALU_PEAK_NOTE = ("measured integer VALU issue rate: tools/ubench_valu.hip v_xor_b32 at 8 waves/SIMD, "
                  "in-kernel clock 2.387 GHz (profiles/r03/ubench_valu.log)")
CUS = 256


def kernel_ms(d, kernel):
    """mean duration of the kernel's dispatches in a counter-collection CSV (ms)"""
    rows = list(csv.DictReader(open(os.path.join(d, "run_counter_collection.csv"))))
    seen = {}
    for r in rows:
        if any(n in r["Kernel_Name"] for n in kernel.split(",")):
            seen[r["Dispatch_Id"]] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-6
    return sum(seen.values()) / len(seen) if seen else None


def agg(d, kernel):
    """Per-launch counter values of the step: for each comma-separated kernel-name substring,
    the mean over its dispatches; summed over the kernels (one step = one launch of each;
    GRBM_GUI_ACTIVE sums to the step's busy clock)."""
    rows = list(csv.DictReader(open(os.path.join(d, "run_counter_collection.csv"))))
    total = collections.defaultdict(float)
    for spec in kernel.split(","):
        # "name*n": the kernel runs n times per step (e.g. once per routed part)
        name, _, times = spec.partition("*")
        n = int(times) if times else 1
        out = collections.defaultdict(list)
        for r in rows:
            if name in r["Kernel_Name"]:
                out[r["Counter_Name"]].append(float(r["Counter_Value"]))
        for k, v in out.items():
            total[k] += n * sum(v) / len(v)
    return dict(total)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", required=True)
    ap.add_argument("--kernel", required=True,
                    help="kernel-name substring; several, comma-separated, for a multi-kernel step; "
                         "name*n for a kernel launched n times per step")
    ap.add_argument("--fetch", required=True)
    ap.add_argument("--write", required=True)
    ap.add_argument("--sq", default=None)
    ap.add_argument("--valu", default=None,
                    help="pass with SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_INSTS_VALU "
                         "GRBM_GUI_ACTIVE (VALUBusy, clock)")
    ap.add_argument("--tcc", default=None,
                    help="pass with TCC_EA0_RDREQ_sum / TCC_HIT_sum / TCC_MISS_sum (probes)")
    ap.add_argument("--ms", type=float, default=None,
                    help="step time per launch (ms, the bench's HIP events): the request rate of "
                         "--tcc and the effective clock of --valu")
    ap.add_argument("--keys", type=int, required=True)
    ap.add_argument("--alg-bytes", type=int, required=True)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    f, w = agg(a.fetch, a.kernel), agg(a.write, a.kernel)
    hbm = int(2 * f["FETCH_SIZE"] * 1024 + w["WRITE_SIZE"] * 1024)
    res = {
        "kernel": a.kernel, "workload": a.workload,
        "FETCH_SIZE_KiB": f["FETCH_SIZE"], "WRITE_SIZE_KiB": w["WRITE_SIZE"],
        "correction": "hbm_bytes = 2*FETCH_SIZE*1024 + WRITE_SIZE*1024 (gfx950 FETCH_SIZE "
                      "counts half of 16B/lane streaming reads)",
        "hbm_bytes_per_launch": hbm, "algorithmic_bytes_per_launch": a.alg_bytes,
        "traffic_over_algorithmic": round(hbm / a.alg_bytes, 4),
    }
    if a.sq:
        sq = agg(a.sq, a.kernel)
        clk_cycles = sq["GRBM_GUI_ACTIVE"] / 8
        valu = sq["SQ_INSTS_VALU"]
        res.update({
            "SQ_INSTS_VALU_per_launch": valu, "SQ_WAVES": sq.get("SQ_WAVES"),
            "valu_instr_per_key": round(valu * 64 / a.keys, 1),
            "GRBM_GUI_ACTIVE_per_xcd": clk_cycles,
            "valu_cycles_per_wave_instr_per_simd": round(clk_cycles / (valu / SIMDS), 3),
        })
    if a.valu:
        v = agg(a.valu, a.kernel)
        # the step's time from the bench (HIP events) when given: a dispatch timed under
        # counter collection runs longer than it does alone
        ms = a.ms or kernel_ms(a.valu, a.kernel)
        clk = v["GRBM_GUI_ACTIVE"] / 8  # rocprofv3 sums GRBM_GUI_ACTIVE over the 8 XCDs
        res.update({
            "valu_busy_frac": round(v["SQ_ACTIVE_INST_VALU"] / CUS / clk, 4),
            "valu_busy_note": "VALUBusy = sum SQ_ACTIVE_INST_VALU (quad-cycles, 4 SIMDs) / CUs / "
                              "(GRBM_GUI_ACTIVE / 8): the fraction of cycles each SIMD issues VALU",
            "valu_thread_util": round(v["SQ_THREAD_CYCLES_VALU"] / (v["SQ_ACTIVE_INST_VALU"] * 64), 4),
            "clock_ghz_effective": round(clk / (ms * 1e-3) / 1e9, 3) if ms else None,
            "step_ms": round(ms, 4) if ms else None,
        })
        if "valu_instr_per_key" not in res:
            res["valu_instr_per_key"] = round(v["SQ_INSTS_VALU"] * 64 / a.keys, 1)
    if "valu_instr_per_key" in res:
        res["valu_peak_ginstr_s"] = VALU_PEAK_G
        res["valu_peak_note"] = VALU_PEAK_NOTE
    if a.tcc:
        t = agg(a.tcc, a.kernel)
        req = t["TCC_EA0_RDREQ_sum"]
        res.update({
            "TCC_EA0_RDREQ_per_launch": req, "TCC_HIT_per_launch": t.get("TCC_HIT_sum"),
            "TCC_MISS_per_launch": t.get("TCC_MISS_sum"),
            "ea_read_requests_per_unit": round(req / a.keys, 4),
        })
        if a.ms:
            res["ea_read_requests_g_per_s"] = round(req / (a.ms * 1e-3) / 1e9, 2)
    res["source"] = (f"rocprofv3 --pmc passes: {a.fetch}, {a.write}, {a.sq or '-'}, {a.tcc or '-'}, "
                     f"{a.valu or '-'}")
    out = a.out or os.path.join("profiles", f"traffic_{a.workload}.json")
    with open(out, "w") as fh:
        json.dump(res, fh, indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
