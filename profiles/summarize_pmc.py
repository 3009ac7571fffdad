"""Summarise a scripts/gpurun/pmc.sh session (rocprofv3 kernel trace + separate PMC
passes of one bench command) per kernel.

Usage: python profiles/summarize_pmc.py <session dir> <config> > summary.json
  <session dir>/c<config>_kt/kt_kernel_trace.csv        kernel durations
  <session dir>/c<config>_pmc<i>/pmc<i>_counter_collection.csv  counters

Kernels are keyed by their name up to the argument list, template arguments
kept: kbg_firstfit_kernel<true, false> runs the full-scan mode's batches
(every node of every row), kbg_firstfit_kernel<true, true> the production
mode's grouped batches; the rows-per-workgroup argument (16 / 24 / 32) is
dropped, so each mode's variants are one entry.
Derived figures (MI355X_MICROARCH.md):
  hbm_read_bytes  = 2 x FETCH_SIZE KiB x 1024 (gfx950 tallies 128-B requests
                    at 64 B; Infinity-Cache hits are counted too)
  hbm_write_bytes = WRITE_SIZE KiB x 1024
  valu_issue_floor_us = SQ_INSTS_VALU x 4 cycles / (1024 SIMDs x 2.4 GHz):
                    the time the kernel's wave64 VALU instructions need at
                    full issue on every SIMD of the chip
(No clock is derived from GRBM_GUI_ACTIVE: on dispatches of a few µs that
quotient reads far above the 2.4 GHz peak, MI355X_MICROARCH.md DVFS note.)
"""
import csv
import glob
import json
import os
import re
import statistics
import sys

SIMDS = 1024
CLOCK_GHZ = 2.4
VALU_CYC = 4
WANT = ("kbg_firstfit_kernel", "kbg_fitdelta_kernel", "kbg_scan_kernel", "kbg_select_kernel", "kbg_victim_kernel",
        "kbg_victim_big_kernel", "kbg_victim_prep_kernel", "kbg_apply_kernel", "copyBuffer")


def key(name, grid=0):
    """grid: the launch's work-items. The complete variant (<INT, false, true,
    ROWS>: one round, every word out) runs both modes' batches at C3's table
    size; its launches are told apart by size — a full-scan batch is one row
    per task (thousands of rows, >= 64 workgroups of 1024), a grouped batch
    one row per shape — and filed under <INT, false> / <INT, true>."""
    base = name.split("(")[0]
    base = re.sub(r"^void ", "", base)
    base = base.replace("kbg::", "")
    m = re.match(r"^kbg_firstfit_kernel<(\w+), (\w+), true, \d+>$", base)
    if m:
        return f"kbg_firstfit_kernel<{m.group(1)}, {'false' if grid // 1024 >= 64 else 'true'}>"
    # the fused kernel's rows-per-workgroup variants (16 / 24 / 32) of one mode are one entry
    return re.sub(r"^(kbg_firstfit_kernel<\w+, \w+)(, false)?, \d+>$", r"\1>", base)


def rows(path):
    with open(path) as f:
        return list(csv.DictReader(f))


def main():
    d, cfg = sys.argv[1], sys.argv[2]
    out = {"source": f"scripts/gpurun/pmc.sh: rocprofv3 --kernel-trace --stats, then one --pmc pass per counter group, of "
                     f"`python3 bench.py --config {cfg} --steps 3 --warmup 1 --no-cpu-baseline --no-resident`",
           "config": int(cfg), "kernels": {}}
    ks = out["kernels"]
    for r in rows(os.path.join(d, f"c{cfg}_kt", "kt_kernel_trace.csv")):
        k = key(r["Kernel_Name"], int(r["Grid_Size_X"]) * int(r["Grid_Size_Y"]) * int(r["Grid_Size_Z"]))
        if not any(w in k for w in WANT):
            continue
        ks.setdefault(k, {"durations_ns": []})["durations_ns"].append(
            int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    counters = {}
    for p in sorted(glob.glob(os.path.join(d, f"c{cfg}_pmc*", "*_counter_collection.csv"))):
        for r in rows(p):
            k = key(r["Kernel_Name"], int(r["Grid_Size"]))
            if k not in ks:
                continue
            c = counters.setdefault(k, {}).setdefault(r["Counter_Name"], {})
            c[int(r["Dispatch_Id"])] = c.get(int(r["Dispatch_Id"]), 0.0) + float(r["Counter_Value"])
            dur = counters[k].setdefault("_dur", {}).setdefault(r["Counter_Name"], {})
            dur[int(r["Dispatch_Id"])] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    # rows per launch of the profiled bench commands (the PMC figures scale with them)
    benches = []
    for p in sorted(glob.glob(os.path.join(d, f"c{cfg}_pmc*_bench.json"))):
        try:
            benches.append(json.load(open(p)))
        except (OSError, ValueError):
            pass
    full_rows = [b["scan_kernel"]["rows_per_launch"] for b in benches if "scan_kernel" in b]
    prod_rows = [b["production_mode"]["scan_kernel"]["rows_per_launch"] for b in benches if "production_mode" in b]
    out["bench_rows_per_launch"] = {"full_scan": statistics.mean(full_rows) if full_rows else None,
                                    "grouped": statistics.mean(prod_rows) if prod_rows else None}
    for k, v in ks.items():
        ds = v.pop("durations_ns")
        v.update(launches=len(ds), avg_ns=statistics.mean(ds), median_ns=statistics.median(ds), min_ns=min(ds),
                 max_ns=max(ds))
        c = counters.get(k, {})
        avg = {n: statistics.mean(x.values()) for n, x in c.items() if n != "_dur" and x}
        v["counters_per_launch"] = avg
        if "FETCH_SIZE" in avg:
            v["hbm_read_bytes_per_launch"] = 2 * avg["FETCH_SIZE"] * 1024
        if "WRITE_SIZE" in avg:
            v["hbm_write_bytes_per_launch"] = avg["WRITE_SIZE"] * 1024
        if "hbm_read_bytes_per_launch" in v and "hbm_write_bytes_per_launch" in v:
            v["hbm_bytes_per_launch"] = v["hbm_read_bytes_per_launch"] + v["hbm_write_bytes_per_launch"]
        if avg.get("TCC_HIT_sum", 0) + avg.get("TCC_MISS_sum", 0) > 0:
            v["l2_hit_rate"] = avg["TCC_HIT_sum"] / (avg["TCC_HIT_sum"] + avg["TCC_MISS_sum"])
        if "SQ_INSTS_VALU" in avg:
            v["valu_insts_per_launch"] = avg["SQ_INSTS_VALU"]
            v["valu_issue_floor_us"] = avg["SQ_INSTS_VALU"] * VALU_CYC / (SIMDS * CLOCK_GHZ * 1e3)
            v["valu_issue_frac"] = v["valu_issue_floor_us"] * 1e3 / v["avg_ns"]
            if avg.get("SQ_WAVES"):
                v["valu_insts_per_wave"] = avg["SQ_INSTS_VALU"] / avg["SQ_WAVES"]
        if avg.get("SQ_WAVE_CYCLES") and "SQ_WAIT_ANY" in avg:  # share of the waves' lifetime parked (s_waitcnt / barrier)
            v["wait_any_share"] = avg["SQ_WAIT_ANY"] / avg["SQ_WAVE_CYCLES"]
            if "SQ_WAIT_INST_ANY" in avg:
                v["wait_inst_share"] = avg["SQ_WAIT_INST_ANY"] / avg["SQ_WAVE_CYCLES"]
            if "SQ_ACTIVE_INST_ANY" in avg:
                v["active_inst_share"] = avg["SQ_ACTIVE_INST_ANY"] / avg["SQ_WAVE_CYCLES"]
            if "SQ_WAIT_INST_LDS" in avg:  # issue stalls on the LDS pipe (not lgkmcnt drains)
                v["wait_inst_lds_share"] = avg["SQ_WAIT_INST_LDS"] / avg["SQ_WAVE_CYCLES"]
    json.dump(out, sys.stdout, indent=1)
    print()


if __name__ == "__main__":
    main()
