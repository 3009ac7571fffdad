"""Summarise rocprofv3 outputs of `bench.py` for the scan kernel.

Usage: python profiles/summarize.py <kernel_trace.csv> <fetch.csv> <write.csv> [<tcc.csv>] > summary.json

The bench runs the production (grouped) mode first, then the full-scan mode;
the full-scan phase starts at the first scan dispatch with >= 1024 evaluation
rows (grid y >= 16 workgroups); every later scan dispatch belongs to it. FETCH_SIZE/WRITE_SIZE are in KiB per dispatch; per
MI355X_MICROARCH.md §HBM, FETCH_SIZE counts 128-B requests at 64 B on gfx950,
so HBM read bytes = 2 x FETCH_SIZE x 1024 (uncalibrated for 8-B lane loads:
reported raw alongside).
"""
import csv
import json
import statistics
import sys

SCAN = "kbg_scan_kernel"


def rows(path):
    with open(path) as f:
        return list(csv.DictReader(f))


def main():
    kt = sorted((r for r in rows(sys.argv[1]) if SCAN in r["Kernel_Name"]), key=lambda r: int(r["Dispatch_Id"]))
    start = next(i for i, r in enumerate(kt) if int(r["Grid_Size_Y"]) >= 16)
    out = {"kernel": SCAN}
    for mode, sel in (("full_scan", kt[start:]), ("grouped", kt[:start])):
        d = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) for r in sel]
        if d:
            out[mode] = {"launches": len(d), "avg_ns": statistics.mean(d), "median_ns": statistics.median(d),
                         "min_ns": min(d), "max_ns": max(d)}
    for key, path in (("FETCH_SIZE", sys.argv[2]), ("WRITE_SIZE", sys.argv[3])):
        vals = {}
        pm = sorted((r for r in rows(path) if SCAN in r["Kernel_Name"] and r["Counter_Name"] == key),
                    key=lambda r: int(r["Dispatch_Id"]))
        x_blocks = int(kt[start]["Grid_Size_X"]) // int(kt[start]["Workgroup_Size_X"])
        first = next(i for i, r in enumerate(pm)
                     if int(r["Grid_Size"]) // int(r["Workgroup_Size"]) >= 16 * x_blocks)
        for i, r in enumerate(pm):
            vals.setdefault("full_scan" if i >= first else "grouped", []).append(float(r["Counter_Value"]))
        for mode, v in vals.items():
            out.setdefault(mode, {})[key + "_KiB_avg"] = statistics.mean(v)
    for mode in ("full_scan", "grouped"):
        m = out.get(mode, {})
        if "FETCH_SIZE_KiB_avg" in m:
            m["hbm_read_bytes_per_launch_corrected"] = 2 * m["FETCH_SIZE_KiB_avg"] * 1024
        if "WRITE_SIZE_KiB_avg" in m:
            m["hbm_write_bytes_per_launch"] = m["WRITE_SIZE_KiB_avg"] * 1024
        if "hbm_read_bytes_per_launch_corrected" in m and "hbm_write_bytes_per_launch" in m:
            m["hbm_bytes_per_launch"] = m["hbm_read_bytes_per_launch_corrected"] + m["hbm_write_bytes_per_launch"]
    if len(sys.argv) > 4:
        hit = miss = 0.0
        for r in rows(sys.argv[4]):
            if SCAN in r["Kernel_Name"]:
                if r["Counter_Name"] == "TCC_HIT_sum":
                    hit += float(r["Counter_Value"])
                elif r["Counter_Name"] == "TCC_MISS_sum":
                    miss += float(r["Counter_Value"])
        if hit + miss:
            out["l2_hit_rate"] = hit / (hit + miss)
    json.dump(out, sys.stdout, indent=1)
    print()


if __name__ == "__main__":
    main()
