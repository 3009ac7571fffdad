"""Builds profiles/pmc_scan.json (what bench.py reads for its PMC-based
figures) from the per-config summaries of profiles/summarize_pmc.py:

  python profiles/make_pmc_scan.py profiles/r03 [profiles/r02]
      # reads pmc_c3.json, pmc_c4.json, pmc_c5.json; a config missing from
      # the first directory is taken from the second (a kernel unchanged since)

C3 (5k nodes) gives the fused first-fit kernel in full-scan mode
(kbg_firstfit_kernel<true, false>) and production mode (<true, true>); C5 the
victim kernel; other node counts (C4) go under by_nodes."""
import json
import os
import sys

FIELDS = ("avg_ns", "launches", "hbm_bytes_per_launch", "hbm_write_bytes_per_launch", "l2_hit_rate",
          "valu_insts_per_launch", "wait_any_share", "wait_inst_share", "active_inst_share", "wait_inst_lds_share")


def section(k):
    out = {f: k.get(f) for f in FIELDS}
    out["hbm_read_bytes_per_launch_corrected"] = k.get("hbm_read_bytes_per_launch")
    out["waves_per_launch"] = k.get("counters_per_launch", {}).get("SQ_WAVES")
    return out


FULL, PROD = "kbg_firstfit_kernel<true, false>", "kbg_firstfit_kernel<true, true>"


def scan_modes(s):
    ks = s["kernels"]
    rows = s.get("bench_rows_per_launch", {})
    out = {"full_scan": section(ks[FULL]) if FULL in ks else None,
           "grouped": section(ks[PROD]) if PROD in ks else None}
    for m in out:
        if out[m] is not None:
            out[m]["rows_per_launch"] = rows.get(m)
    return out


def main():
    dirs = sys.argv[1:]
    srcs = {}

    def load(c):
        for dd in dirs:
            p = os.path.join(dd, f"pmc_c{c}.json")
            if os.path.exists(p):
                srcs[c] = os.path.relpath(p, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
                return json.load(open(p))
        return None
    c3, c4, c5 = load(3), load(4), load(5)
    if c4 and not any(k in c4["kernels"] for k in (FULL, PROD)):  # only the current kernel's passes
        c4 = None
        srcs.pop(4)
    out = {"kernel": "kbg_firstfit_kernel", "n_nodes": 5000}
    out.update(scan_modes(c3))
    if c5 and "kbg_victim_kernel" in c5["kernels"]:
        out["victim"] = dict(section(c5["kernels"]["kbg_victim_kernel"]), kernel="kbg_victim_kernel", n_nodes=10000)
    out["source"] = (f"{', '.join(srcs[c] for c in sorted(srcs))} (profiles/summarize_pmc.py over scripts/gpurun/pmc.sh): rocprofv3 "
                     "--kernel-trace --stats, then separate --pmc passes (FETCH_SIZE / WRITE_SIZE / "
                     "TCC_HIT_sum+TCC_MISS_sum / SQ_INSTS_VALU,SQ_WAVES,... / SQ_WAIT_ANY,...) of `python3 bench.py "
                     "--config {3,5} --steps 3 --warmup 1 --no-cpu-baseline --no-resident`; read = 2 x FETCH_SIZE "
                     "(gfx950 correction, MI355X_MICROARCH.md HBM section); FETCH/WRITE count Infinity-Cache hits too")
    if c4:
        out["by_nodes"] = {"20000": dict(scan_modes(c4), source=f"{srcs[4]} (scripts/gpurun/pmc.sh CFGS=4, same "
                                                                "passes as C3)")}
    json.dump(out, sys.stdout, indent=1)
    print()


if __name__ == "__main__":
    main()
