"""Developer tool: where a fused first-fit launch spends its time. Runs
kbg_tool_firstfit_stamps (the diagnostic build tools/libkbg_tools_stamps.so,
kbg_kernels.hip KBG_FF_STAMPS) on a config's table for full-scan and grouped
batches and prints, per batch size, the launch span (first workgroup entry to
last exit, global 100 MHz clock) and each phase's median / max duration over
the workgroups (stamps serialise the kernel a little: read shares, not the
span). python kube-arbitrator_amd/tools/ff_stamps.py [config]"""
import ctypes
import json
import os
import statistics
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))

PHASES = ["rows_in", "scan", "round_barrier", "place", "append", "end"]


def main(cid):
    from kbgpu import _abi, synth
    from kbgpu.cache import FakeBinder, cache_from_fixture
    from kbgpu.fixture import _OrderedCache, fixture_tiers
    from kbgpu.snapshot import FlatSnapshot
    L = ctypes.CDLL(os.environ.get("TOOLS_LIB", os.path.join(HERE, "libkbg_tools_stamps.so")))
    fx = synth.config_fixture(cid)
    s = _OrderedCache(cache_from_fixture(fx, FakeBinder()), fx).snapshot()
    f = FlatSnapshot(s.nodes, s.jobs, s.queues, s.others, fixture_tiers(fx))
    MAXWG = 8192
    buf = (ctypes.c_ulonglong * (MAXWG * 8))()
    for full, G in ((1, 4174), (1, 4655), (1, 8192), (0, 8192), (0, 1024)):
        o = _abi.kbg_options()
        o.full_scan = full
        o.batch_tasks = 8192
        n = L.kbg_tool_firstfit_stamps(ctypes.byref(f.snap), ctypes.byref(o), G, buf, MAXWG)
        if n <= 0:
            print(json.dumps({"full": full, "G": G, "error": n}))
            continue
        st = [[buf[w * 8 + k] for k in range(8)] for w in range(n)]
        t0 = min(x[0] for x in st)
        res = {"mode": "full" if full else "grouped", "G": G, "workgroups": n,
               "span_us": (max(x[6] for x in st) - t0) / 100.0,
               "entry_us": {"median": statistics.median((x[0] - t0) / 100 for x in st),
                            "max": max((x[0] - t0) / 100 for x in st)},
               "wg_us": {"median": statistics.median((x[6] - x[0]) / 100 for x in st),
                         "max": max((x[6] - x[0]) / 100 for x in st)}}
        for k, name in enumerate(PHASES):
            d = [(x[k + 1] - x[k]) / 100 for x in st if x[k + 1] >= x[k]]
            if d:
                res[name] = {"median": statistics.median(d), "max": max(d)}
        print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main(int(sys.argv[1]) if len(sys.argv) > 1 else 3)
