"""Developer tool: scan-kernel timing of one or more builds of libkbgpu.so on
C3 (full-scan and grouped cycles). python tools/scan_bench.py lib1.so [lib2.so ...]
Each library runs in its own subprocess (ctypes cannot unload)."""
import ctypes
import json
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))


def run_one(lib, cid, reps):
    from kbgpu import _abi, synth
    _abi.LIB_PATH = lib
    from kbgpu.cache import cache_from_fixture
    from kbgpu.fixture import fixture_tiers
    from kbgpu.framework import open_session
    fx = synth.config_fixture(cid)
    cache = cache_from_fixture(fx)
    L = _abi.lib()
    out = {"lib": os.path.basename(lib), "config": cid, "general": bool(os.environ.get("KBG_FORCE_GENERAL_SCAN"))}
    for mode in (1, 0):
        ssn = open_session(cache, fixture_tiers(fx), {"full_scan": mode})
        cap = max(1, ssn.flat.pending_count)
        buf = (_abi.kbg_decision * cap)()
        n = ctypes.c_int32()
        best = None
        for _ in range(reps):
            _abi.check(L.kbg_session_reset(ssn.handle))
            _abi.check(L.kbg_allocate(ssn.handle, buf, cap, ctypes.byref(n)))
            st = ssn.stats()
            r = {"scan_us_per_launch": st.scan_kernel_ms * 1e3 / max(1, st.scan_launches),
                 "rows_per_launch": st.evaluations / max(1, st.scan_launches), "launches": st.scan_launches,
                 "scan_ms": st.scan_kernel_ms, "select_ms": st.select_kernel_ms, "cycle_ms": st.allocate_ms}
            if best is None or r["scan_ms"] < best["scan_ms"]:
                best = r
        out["full_scan" if mode else "grouped"] = best
        ssn.close()
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    if sys.argv[1] == "--one":
        run_one(sys.argv[2], int(sys.argv[3]), int(sys.argv[4]))
    else:
        cid = int(os.environ.get("CONFIG", "3"))
        for lib in sys.argv[1:]:
            subprocess.run([sys.executable, __file__, "--one", os.path.abspath(lib), str(cid), "5"], check=True)
