"""Developer tool: per-cycle statistics of N allocate cycles on one session (GPU).
python kube-arbitrator_amd/tools/cycle_stats.py [config] [full_scan] [cycles]"""
import ctypes
import os
import statistics
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))


def main():
    cid = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    full = int(sys.argv[2]) if len(sys.argv) > 2 else 0
    n = int(sys.argv[3]) if len(sys.argv) > 3 else 30
    if os.environ.get("TORCH"):  # the bench's process: torch imported, its HIP context up
        import torch
        torch.cuda.set_device(0)
        torch.cuda.synchronize()
    from kbgpu import _abi, synth
    if os.environ.get("KBG_LIB"):  # A/B of library builds
        _abi.LIB_PATH = os.path.abspath(os.environ["KBG_LIB"])
    from kbgpu.cache import cache_from_fixture
    from kbgpu.fixture import fixture_tiers
    from kbgpu.framework import open_session
    fx = synth.config_fixture(cid)
    ssn = open_session(cache_from_fixture(fx), fixture_tiers(fx), {"device": 0, "full_scan": full})
    L = _abi.lib()
    cap = max(1, ssn.flat.pending_count)
    buf = (_abi.kbg_decision * cap)()
    out = ctypes.c_int32(0)
    rows = []
    for i in range(n + 2):
        _abi.check(L.kbg_session_reset(ssn.handle))
        _abi.check(L.kbg_allocate(ssn.handle, buf, cap, ctypes.byref(out)))
        st = ssn.stats()
        if i >= 2:
            rows.append((st.allocate_ms, st.engine_ms, st.resolve_ms, st.device_ms, st.delta_ms, st.batches))
    ssn.close()
    tag = os.environ.get("TAG", "")
    for r in rows:
        print(f"{tag} alloc {r[0]:7.3f} engine {r[1]:7.3f} resolve {r[2]:7.3f} device {r[3]:7.3f} delta {r[4]:7.3f} "
              f"batches {r[5]}")
    a = [r[0] for r in rows]
    print(f"{tag} SUMMARY p50 {statistics.median(a):.3f} mean {statistics.mean(a):.3f} max {max(a):.3f} "
          f"engine p50 {statistics.median(r[1] for r in rows):.3f}", flush=True)


if __name__ == "__main__":
    main()
