"""Developer tool: timeline of one allocate cycle (KBG_TRACE) on the GPU.
python kube-arbitrator_amd/tools/trace_cycle.py [config] [full_scan] 2> trace.txt
(COMM=1: on a one-rank RCCL communicator, e.g. with KBG_SCAN_SERVICE=1)"""
import ctypes
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))


def main():
    cid = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    full = int(sys.argv[2]) if len(sys.argv) > 2 else 0
    from kbgpu import _abi, synth
    from kbgpu.cache import cache_from_fixture
    from kbgpu.fixture import fixture_tiers
    from kbgpu.framework import open_session
    fx = synth.config_fixture(cid)
    opts = {"device": 0, "full_scan": full}
    comm = None
    if os.environ.get("COMM") == "1":
        from kbgpu.dist import ShardComm
        comm = ShardComm(device=0, rank=0, world=1)
        opts["comm"] = comm
    ssn = open_session(cache_from_fixture(fx), fixture_tiers(fx), opts)
    L = _abi.lib()
    cap = max(1, ssn.flat.pending_count)
    buf = (_abi.kbg_decision * cap)()
    n = ctypes.c_int32(0)
    for i in range(4):
        if i == 3:
            os.environ["KBG_TRACE"] = "1"
        _abi.check(L.kbg_session_reset(ssn.handle))
        _abi.check(L.kbg_allocate(ssn.handle, buf, cap, ctypes.byref(n)))
        st = ssn.stats()
        print(f"cycle {i}: {n.value} decisions, allocate {st.allocate_ms:.3f} ms, engine {st.engine_ms:.3f}, "
              f"resolve {st.resolve_ms:.3f}, device {st.device_ms:.3f}, batches {st.batches}", flush=True)
    os.environ.pop("KBG_TRACE", None)
    ssn.close()
    if comm:
        comm.close()


if __name__ == "__main__":
    main()
