"""Developer tool: A/B of host-engine builds (tools libraries built with
different compile-time options) on one snapshot, alternating in one process.
python kube-arbitrator_amd/tools/engine_ab.py CONFIG lib1.so lib2.so ..."""
import ctypes
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))


def main():
    cid = int(sys.argv[1])
    libs = sys.argv[2:]
    from kbgpu import _abi, synth
    from kbgpu.cache import cache_from_fixture
    from kbgpu.fixture import fixture_tiers
    from kbgpu.snapshot import FlatSnapshot
    fx = synth.config_fixture(cid)
    s = cache_from_fixture(fx).snapshot()
    flat = FlatSnapshot(s.nodes, s.jobs, s.queues, s.others, fixture_tiers(fx))
    opts = _abi.kbg_options()
    loaded = []
    for p in libs:
        L = ctypes.CDLL(os.path.abspath(p))
        L.kbg_tool_engine_ns_per_step.restype = ctypes.c_double
        loaded.append((p, L))
    best = {p: 1e30 for p in libs}
    for rnd in range(int(os.environ.get("ROUNDS", "4"))):
        for p, L in loaded:
            steps, chk = ctypes.c_int64(), ctypes.c_double()
            ns = L.kbg_tool_engine_ns_per_step(ctypes.byref(flat.snap), ctypes.byref(opts), 3, ctypes.byref(steps),
                                               ctypes.byref(chk), 0)
            best[p] = min(best[p], ns)
            print(f"C{cid} round {rnd} {os.path.basename(p)}: {ns:.1f} ns/step (checksum {chk.value:.0f})", flush=True)
    for p in libs:
        print(f"C{cid} best {os.path.basename(p)}: {best[p]:.1f} ns/step")


if __name__ == "__main__":
    main()
