"""Developer tool: host cost of a fused launch and of its round trip, with and
without the kernel's start / stop events (GPU):
python kube-arbitrator_amd/tools/launch_cost.py [config]"""
import ctypes
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))


def main():
    cid = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    from kbgpu import _abi, synth
    from kbgpu.cache import cache_from_fixture
    from kbgpu.fixture import fixture_tiers
    from kbgpu.snapshot import FlatSnapshot
    fx = synth.config_fixture(cid)
    s = cache_from_fixture(fx).snapshot()
    flat = FlatSnapshot(s.nodes, s.jobs, s.queues, s.others, fixture_tiers(fx))
    L = ctypes.CDLL(os.environ.get("TOOLS_LIB", os.path.join(HERE, "libkbg_tools.so")))
    out = {"config": cid}
    for full in (0, 1):
        opts = _abi.kbg_options()
        opts.full_scan = full
        for G in (64, 1024, 8192):
            for untimed in (0, 1):
                lu, ru = ctypes.c_double(), ctypes.c_double()
                rows = L.kbg_tool_launch_cost(ctypes.byref(flat.snap), ctypes.byref(opts), G, 200, untimed,
                                              ctypes.byref(lu), ctypes.byref(ru))
                out[f"{'full' if full else 'grouped'}_{G}_{'untimed' if untimed else 'timed'}"] = \
                    {"rows": rows, "launch_us": round(lu.value, 2), "roundtrip_us": round(ru.value, 2)}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
