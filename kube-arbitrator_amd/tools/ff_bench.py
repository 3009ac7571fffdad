"""Developer tool: the fused first-fit kernel alone (kbg_tool_firstfit_bench),
median event-timed launch in microseconds on a config's table (default C3),
for full-scan and grouped batches of G rows. The event pair around a launch
adds about 4 us (an empty kernel of the same shape measures 4.1 us).
python kube-arbitrator_amd/tools/ff_bench.py [config]"""
import ctypes
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))


def one(cid):
    from kbgpu import _abi, synth
    from kbgpu.cache import FakeBinder, cache_from_fixture
    from kbgpu.fixture import _OrderedCache, fixture_tiers
    from kbgpu.snapshot import FlatSnapshot
    L = ctypes.CDLL(os.environ.get("TOOLS_LIB", os.path.join(HERE, "libkbg_tools.so")))
    L.kbg_tool_firstfit_bench.restype = ctypes.c_double
    fx = synth.config_fixture(cid)
    s = _OrderedCache(cache_from_fixture(fx, FakeBinder()), fx).snapshot()
    f = FlatSnapshot(s.nodes, s.jobs, s.queues, s.others, fixture_tiers(fx))
    res = {"config": cid}
    for full in (1, 0):
        for G in ((16, 64, 1024, 4096, 4174, 4655, 8192) if full else (16, 64, 256, 1024)):
            o = _abi.kbg_options()
            o.full_scan = full
            o.batch_tasks = 8192
            res[f"{'full' if full else 'grouped'}_{G}"] = round(
                L.kbg_tool_firstfit_bench(ctypes.byref(f.snap), ctypes.byref(o), G, 21), 2)
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    one(int(sys.argv[1]) if len(sys.argv) > 1 else 3)
