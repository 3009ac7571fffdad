"""Developer tool: host-side timing of kbg_session_update (event application +
derive phases) on a churn step of a BASELINE config, without a device.
KBG_PROFILE_OPEN=1 python kube-arbitrator_amd/tools/update_profile.py [config] [churn]
(DECISIONS_CACHE=file.json keeps the oracle cycle's decisions between runs)"""
import ctypes
import json
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.dirname(HERE)
ROOT = os.path.dirname(PKG)
sys.path.insert(0, PKG)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def main():
    cid = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    churn = float(sys.argv[2]) if len(sys.argv) > 2 else 0.01
    os.environ["KBG_TOOL_TIME"] = "1"
    subprocess.run(["make", "-s", "-C", PKG, "tools"], check=True)
    from kbgpu import _abi, synth
    from helpers import run_oracle
    from test_update_host import events, flat
    fx = synth.config_fixture(cid)
    f0, s0 = flat(fx)
    # binds of the first `churn` share of the cycle's decisions (NO_ORACLE=1: new pods only)
    decided = []
    if not os.environ.get("NO_ORACLE"):
        cache = os.environ.get("DECISIONS_CACHE")  # a JSON file: the oracle's decisions, kept between runs
        if cache and os.path.exists(cache):
            with open(cache) as f:
                dec = json.load(f)
        else:
            dec = run_oracle(fx, "--threads", str(min(8, os.cpu_count() or 1)))["decisions"]
            if cache:
                with open(cache, "w") as f:
                    json.dump(dec, f)
        decided = dec[:int(churn * len(dec))]
    uids = {t.uid for t in f0.task_objs}
    changes, _ = synth.churn(fx, 5, uids, decided, bind=1.0, done=churn, delete=0.0, add=churn, node_frac=0.0)
    evs, keep, tidx = events(f0, changes)
    L = ctypes.CDLL(os.environ.get("TOOLS_LIB", os.path.join(HERE, "libkbg_tools.so")))
    N = len(f0.node_names)
    idle, rel = (ctypes.c_double * (3 * N))(), (ctypes.c_double * (3 * N))()
    nt = (ctypes.c_int32 * N)()
    pend = (ctypes.c_int32 * max(1, len(tidx)))()
    npend = ctypes.c_int32()
    for _ in range(3):
        rc = L.kbg_tool_update_nodes(ctypes.byref(f0.snap), ctypes.byref(_abi.kbg_options()), evs, len(changes), idle,
                                     rel, nt, pend, ctypes.byref(npend))
        print(f"C{cid}: {len(changes)} events, rc {rc}", flush=True)


if __name__ == "__main__":
    main()
