"""Test helpers: run the kbref oracle (the checker) and compare outputs."""
import json
import os
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE = os.path.join(ROOT, "oracle", "build", "kbref")
GOLDEN = os.path.join(ROOT, "tests", "golden")
sys.path.insert(0, os.path.join(ROOT, "kube-arbitrator_amd"))

from kbgpu.digest import close, digest_mismatches, digest_outputs  # noqa: E402,F401


def ensure_oracle():
    if not os.path.exists(ORACLE):
        subprocess.run(["make", "-C", os.path.join(ROOT, "oracle")], check=True, capture_output=True)
    return ORACLE


def run_oracle(fx, *flags):
    ensure_oracle()
    with tempfile.TemporaryDirectory() as d:
        src = os.path.join(d, "fx.json")
        dst = os.path.join(d, "out.json")
        with open(src, "w") as f:
            json.dump(fx, f)
        subprocess.run([ORACLE, *flags, src, "-o", dst], check=True)
        with open(dst) as f:
            return json.load(f)


def load_golden(name):
    with open(os.path.join(GOLDEN, name)) as f:
        return json.load(f)


def compare_outputs(ref, got):
    """Bit-exact decisions (task, node, kind, order, dispatch), gang readiness
    and node state; drf/proportion shares within 1e-12 relative (north star)."""
    assert got["status"] == ref["status"], (ref.get("error"), got.get("error"))
    if ref["status"] != "ok":
        return
    rd, gd = ref["decisions"], got["decisions"]
    for i, (a, b) in enumerate(zip(rd, gd)):
        assert a == b, f"decision {i}: oracle {a} != device {b}"
    assert len(rd) == len(gd)
    assert ref["binds"] == got["binds"]
    assert ref.get("evictions", []) == got.get("evictions", [])
    assert [(j["uid"], j["ready_num"], j["ready"]) for j in ref["jobs"]] == \
           [(j["uid"], j["ready_num"], j["ready"]) for j in got["jobs"]]
    for a, b in zip(ref["jobs"], got["jobs"]):
        assert a["allocated"] == b["allocated"], (a, b)
        if not a["ready"]:  # gang reports FitError for jobs that are not ready (gang.go:169-190)
            assert b.get("fit_error") == a["fit_error"], (a, b)
        if "drf_share" in a:
            assert close(a["drf_share"], b["drf_share"]), (a, b)
    assert sorted(q["uid"] for q in ref["queues"]) == sorted(q["uid"] for q in got["queues"])
    gq = {q["uid"]: q for q in got["queues"]}
    for a in ref["queues"]:
        b = gq[a["uid"]]
        assert close(a["share"], b["share"]), (a, b)
        for k in ("deserved", "allocated", "request"):
            assert all(close(x, y) for x, y in zip(a[k], b[k])), (k, a, b)
    for a, b in zip(ref["nodes"], got["nodes"]):
        assert a["name"] == b["name"] and a["ntasks"] == b["ntasks"], (a, b)
        assert a["idle"] == b["idle"] and a["releasing"] == b["releasing"], (a, b)


def compare_digests(ref, got):
    """Digests (kbgpu.digest.digest_outputs) of sessions too large to keep the
    oracle's whole output under tests/golden (C3, C4, C5)."""
    assert not digest_mismatches(ref, got), digest_mismatches(ref, got)


def churn_chain(fx0, seed, rounds, run):
    """Resident-session churn of a seeded session (synth.churn, the events of
    tests/test_update_gpu.py): yields (r, changes, fx_r, out_r) for r = 0 ..
    rounds, where fx_0 is `fx0` in its session order, fx_{r+1}
    the cache after round r's events `changes` — the binds of out_r's
    Allocate decisions, completions, deletions, new pods, node growth — and
    out_r = run(fx_r, changes) in the oracle's output schema (the oracle itself in
    make_digests.py, the device on the GPU box: the same chain whenever the
    two agree on every decision)."""
    import sys
    sys.path.insert(0, os.path.join(ROOT, "kube-arbitrator_amd"))
    from kbgpu import synth
    from kbgpu.cache import FakeBinder, cache_from_fixture
    from kbgpu.fixture import _OrderedCache
    snap = _OrderedCache(cache_from_fixture(fx0, FakeBinder()), fx0).snapshot()
    fx = dict(fx0, sessionOrder={"jobs": [j.uid for j in snap.jobs], "nodes": [n.name for n in snap.nodes]})
    uids = {t.uid for j in snap.jobs for t in j.tasks.values()}
    changes = []
    for r in range(rounds + 1):
        out = run(fx, changes)
        yield r, changes, fx, out
        if r == rounds or out["status"] != "ok":
            return
        changes, fx = synth.churn(fx, seed * 31 + r, uids, out["decisions"])
        uids |= {p["uid"] for kind, p in changes if kind == "pod_add"}


def build_tools():
    """`make tools` (the CPU tool library) under a file lock: parallel test
    workers must not relink the library while another loads it."""
    import fcntl
    import subprocess
    pkg = os.path.join(ROOT, "kube-arbitrator_amd")
    with open(os.path.join(pkg, "tools", ".build.lock"), "w") as f:
        fcntl.flock(f, fcntl.LOCK_EX)
        subprocess.run(["make", "-s", "-C", pkg, "tools"], check=True)
        return os.path.join(pkg, "tools", "libkbg_tools.so")
