"""Test helpers: run the kbref oracle (the checker) and compare outputs."""
import json
import math
import os
import subprocess
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE = os.path.join(ROOT, "oracle", "build", "kbref")
GOLDEN = os.path.join(ROOT, "tests", "golden")


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


def close(a, b, rel=1e-12):
    if a == b:
        return True
    return abs(a - b) <= rel * max(abs(a), abs(b))


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
