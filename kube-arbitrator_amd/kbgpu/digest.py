"""Size-independent digests of a session's outputs (the kbref oracle's output
schema: decision log, binds, evictions, node / job / queue states).

The golden digests under tests/golden/digest_*.json hold the oracle's digest
of a seeded session; a device run is checked against one without running the
oracle: bit-exact fields as sha256 of their canonical JSON, drf / proportion
shares kept as numbers and compared within 1e-12 relative (BASELINE north
star). Used by the parity tests and by bench.py, which checks the decision log
of its last timed cycle in each mode.
"""
import hashlib
import json

EXACT_FIELDS = ("n_decisions", "decisions", "binds", "evictions", "nodes", "jobs")


def _h(x):
    return hashlib.sha256(json.dumps(x, separators=(",", ":")).encode()).hexdigest()


def _f(v):  # the oracle prints integral doubles without a fraction: hash every resource as a float
    return [float(x) for x in v]


def digest_outputs(out):
    d = {"status": out["status"]}
    if out["status"] != "ok":
        return d
    d["n_decisions"] = len(out["decisions"])
    d["decisions"] = _h([[x["task"], x["job"], x["node"], x["kind"], x["dispatched_at"], x.get("action", "")]
                         for x in out["decisions"]])
    d["binds"] = _h(sorted(out["binds"].items()))
    d["evictions"] = _h(out.get("evictions", []))
    d["nodes"] = _h([[n["name"], _f(n["idle"]), _f(n["releasing"]), n["ntasks"]] for n in out["nodes"]])
    d["jobs"] = _h([[j["uid"], j["ready_num"], j["ready"], _f(j["allocated"]), None if j["ready"] else j["fit_error"]]
                    for j in out["jobs"]])
    d["drf_shares"] = [j["drf_share"] for j in out["jobs"] if "drf_share" in j]
    d["queues"] = sorted(([q["uid"], q["share"], q["deserved"], q["allocated"], q["request"]] for q in out["queues"]))
    return d


def close(a, b, rel=1e-12):
    if a == b:
        return True
    return abs(a - b) <= rel * max(abs(a), abs(b))


def digest_mismatches(ref, got):
    """The fields in which digest `got` differs from `ref` (empty: parity)."""
    if got.get("status") != ref.get("status"):
        return ["status"]
    if ref["status"] != "ok":
        return []
    bad = [k for k in EXACT_FIELDS if got.get(k) != ref.get(k)]
    rs, gs = ref["drf_shares"], got.get("drf_shares", [])
    if len(rs) != len(gs) or not all(close(a, b) for a, b in zip(rs, gs)):
        bad.append("drf_shares")
    rq, gq = ref["queues"], got.get("queues", [])
    if [q[0] for q in rq] != [q[0] for q in gq] or not all(
            close(a[1], b[1]) and all(close(x, y) for u, v in zip(a[2:], b[2:]) for x, y in zip(u, v))
            for a, b in zip(rq, gq)):
        bad.append("queues")
    return bad
