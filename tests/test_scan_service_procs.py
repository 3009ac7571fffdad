"""The node-axis sharded session across real processes on the
MI355X: R processes (tests/svc_procs_worker.py), each with its own device
session on GPU 0 holding shard r of R, joined by the host transport
(kbgpu.h kbg_comm_init_host: the same collectives the RCCL transport runs,
through POSIX shared memory). This is the code `bench.py --gpus N` runs on N
GPUs, minus RCCL itself (RCCL refuses two ranks on one device):

- allocate through the scan service (kbg_session.cpp allocate_svc_root /
  allocate_serve): rank 0's launch messages — header then payload broadcast
  from its 4-slot pinned ring —, every rank's own-word kbg_firstfit_kernel,
  the grouped sum-reduce of info words and word masks, rank 0's commits
  replayed on the other ranks' Logger / Replayer threads, the FitError counts
  summed at the end (sum_host);
- backfill's all-gathered bitmap slots and reclaim / preempt's max-reduced
  victim-scan words (the contended fixtures run reclaim, allocate, backfill,
  preempt);
- the owner-resolve protocol (KBG_OWNER_RESOLVE=1) on the same transport.

Every rank's outputs must equal the oracle's (allocate.go:119-162 and the
other actions), or its committed digest at C2 / C3 / the saturated C3-scale
session. The failure cases: a rank that exits mid-cycle (fault injection
KBG_HOST_COMM_EXIT_AFTER) makes every other rank return KBG_E_RCCL within
seconds, whether it is a serving rank or rank 0.
"""
import json
import os
import subprocess
import sys
import time
import uuid

import pytest

from helpers import ROOT, compare_outputs, load_golden, run_oracle

pytestmark = pytest.mark.gpu

kbgpu = pytest.importorskip("kbgpu")
from kbgpu import _abi, synth  # noqa: E402
from kbgpu.digest import digest_mismatches  # noqa: E402

WORKER = os.path.join(ROOT, "tests", "svc_procs_worker.py")


@pytest.fixture(scope="module", autouse=True)
def _need_device():
    if _abi.lib().kbg_device_count() < 1:
        pytest.fail("no HIP device: the gpu tests must run on an MI355X (no CPU fallback)")


def run_ranks(tmp_path, R, cases, env_of=lambda r: {}, timeout=240):
    """Runs the R ranks over `cases`; returns (per-rank results or None, exit codes, logs)."""
    name = f"p{os.getpid()}-{uuid.uuid4().hex[:10]}"
    cpath = tmp_path / "cases.json"
    cpath.write_text(json.dumps(cases))
    procs, outs, logs = [], [], []
    for r in range(R):
        out = tmp_path / f"out{r}.json"
        log = open(tmp_path / f"rank{r}.log", "w")
        env = dict(os.environ, **env_of(r))
        procs.append(subprocess.Popen([sys.executable, "-u", WORKER, name, str(R), str(r), str(cpath), str(out)],
                                      stdout=log, stderr=subprocess.STDOUT, env=env, cwd=ROOT))
        outs.append(out)
        logs.append(tmp_path / f"rank{r}.log")
    t0 = time.time()
    codes = []
    try:
        for p in procs:
            codes.append(p.wait(timeout=max(1.0, timeout - (time.time() - t0))))
    except subprocess.TimeoutExpired:
        for p in procs:
            p.kill()
        for p in procs:
            p.wait()
        raise AssertionError("ranks hung: " + " | ".join(open(x).read()[-400:] for x in logs))
    res = [json.loads(o.read_text()) if o.exists() else None for o in outs]
    return res, codes, [open(x).read() for x in logs]


def check_ranks(res, codes, logs, R, cases):
    assert codes == [0] * R, (codes, [lg[-1500:] for lg in logs])
    for r in range(R):
        assert [x["id"] for x in res[r]] == [c["id"] for c in cases]
        for x in res[r]:
            if "stats" in x:
                assert x["stats"]["shards"] == R and x["stats"]["shard_index"] == r, x["stats"]
            assert x.get("cycles_equal", True), (r, x["id"])


def oracle_cases(cases):
    from svc_procs_worker import make_fixture
    return {c["id"]: run_oracle(make_fixture(c)) for c in cases if not c.get("digest")}


def compare_all(res, cases, refs, R):
    for c, *per_rank in zip(cases, *res):
        for r, x in enumerate(per_rank):
            if c.get("digest"):
                bad = digest_mismatches(load_golden(c["digest"]), x["out"])
                assert not bad, (c["id"], r, bad)
            else:
                try:
                    compare_outputs(refs[c["id"]], x["out"])
                except AssertionError as e:
                    raise AssertionError(f"{c['id']} rank {r}/{R}: {e}") from e


SMALL = [
    {"id": "c1", "gen": "config", "arg": 1},
    {"id": "c1-full", "gen": "config", "arg": 1, "opts": {"full_scan": 1}},
    {"id": "c2-digest", "gen": "config", "arg": 2, "digest": "digest_c2.json"},
]
FUZZ = (
    [{"id": f"random-{s}", "gen": "random", "arg": 15000 + s, "allocate_only": True,
      "opts": {"batch_tasks": 1 + s % 9, "candidates": 1 + s % 4, "full_scan": s % 2}} for s in range(0, 12, 3)] +
    [{"id": f"contended-{s}", "gen": "contended", "arg": 16000 + s, "kw": {"nodes": 200, "jobs": 40, "tasks": 12},
      "allocate_only": True} for s in range(1, 12, 5)] +
    [{"id": f"actions-{s}", "gen": "contended", "arg": s} for s in range(0, 16, 5)] +  # reclaim/allocate/backfill/preempt
    [{"id": f"affinity-{s}", "gen": "affinity", "arg": s, "allocate_only": True,
      "opts": {"batch_tasks": 1 + s % 7}} for s in range(0, 9, 3)] +
    [{"id": f"ports-{s}", "gen": "contended", "arg": 8000 + s, "kw": {"nodes": 12, "jobs": 14, "tasks": 8, "ports": 0.4},
      "allocate_only": True} for s in (0, 3)]
)


@pytest.mark.parametrize("R", [2, 4])
def test_procs_configs(tmp_path, R):
    """C1 (both scan modes) against the oracle and C2 against its digest, on
    every rank."""
    refs = oracle_cases(SMALL)
    res, codes, logs = run_ranks(tmp_path, R, SMALL)
    check_ranks(res, codes, logs, R, SMALL)
    compare_all(res, SMALL, refs, R)
    for r in range(R):
        assert res[r][0]["stats"]["scan_launches"] > 0 and res[r][0]["stats"]["owner_rounds"] == 0


@pytest.mark.parametrize("R", [2, 4])
def test_procs_fuzz(tmp_path, R):
    """16 random, contended, full-action, pod-affinity and host-port sessions
    (the scan service, backfill's all-gather, the victim scans' max-reduce)."""
    refs = oracle_cases(FUZZ)
    cases = [c for c in FUZZ if refs[c["id"]]["status"] in ("ok", "ref_panic")]
    assert len(cases) >= 12
    res, codes, logs = run_ranks(tmp_path, R, cases)
    check_ranks(res, codes, logs, R, cases)
    compare_all(res, cases, refs, R)


@pytest.mark.parametrize("R", [2, 4])
def test_procs_saturated_two_cycles(tmp_path, R):
    """C3's cluster filling up mid-cycle (mispredictions, contended rescans,
    reused lists on rank 0, every scan served by the ranks), against
    tests/golden/digest_saturated.json; a second cycle on the reset sessions
    must reproduce the first's log on every rank."""
    cases = [{"id": "saturated", "gen": "saturated", "digest": "digest_saturated.json", "cycles": 2}]
    res, codes, logs = run_ranks(tmp_path, R, cases)
    check_ranks(res, codes, logs, R, cases)
    compare_all(res, cases, {}, R)


@pytest.mark.slow
@pytest.mark.parametrize("R", [2, 4])
def test_procs_config3(tmp_path, R):
    """The bench workload (BASELINE C3: 5k nodes x 100k tasks) against
    tests/golden/digest_c3.json on every rank."""
    cases = [{"id": "c3", "gen": "config", "arg": 3, "digest": "digest_c3.json"}]
    res, codes, logs = run_ranks(tmp_path, R, cases, timeout=400)
    check_ranks(res, codes, logs, R, cases)
    compare_all(res, cases, {}, R)


def test_procs_owner_resolve(tmp_path):
    """The owner-resolve protocol (KBG_OWNER_RESOLVE=1) across 3 processes."""
    cases = [c for c in SMALL if not c.get("digest")] + FUZZ[:4]
    refs = oracle_cases(cases)
    res, codes, logs = run_ranks(tmp_path, 3, cases, env_of=lambda r: {"KBG_OWNER_RESOLVE": "1"})
    check_ranks(res, codes, logs, 3, cases)
    compare_all(res, cases, refs, 3)
    assert res[0][0]["stats"]["owner_rounds"] > 0


@pytest.mark.parametrize("dead", [1, 0])
def test_procs_rank_exit_mid_cycle(tmp_path, dead):
    """Rank `dead` exits at its 6th collective, inside C2's allocate (a
    serving rank, or rank 0 with its launch messages): every other rank's
    allocate returns KBG_E_RCCL within seconds, naming the rank that left."""
    R = 3
    cases = [{"id": "c2", "gen": "config", "arg": 2, "digest": "digest_c2.json"}]
    t0 = time.time()
    res, codes, logs = run_ranks(tmp_path, R, cases, timeout=120,
                                 env_of=lambda r: {"KBG_HOST_COMM_EXIT_AFTER": "6"} if r == dead else
                                 {"KBG_COMM_TIMEOUT_MS": "60000"})
    assert time.time() - t0 < 90
    assert codes[dead] == 3 and res[dead] is None, (codes, logs[dead][-800:])
    for r in range(R):
        if r == dead:
            continue
        assert codes[r] == 0, (r, logs[r][-1500:])
        out = res[r][0]["out"]
        assert out["status"] == "rccl", (r, out)
