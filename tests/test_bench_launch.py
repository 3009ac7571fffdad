"""bench.py's `--gpus N` contract on the CPU (no device call: --dry-run stops
after the rendezvous): without a launcher bench.py starts N rank processes
itself, each with RANK / LOCAL_RANK / WORLD_SIZE, and the result line's
n_gpus is N; under a launcher whose world size differs from --gpus it exits
non-zero instead of reporting a different N."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(ROOT, "bench.py")


def _env(**extra):
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_PORT")}
    env.update(extra)
    return env


def test_gpus_two_starts_two_ranks():
    p = subprocess.run([sys.executable, BENCH, "--gpus", "2", "--dry-run"], capture_output=True, text=True,
                       timeout=300, env=_env())
    assert p.returncode == 0, p.stderr
    lines = [ln for ln in p.stdout.splitlines() if ln.strip()]
    assert len(lines) == 1, p.stdout
    line = json.loads(lines[0])
    assert line["n_gpus"] == 2 and line["ranks_reporting"] == 2
    assert "rank 0 of 2 (local rank 0)" in p.stderr and "rank 1 of 2 (local rank 1)" in p.stderr


def test_gpus_one_is_one_rank():
    p = subprocess.run([sys.executable, BENCH, "--dry-run"], capture_output=True, text=True, timeout=300, env=_env())
    assert p.returncode == 0, p.stderr
    assert json.loads(p.stdout.strip())["n_gpus"] == 1


def test_launcher_world_size_must_match():
    p = subprocess.run([sys.executable, BENCH, "--gpus", "2", "--dry-run"], capture_output=True, text=True,
                       timeout=300, env=_env(RANK="0", LOCAL_RANK="0", WORLD_SIZE="3", MASTER_ADDR="127.0.0.1",
                                             MASTER_PORT="29555"))
    assert p.returncode != 0
    assert "WORLD_SIZE=3" in p.stderr and not p.stdout.strip()


def test_parity_verdict_against_golden_digest():
    """bench.py's own parity check: the oracle's C1 output digested as the
    bench digests its timed cycles matches tests/golden/digest_c1.json, and a
    perturbed decision log or share is reported (and would exit non-zero)."""
    import importlib.util
    from helpers import run_oracle
    spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(ROOT, "bench.py"))
    bench = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(bench)
    sys.path.insert(0, os.path.join(ROOT, "kube-arbitrator_amd"))
    from kbgpu import synth
    from kbgpu.digest import digest_outputs
    dg = digest_outputs(run_oracle(synth.config_fixture(1)))
    v = bench.parity_verdict(1, {"production": dg, "full_scan": dg})
    assert v["ok"] is True and v["production"] is True and v["full_scan"] is True
    bad = dict(dg, binds="0" * 64)
    v = bench.parity_verdict(1, {"production": dg, "full_scan": bad})
    assert v["ok"] is False and v["full_scan"] == {"mismatch": ["binds"]}
    assert bench.parity_verdict(99, {"production": dg})["ok"] is None  # no golden digest for the config
