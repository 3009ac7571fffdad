"""Parity of the MI355X path against the kbref oracle (run on the GPU box).

Decisions must be bit-exact (task -> node, Allocate/Pipeline kind, order,
gang dispatch); drf/proportion shares within 1e-12 relative.
"""
import copy

import pytest

from helpers import compare_outputs, load_golden, run_oracle

pytestmark = pytest.mark.gpu

kbgpu = pytest.importorskip("kbgpu")
from kbgpu import synth  # noqa: E402
from kbgpu.fixture import run_fixture  # noqa: E402


def device_available():
    from kbgpu import _abi
    return _abi.lib().kbg_device_count() > 0


@pytest.fixture(scope="module", autouse=True)
def _need_device():
    if not device_available():
        pytest.fail("no HIP device: the gpu tests must run on an MI355X (no CPU fallback)")


@pytest.mark.parametrize("case", ["ref_allocate_case1", "ref_allocate_case2"])
def test_reference_allocate_cases(case):
    """pkg/scheduler/actions/allocate/allocate_test.go:140-300, through the device path."""
    fx = load_golden(case + ".json")
    got, ssn = run_fixture(fx)
    assert got["status"] == "ok"
    assert got["binds"] == fx["expected"]["binds"]
    compare_outputs(run_oracle(fx), got)
    ssn.close()


def test_allocate_like_reference_test():
    """The allocate_test.go harness, verbatim in shape: cache -> OpenSession -> Execute -> binds."""
    from kbgpu import actions, framework
    from kbgpu.cache import FakeBinder, SchedulerCache
    from kbgpu.conf import PluginOption, Tier

    def res(cpu, mem):
        return {"cpu": cpu, "memory": mem, "nvidia.com/gpu": "0"}

    def pod(ns, n):
        return {"uid": f"{ns}-{n}", "namespace": ns, "name": n, "phase": "Pending",
                "annotations": {"scheduling.k8s.io/group-name": "pg1" if ns == "c1" else "pg2"},
                "containers": [{"requests": res("1", "1G")}]}

    binder = FakeBinder()
    cache = SchedulerCache(binder=binder)
    cache.add_node({"name": "n1", "allocatable": res("2", "4G")})
    for ns in ("c1", "c2"):
        for n in ("p1", "p2"):
            cache.add_pod(pod(ns, n))
    cache.add_pod_group({"namespace": "c1", "name": "pg1"})
    cache.add_pod_group({"namespace": "c2", "name": "pg2"})
    cache.add_queue({"name": "c1", "weight": 1})
    cache.add_queue({"name": "c2", "weight": 1})
    ssn = framework.open_session(cache, [Tier([PluginOption("drf"), PluginOption("proportion")])])
    actions.new().execute(ssn)
    framework.close_session(ssn)
    assert binder.binds == {"c2/p1": "n1", "c1/p1": "n1"}


@pytest.mark.parametrize("cid", [1, 2])
def test_config_parity(cid):
    fx = synth.config_fixture(cid)
    got, ssn = run_fixture(fx)
    compare_outputs(run_oracle(fx), got)
    ssn.close()


@pytest.mark.parametrize("opts", [
    {"batch_tasks": 1, "candidates": 1},
    {"batch_tasks": 7, "candidates": 2},
    {"batch_tasks": 64, "candidates": 4},
    {"batch_tasks": 4096, "candidates": 256},
    {"batch_tasks": 1, "candidates": 1, "full_scan": 1},
    {"batch_tasks": 7, "candidates": 2, "full_scan": 1},
    {"batch_tasks": 64, "candidates": 4, "full_scan": 1},
    {"batch_tasks": 2048, "candidates": 32, "full_scan": 1},
])
def test_batching_is_exact(opts):
    """Speculation, truncation and replay must not change any decision."""
    fx = synth.config_fixture(1)
    got, ssn = run_fixture(fx, opts)
    compare_outputs(run_oracle(fx), got)
    ssn.close()


@pytest.mark.parametrize("seed", range(300))
def test_fuzz_parity(seed):
    fx = synth.random_fixture(seed)
    ref = run_oracle(fx)
    got, ssn = run_fixture(fx, {"batch_tasks": 1 + seed % 9, "candidates": 1 + seed % 5, "full_scan": seed % 2})
    compare_outputs(ref, got)
    if ssn:
        ssn.close()


@pytest.mark.parametrize("seed", range(40))
def test_fuzz_parity_heap_rule(seed):
    fx = synth.random_fixture(1000 + seed, max_nodes=6, max_jobs=14, max_tasks=5)
    fx["options"] = {"heapDownRule": "go1.13"}
    got, ssn = run_fixture(fx)
    compare_outputs(run_oracle(fx), got)
    if ssn:
        ssn.close()


@pytest.mark.slow
@pytest.mark.parametrize("full_scan", [0, 1])
def test_config3_full_parity(full_scan, c3_oracle):
    """C3 (5k nodes x 100k tasks) end to end, every decision, both scan modes."""
    fx, ref = c3_oracle
    got, ssn = run_fixture(fx, {"full_scan": full_scan})
    compare_outputs(ref, got)
    ssn.close()


@pytest.fixture(scope="module")
def c3_oracle():
    fx = synth.config_fixture(3)
    return fx, run_oracle(fx)
