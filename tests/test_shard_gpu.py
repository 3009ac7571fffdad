"""Node-axis sharding against the kbref oracle, on the GPU box.

`shards=R` without a communicator keeps all R shards in one process: the
same scan geometry, slot layout and select walk as R GPUs exchanging their
slots over RCCL, with the slots written locally instead of all-gathered. A
one-rank RCCL communicator runs the all-gather itself. Decisions must stay
bit-exact for every shard count, including shards that hold no node.
"""
import pytest

from helpers import compare_outputs, run_oracle

pytestmark = pytest.mark.gpu

kbgpu = pytest.importorskip("kbgpu")
from kbgpu import synth  # noqa: E402
from kbgpu.fixture import run_fixture  # noqa: E402


@pytest.fixture(scope="module", autouse=True)
def _need_device():
    from kbgpu import _abi
    if _abi.lib().kbg_device_count() < 1:
        pytest.fail("no HIP device: the gpu tests must run on an MI355X (no CPU fallback)")


@pytest.mark.parametrize("shards", [2, 3, 8, 64])
@pytest.mark.parametrize("cid", [1, 2])
def test_local_shards_config_parity(cid, shards):
    fx = synth.config_fixture(cid)
    got, ssn = run_fixture(fx, {"shards": shards})
    assert ssn.stats().shards == shards and ssn.stats().shard_index == -1
    compare_outputs(run_oracle(fx), got)
    ssn.close()


@pytest.mark.parametrize("seed", range(0, 120, 2))
def test_local_shards_fuzz_parity(seed):
    fx = synth.random_fixture(seed)
    opts = {"shards": 2 + seed % 7, "batch_tasks": 1 + seed % 9, "candidates": 1 + seed % 5, "full_scan": seed % 4 == 0}
    opts["full_scan"] = int(opts["full_scan"])
    got, ssn = run_fixture(fx, opts)
    compare_outputs(run_oracle(fx), got)
    if ssn:
        ssn.close()


@pytest.mark.slow
def test_local_shards_config3():
    from helpers import compare_digests, digest_outputs, load_golden
    got, ssn = run_fixture(synth.config_fixture(3), {"shards": 8})
    ssn.close()
    compare_digests(load_golden("digest_c3.json"), digest_outputs(got))


@pytest.fixture(scope="module")
def comm1():
    from kbgpu.dist import ShardComm
    c = ShardComm(device=0, rank=0, world=1)
    yield c
    c.close()


@pytest.mark.parametrize("cid", [1, 2])
def test_rccl_one_rank_parity(cid, comm1):
    """The sharded entry point end to end: scan of the own slot, ncclAllGather
    in place, select over the gathered slots."""
    fx = synth.config_fixture(cid)
    got, ssn = run_fixture(fx, {"comm": comm1})
    st = ssn.stats()
    assert st.shards == 1 and st.shard_index == 0 and st.exchange_ms > 0.0
    compare_outputs(run_oracle(fx), got)
    ssn.close()


@pytest.mark.parametrize("seed", range(0, 40, 5))
def test_rccl_one_rank_fuzz(seed, comm1):
    fx = synth.random_fixture(seed)
    got, ssn = run_fixture(fx, {"comm": comm1, "batch_tasks": 1 + seed % 9, "candidates": 1 + seed % 5})
    compare_outputs(run_oracle(fx), got)
    if ssn:
        ssn.close()


@pytest.mark.parametrize("seed", range(0, 60, 6))
def test_rccl_one_rank_reclaim_preempt(seed, comm1):
    """Victim scans of a comm session: the shard's nodes, then ncclAllReduce(min)."""
    fx = synth.contended_fixture(seed)
    got, ssn = run_fixture(fx, {"comm": comm1})
    compare_outputs(run_oracle(fx), got)
    if ssn:
        ssn.close()


@pytest.mark.parametrize("seed", range(1, 60, 4))
def test_local_shards_reclaim_preempt(seed):
    fx = synth.contended_fixture(seed)
    got, ssn = run_fixture(fx, {"shards": 2 + seed % 5})
    compare_outputs(run_oracle(fx), got)
    if ssn:
        ssn.close()


def test_rccl_shard_count_must_match(comm1):
    fx = synth.config_fixture(1)
    got, ssn = run_fixture(fx, {"comm": comm1, "shards": 2})
    assert got["status"] == "invalid" and ssn is None


@pytest.mark.parametrize("seed", range(0, 60, 3))
def test_local_shards_affinity_parity(seed):
    """Pod-affinity mask deltas reach every shard's copy of the class masks."""
    fx = synth.affinity_fixture(seed)
    got, ssn = run_fixture(fx, {"shards": 2 + seed % 5, "batch_tasks": 1 + seed % 7})
    compare_outputs(run_oracle(fx), got)
    if ssn:
        ssn.close()


@pytest.mark.parametrize("seed", range(0, 40, 4))
def test_rccl_one_rank_affinity(seed, comm1):
    fx = synth.affinity_fixture(seed)
    got, ssn = run_fixture(fx, {"comm": comm1, "batch_tasks": 1 + seed % 5})
    compare_outputs(run_oracle(fx), got)
    if ssn:
        ssn.close()


@pytest.fixture
def owner_resolve(monkeypatch):
    """Allocate through the owner-resolve protocol (allocate_sharded) on the
    one-rank communicator: ncclBroadcast of the batch, the own-word select,
    the availability sum-reduce and the winner min-reduce rounds over RCCL."""
    monkeypatch.setenv("KBG_OWNER_RESOLVE", "1")


@pytest.mark.parametrize("cid", [1, 2])
def test_rccl_owner_resolve_parity(cid, comm1, owner_resolve):
    fx = synth.config_fixture(cid)
    got, ssn = run_fixture(fx, {"comm": comm1})
    st = ssn.stats()
    assert st.owner_rounds >= st.batches > 0 and st.exchange_ms > 0.0
    compare_outputs(run_oracle(fx), got)
    ssn.close()


@pytest.mark.parametrize("seed", range(0, 60, 3))
def test_rccl_owner_resolve_fuzz(seed, comm1, owner_resolve):
    fx = synth.random_fixture(seed)
    opts = {"comm": comm1, "batch_tasks": 1 + seed % 9, "candidates": 1 + seed % 5, "full_scan": seed % 2}
    got, ssn = run_fixture(fx, opts)
    compare_outputs(run_oracle(fx), got)
    if ssn:
        ssn.close()


@pytest.mark.parametrize("seed", range(0, 40, 4))
def test_rccl_owner_resolve_contended(seed, comm1, owner_resolve):
    """Allocate by owner-resolve inside a reclaim, allocate, backfill, preempt
    cycle (the victim actions keep the all-reduced stop maps)."""
    fx = synth.contended_fixture(seed)
    got, ssn = run_fixture(fx, {"comm": comm1})
    compare_outputs(run_oracle(fx), got)
    if ssn:
        ssn.close()


def test_rccl_local_failure_aborts_comm(monkeypatch):
    """A rank failing between two owner-resolve rounds aborts the communicator
    (its peers would otherwise block in the next collective forever): the
    failing call reports the local error, every later call on the
    communicator KBG_E_RCCL, and destroying it still works."""
    from kbgpu import _abi
    from kbgpu.dist import ShardComm
    monkeypatch.setenv("KBG_OWNER_RESOLVE", "1")
    fx = synth.config_fixture(1)
    c = ShardComm(device=0, rank=0, world=1)
    try:
        monkeypatch.setenv("KBG_TEST_FAULT", "push")
        with pytest.raises(_abi.KbgError) as e:
            run_fixture(fx, {"comm": c})
        assert e.value.status == "hip" and "injected" in str(e.value)
        monkeypatch.delenv("KBG_TEST_FAULT")
        got, ssn = run_fixture(fx, {"comm": c})
        assert got["status"] == "rccl" and ssn is None and "aborted" in got["error"]
    finally:
        c.close()


@pytest.fixture
def scan_service(monkeypatch):
    """Allocate through the scan service (allocate_svc_root) on the one-rank
    communicator: the launch messages' ncclBroadcasts, the own-word kernel into
    the (slot, rank) info column and [slot][W] masks, their ncclAllReduce."""
    monkeypatch.setenv("KBG_SCAN_SERVICE", "1")


@pytest.mark.parametrize("cid", [1, 2])
def test_rccl_scan_service_parity(cid, comm1, scan_service):
    fx = synth.config_fixture(cid)
    got, ssn = run_fixture(fx, {"comm": comm1})
    st = ssn.stats()
    assert st.shards == 1 and st.owner_rounds == 0 and st.scan_launches > 0
    compare_outputs(run_oracle(fx), got)
    ssn.close()


@pytest.mark.parametrize("seed", range(0, 60, 3))
def test_rccl_scan_service_fuzz(seed, comm1, scan_service):
    fx = synth.random_fixture(seed)
    opts = {"comm": comm1, "batch_tasks": 1 + seed % 9, "candidates": 1 + seed % 5, "full_scan": seed % 2}
    got, ssn = run_fixture(fx, opts)
    compare_outputs(run_oracle(fx), got)
    if ssn:
        ssn.close()


@pytest.mark.parametrize("seed", range(0, 40, 4))
def test_rccl_scan_service_contended(seed, comm1, scan_service):
    """The service's allocate inside a reclaim, allocate, backfill, preempt cycle."""
    fx = synth.contended_fixture(seed)
    got, ssn = run_fixture(fx, {"comm": comm1})
    compare_outputs(run_oracle(fx), got)
    if ssn:
        ssn.close()


@pytest.mark.parametrize("seed", range(0, 30, 5))
def test_rccl_scan_service_affinity(seed, comm1, scan_service):
    fx = synth.affinity_fixture(seed)
    got, ssn = run_fixture(fx, {"comm": comm1, "batch_tasks": 1 + seed % 5})
    compare_outputs(run_oracle(fx), got)
    if ssn:
        ssn.close()
