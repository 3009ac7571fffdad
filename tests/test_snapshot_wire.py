"""Snapshot wire format (include/kbgpu.h): encode / decode
round trips, validation of corrupt input, and (GPU) sessions opened from a
decoded snapshot make the same decisions as from the original."""
import ctypes
import os

import pytest

from helpers import compare_outputs, run_oracle  # noqa: F401
from kbgpu import _abi, synth
from kbgpu.cache import cache_from_fixture
from kbgpu.fixture import fixture_tiers
from kbgpu.snapshot import FlatSnapshot, SnapshotBlob, encode


def flat_of(fx):
    from kbgpu.api import RefPanic
    try:
        s = cache_from_fixture(fx).snapshot()
    except RefPanic:  # the fixture overcommits a node: the cache panics like the reference (AddPod)
        pytest.skip("cache panics on this fixture")
    return FlatSnapshot(s.nodes, s.jobs, s.queues, s.others, fixture_tiers(fx))


FIXTURES = ([("random", s) for s in range(0, 40, 4)] + [("affinity", s) for s in range(0, 20, 4)] +
            [("contended", s) for s in range(0, 20, 5)] + [("config", 1), ("config", 2)])


def make(kind, seed):
    return {"random": synth.random_fixture, "affinity": synth.affinity_fixture,
            "contended": synth.contended_fixture, "config": synth.config_fixture}[kind](seed)


@pytest.mark.parametrize("kind,seed", FIXTURES)
def test_round_trip_is_byte_identical(kind, seed):
    flat = flat_of(make(kind, seed))
    data = encode(flat.snap)
    assert data[:4] == b"KBGS"
    blob = SnapshotBlob.decode(data)
    assert blob.snap.n_tasks == flat.snap.n_tasks and blob.snap.n_nodes == flat.snap.n_nodes
    assert encode(blob.snap) == data
    blob.close()


def test_blob_view_keeps_its_owner_alive():
    """`SnapshotBlob.decode(...).snap` alone must stay valid: the view holds
    its blob (the library frees the arrays only when the blob goes away)."""
    import gc
    flat = flat_of(synth.config_fixture(1))
    data = encode(flat.snap)
    snap = SnapshotBlob.decode(data).snap
    gc.collect()
    assert encode(snap) == data


def test_save_and_load(tmp_path):
    flat = flat_of(synth.config_fixture(1))
    path = tmp_path / "c1.kbgs"
    _abi.check(_abi.lib().kbg_snapshot_save(ctypes.byref(flat.snap), str(path).encode()))
    blob = SnapshotBlob.load(path)
    assert encode(blob.snap) == encode(flat.snap) == path.read_bytes()
    blob.close()


def test_corrupt_input_is_rejected():
    keep = flat_of(synth.random_fixture(7))  # owns the arrays behind .snap
    data = bytearray(encode(keep.snap))
    for bad in (b"", data[:10], data[:-1], data + b"x", b"XXXX" + data[4:]):
        with pytest.raises(_abi.KbgError):
            SnapshotBlob.decode(bytes(bad))
    wrong_layout = bytearray(data)
    wrong_layout[8] ^= 0xFF  # the layout word (struct sizes)
    with pytest.raises(_abi.KbgError):
        SnapshotBlob.decode(bytes(wrong_layout))
    # inflated counts: rejected before anything is allocated (no bad_alloc, no OOM)
    for off in range(12, 12 + 4 * 23, 4):  # n_strings, then the 22 array counts
        big = bytearray(data)
        big[off:off + 4] = (0x7FFFFFFF).to_bytes(4, "little")
        with pytest.raises(_abi.KbgError):
            SnapshotBlob.decode(bytes(big))
    # a negative count in a snapshot: encode refuses it up front
    flat = flat_of(synth.random_fixture(7))
    flat.snap.n_taints = -1
    with pytest.raises(_abi.KbgError):
        encode(flat.snap)
    # a task pointing past the job table: decode validates like kbg_session_open
    flat = flat_of(synth.random_fixture(7))
    flat.arrays["tasks"][0]["job"] = 10_000
    with pytest.raises(_abi.KbgError):
        encode(flat.snap)


def _decisions(snap):
    L = _abi.lib()
    h = ctypes.c_void_p()
    opts = _abi.kbg_options()
    opts.device = 0
    _abi.check(L.kbg_session_open(ctypes.byref(snap), ctypes.byref(opts), ctypes.byref(h)))
    try:
        cap = max(1, snap.n_tasks)
        buf = (_abi.kbg_decision * cap)()
        n = ctypes.c_int32(0)
        code = L.kbg_allocate(h, buf, cap, ctypes.byref(n))
        return code, [(buf[i].task, buf[i].node, buf[i].kind, buf[i].dispatched_at) for i in range(n.value)]
    finally:
        L.kbg_session_close(h)


@pytest.mark.gpu
@pytest.mark.parametrize("kind,seed", FIXTURES + [("config", 3)])
def test_session_from_decoded_snapshot(kind, seed):
    flat = flat_of(make(kind, seed))
    blob = SnapshotBlob.decode(encode(flat.snap))
    assert _decisions(blob.snap) == _decisions(flat.snap)
    blob.close()
