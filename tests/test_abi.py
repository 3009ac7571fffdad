"""The C-ABI library loads, exports every symbol include/kbgpu.h declares, and
its struct layouts match the ctypes mirror (CPU; no compute calls)."""
import ctypes
import os
import re
import subprocess

import pytest

from helpers import ROOT

HEADER = os.path.join(ROOT, "include", "kbgpu.h")


def declared_functions():
    txt = open(HEADER).read()
    return sorted(set(re.findall(r"^\s*(?:kbg_status|int32_t|const char\*|const kbg_snapshot\*|void)\s+(kbg_\w+)\s*\(",
                                 txt, re.M)))


def test_header_declares_functions():
    fns = declared_functions()
    assert "kbg_session_open" in fns and "kbg_allocate" in fns and len(fns) >= 12


def test_library_exports_every_declared_symbol():
    from kbgpu import _abi
    L = _abi.lib()
    for fn in declared_functions():
        assert hasattr(L, fn), fn
    assert set(declared_functions()) == set(_abi.SIGNATURES)
    assert L.kbg_abi_version() == _abi.ABI_VERSION == 13
    assert L.kbg_device_count() >= 0


STRUCTS = ["kbg_resource", "kbg_node", "kbg_host_port", "kbg_taint", "kbg_job", "kbg_queue", "kbg_task", "kbg_spec", "kbg_pod_term", "kbg_term",
           "kbg_requirement", "kbg_toleration", "kbg_plugin_option", "kbg_snapshot", "kbg_options", "kbg_decision",
           "kbg_job_state", "kbg_queue_state", "kbg_node_state", "kbg_stats", "kbg_eviction", "kbg_event"]


def test_struct_layouts_match_c(tmp_path):
    from kbgpu import _abi
    lines = ["#include <stdio.h>", "#include <stddef.h>", '#include "kbgpu.h"', "int main(void){"]
    for s in STRUCTS:
        cls = getattr(_abi, s)
        lines.append(f'printf("{s} %zu\\n", sizeof({s}));')
        for fname, _ in cls._fields_:
            lines.append(f'printf("{s}.{fname} %zu\\n", offsetof({s}, {fname}));')
    lines.append("return 0;}")
    src = tmp_path / "layout.c"
    src.write_text("\n".join(lines))
    exe = tmp_path / "layout"
    subprocess.run(["gcc", "-I", os.path.join(ROOT, "include"), str(src), "-o", str(exe)], check=True)
    got = dict(l.split() for l in subprocess.run([str(exe)], check=True, capture_output=True, text=True).stdout.split("\n") if l)
    for s in STRUCTS:
        cls = getattr(_abi, s)
        assert int(got[s]) == ctypes.sizeof(cls), s
        for fname, _ in cls._fields_:
            assert int(got[f"{s}.{fname}"]) == getattr(cls, fname).offset, (s, fname)


def test_open_without_device_fails_loudly():
    from kbgpu import _abi
    L = _abi.lib()
    if L.kbg_device_count() > 0:
        pytest.skip("a device is present")
    h = ctypes.c_void_p()
    snap = _abi.kbg_snapshot()
    code = L.kbg_session_open(ctypes.byref(snap), None, ctypes.byref(h))
    assert code == _abi.KBG_E_HIP
    assert b"device" in L.kbg_last_error()
    assert not h.value


def test_invalid_snapshot_rejected():
    from kbgpu import _abi
    L = _abi.lib()
    h = ctypes.c_void_p()
    snap = _abi.kbg_snapshot()
    jobs = (_abi.kbg_job * 1)()
    jobs[0].queue = 5  # no queues
    snap.jobs = ctypes.cast(jobs, ctypes.POINTER(_abi.kbg_job))
    snap.n_jobs = 1
    strs = (ctypes.c_char_p * 1)(b"j")
    snap.strings = ctypes.cast(strs, ctypes.POINTER(ctypes.c_char_p))
    snap.n_strings = 1
    assert L.kbg_session_open(ctypes.byref(snap), None, ctypes.byref(h)) == _abi.KBG_E_INVALID


def _registry_session(extra_plugin, registered, registry=1, drop_flag=()):
    """C1's session with `extra_plugin` added to the first tier; every entry's
    KBG_PLUGIN_REGISTERED flag as the caller's registry says."""
    from kbgpu import _abi, synth
    from kbgpu.cache import FakeBinder, cache_from_fixture
    from kbgpu.conf import PluginOption, Tier
    from kbgpu.fixture import _OrderedCache, fixture_tiers
    from kbgpu.snapshot import FlatSnapshot
    fx = synth.config_fixture(1)
    tiers = fixture_tiers(fx)
    tiers = [Tier(list(tiers[0].plugins) + [PluginOption(extra_plugin)])] + list(tiers[1:])
    s = _OrderedCache(cache_from_fixture(fx, FakeBinder()), fx).snapshot()
    flat = FlatSnapshot(s.nodes, s.jobs, s.queues, s.others, tiers,
                        registered=lambda n: n in registered and n not in drop_flag)
    o = _abi.kbg_options()
    o.device = -1
    o.plugin_registry = registry
    return flat, o


@pytest.mark.parametrize("registry", [0, 1])
def test_registered_unknown_plugin_refuses_the_session(registry):
    """framework.go:30-35: a tier entry with a builder in the caller's process
    is instantiated. One this path does not implement must not be dropped
    silently: kbg_session_open refuses (KBG_E_UNSUPPORTED) before any device
    work; with plugin_registry = 0 the library cannot know, and skips it."""
    from kbgpu import _abi
    L = _abi.lib()
    known = {"priority", "gang", "drf", "predicates", "proportion"}
    flat, o = _registry_session("binpack", known | {"binpack"}, registry)
    h = ctypes.c_void_p()
    code = L.kbg_session_open(ctypes.byref(flat.snap), ctypes.byref(o), ctypes.byref(h))
    if registry:
        assert code == _abi.KBG_E_UNSUPPORTED and b"binpack" in L.kbg_last_error()
    else:
        assert code in (_abi.KBG_OK, _abi.KBG_E_HIP)  # accepted (no device here: the open then stops at HIP)
    if h.value:
        L.kbg_session_close(h)


def test_unregistered_plugins_are_skipped():
    """A name without a builder is skipped like GetPluginBuilder's miss
    (framework.go:30-35), whether or not this path implements it: the open
    proceeds to the device."""
    from kbgpu import _abi
    L = _abi.lib()
    known = {"priority", "gang", "drf", "predicates", "proportion"}
    for extra, drop in (("binpack", ()), ("nodeorder", ("gang",))):
        flat, o = _registry_session(extra, known, 1, drop_flag=drop)
        h = ctypes.c_void_p()
        code = L.kbg_session_open(ctypes.byref(flat.snap), ctypes.byref(o), ctypes.byref(h))
        assert code in (_abi.KBG_OK, _abi.KBG_E_HIP), L.kbg_last_error()
        if h.value:
            L.kbg_session_close(h)
