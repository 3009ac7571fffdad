"""The resolver's whole-word re-checks (kube-arbitrator_amd/csrc/kbg_walk.cpp,
AVX-512 on the host) against the node-by-node checks they replace — res_le
(Resource.LessEqual with its tolerances, resource_info.go:142-146), the pod
cap (predicates.go:125-127), the touched-since-scan and panic-node tests — on
seeded random words with values on and beside the tolerance edges. Bit-exact:
the word checks use the same IEEE compares, subtractions and absolute values."""
import ctypes
import os
import subprocess

import pytest

from helpers import ROOT

PKG = os.path.join(ROOT, "kube-arbitrator_amd")


def test_word_checks_match_node_checks():
    subprocess.run(["make", "-s", "-C", PKG, "tools"], check=True)
    L = ctypes.CDLL(os.path.join(PKG, "tools", "libkbg_tools.so"))
    L.kbg_tool_walk_check.restype = ctypes.c_int64
    bad = L.kbg_tool_walk_check(ctypes.c_uint64(20261017), 20000)
    if bad == -1:
        pytest.skip("no AVX-512 on this CPU: the library walks node by node")
    assert bad == 0
