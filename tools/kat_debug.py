"""Debug helper (GPU box): one fixture through the device, with its stats."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "kube-arbitrator_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))

from helpers import load_golden, run_oracle  # noqa: E402
from kbgpu.fixture import run_fixture  # noqa: E402

fx = load_golden(sys.argv[1])
opts = json.loads(sys.argv[2]) if len(sys.argv) > 2 else None
got, ssn = run_fixture(fx, opts)
ref = run_oracle(fx)
print("ref", ref["status"], [(d["task"], d["node"]) for d in ref["decisions"]])
print("dev", got["status"], got.get("error"), [(d["task"], d["node"]) for d in got["decisions"]])
if ssn:
    st = ssn.stats()
    print({k: getattr(st, k) for k, _ in st._fields_})
