"""Run fuzz fixtures through the device and the oracle; print every mismatch.

Debug tool (GPU box): python tools/fuzz_diff.py [first] [last]
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "kube-arbitrator_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))

from helpers import compare_outputs, run_oracle  # noqa: E402
from kbgpu import synth  # noqa: E402
from kbgpu.fixture import run_fixture  # noqa: E402


def main():
    lo = int(sys.argv[1]) if len(sys.argv) > 1 else 0
    hi = int(sys.argv[2]) if len(sys.argv) > 2 else 300
    bad = 0
    for seed in range(lo, hi):
        fx = synth.random_fixture(seed)
        ref = run_oracle(fx)
        got, ssn = run_fixture(fx, {"batch_tasks": 1 + seed % 9, "candidates": 1 + seed % 5, "full_scan": seed % 2})
        try:
            compare_outputs(ref, got)
        except AssertionError as e:
            bad += 1
            print(f"== seed {seed} actions={fx.get('actions')} tiers={json.dumps(fx.get('tiers'))}: {e}")
            rd, gd = ref.get("decisions", []), got.get("decisions", [])
            for i in range(max(len(rd), len(gd))):
                a = rd[i] if i < len(rd) else None
                b = gd[i] if i < len(gd) else None
                print(f"  {i:3d} {'  ' if a == b else '!!'} ref={a} dev={b}")
            print("  ref evictions", ref.get("evictions"), "dev evictions", got.get("evictions"))
            if ssn is not None:
                try:
                    print("  stats", ssn.stats())
                except Exception as ex:  # noqa: BLE001
                    print("  stats n/a", ex)
        if ssn is not None:
            ssn.close()
    print(f"{bad} mismatching seeds in [{lo},{hi})")


if __name__ == "__main__":
    main()
