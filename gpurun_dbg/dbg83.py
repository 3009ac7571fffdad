import json, sys
sys.path.insert(0, 'kube-arbitrator_amd'); sys.path.insert(0, 'tests')
from helpers import run_oracle
from kbgpu.fixture import run_fixture
for r in (0, 1):
    fx = json.load(open(f'gpurun_dbg/fx83_{r}.json'))
    ref = run_oracle(fx)
    for opts in ({"batch_tasks": 3, "candidates": 4, "full_scan": 1}, {}):
        got, ssn = run_fixture(fx, opts)
        rd, gd = ref.get("decisions", []), got.get("decisions", [])
        print("round", r, opts, ref["status"], got["status"], len(rd), len(gd), "evictions", len(ref.get("evictions", [])), len(got.get("evictions", [])))
        if rd != gd:
            print(" ref:", rd)
            print(" got:", gd)
            print(" ref ev:", ref.get("evictions"))
            print(" got ev:", got.get("evictions"))
        if ssn: ssn.close()
