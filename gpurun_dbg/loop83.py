import json, sys, collections
sys.path.insert(0, 'kube-arbitrator_amd'); sys.path.insert(0, 'tests')
from helpers import run_oracle
from kbgpu.fixture import run_fixture
cnt = collections.Counter()
for r in (0, 1):
    fx = json.load(open(f'gpurun_dbg/fx83_{r}.json'))
    ref = run_oracle(fx)
    for it in range(150):
        for opts in ({"batch_tasks": 3, "candidates": 4, "full_scan": 1}, {"batch_tasks": 1 + it % 9, "candidates": 1 + it % 5, "full_scan": it % 2}):
            got, ssn = run_fixture(fx, opts)
            ok = got.get("decisions") == ref.get("decisions") and got.get("evictions") == ref.get("evictions")
            cnt[(r, ok)] += 1
            if not ok and cnt[(r, False)] <= 2:
                print("MISMATCH round", r, it, opts)
                print(" ref:", ref.get("decisions"), ref.get("evictions"))
                print(" got:", got.get("decisions"), got.get("evictions"))
            if ssn: ssn.close()
print(cnt, flush=True)
