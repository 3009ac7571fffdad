"""Session-open phase timing (GPU box): python tools/open_profile.py [config]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "kube-arbitrator_amd"))
os.environ["KBG_PROFILE_OPEN"] = "1"

from kbgpu import synth  # noqa: E402
from kbgpu.cache import cache_from_fixture  # noqa: E402
from kbgpu.fixture import fixture_tiers  # noqa: E402
from kbgpu.framework import open_session  # noqa: E402
from kbgpu.snapshot import FlatSnapshot  # noqa: E402

cid = int(sys.argv[1]) if len(sys.argv) > 1 else 3
fx = synth.config_fixture(cid)
t0 = time.time()
cache = cache_from_fixture(fx)
t1 = time.time()
snap = cache.snapshot()
t2 = time.time()
s = FlatSnapshot(snap.nodes, snap.jobs, snap.queues, snap.others, fixture_tiers(fx))
t3 = time.time()
print(f"python cache {t1 - t0:.3f}s snapshot {t2 - t1:.3f}s flatten {t3 - t2:.3f}s", file=sys.stderr)
for _ in range(3):
    ssn = open_session(cache, fixture_tiers(fx), {"device": 0})
    print("open_ms", ssn.stats().open_ms, file=sys.stderr)
    ssn.close()
