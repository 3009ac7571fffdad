"""Developer tool: A/B of library builds on the C3 bench (production and full-scan
p50), alternating in one GPU session: python kube-arbitrator_amd/tools/ab_bench.py lib1.so lib2.so
(CONFIG=4: another BASELINE config; REPS: rounds; lib.so@KEY=VAL sets a variant's environment).
Per run: p50 cycle ms (production, full-scan), production scan launch us, production device round trip ms,
production re-checks and resolve ms
(RESIDENT=1: and the p50 resident churn update ms, the bind update ms, the p50 churn allocate ms; STEPS: timed steps)"""
import json, os, subprocess, sys
res = {}
cfg = os.environ.get("CONFIG", "3")
resident = bool(os.environ.get("RESIDENT"))  # also the resident session's churn updates (p50 update ms)
steps = os.environ.get("STEPS", "10")
for rep in range(int(os.environ.get("REPS", "3"))):
    for v in sys.argv[1:]:
        code = ("import sys; sys.path.insert(0,'kube-arbitrator_amd'); from kbgpu import _abi; _abi.LIB_PATH='%s'; "
                "sys.argv=['bench.py','--config','%s','--steps','%s','--warmup','2','--no-cpu-baseline'%s]; "
                "import runpy; runpy.run_path('bench.py', run_name='__main__')") % (v, cfg, steps, "" if resident else ",'--no-resident'")
        env = dict(os.environ)
        for kv in v.split("@")[1:]:  # lib.so@KEY=VAL@...: the variant's environment
            k, _, val = kv.partition("=")
            env[k] = val
        out = subprocess.run([sys.executable, "-c", code.replace(v, v.split("@")[0])], capture_output=True, text=True,
                             timeout=300, env=env)
        d = json.loads(out.stdout.strip().splitlines()[-1])
        pm = d.get("production_mode", {})
        res.setdefault(v, []).append((round(d["p50_cycle_ms"], 2), round(d.get("full_scan_mode", {}).get("p50_cycle_ms") or 0, 2),
                                      round(pm.get("scan_kernel", {}).get("avg_launch_us") or 0, 1),
                                      round(pm.get("breakdown", {}).get("device_roundtrip_ms") or 0, 2),
                                      pm.get("breakdown", {}).get("resolve_rechecks"),
                                      round(pm.get("breakdown", {}).get("host_resolve_ms") or 0, 2))
                                     + ((round(d["resident_session"]["churn_update_ms_p50"], 2),
                                         round(d["resident_session"]["bind_update_ms"], 2),
                                         round(d["resident_session"]["churn_allocate_ms_p50"], 2)) if resident else ()))
        print(v, res[v][-1], flush=True)
print(json.dumps(res))
