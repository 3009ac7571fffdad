"""Developer tool: A/B of library builds on the C3 bench (production and full-scan
p50), alternating in one GPU session: python kube-arbitrator_amd/tools/ab_bench.py lib1.so lib2.so"""
import json, subprocess, sys
res = {}
for rep in range(3):
    for v in sys.argv[1:]:
        code = ("import sys; sys.path.insert(0,'kube-arbitrator_amd'); from kbgpu import _abi; _abi.LIB_PATH='%s'; "
                "sys.argv=['bench.py','--steps','10','--warmup','2','--no-cpu-baseline','--no-resident']; "
                "import runpy; runpy.run_path('bench.py', run_name='__main__')") % v
        out = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=300)
        d = json.loads(out.stdout.strip().splitlines()[-1])
        res.setdefault(v, []).append((round(d["p50_cycle_ms"], 2), round(d["full_scan_mode"]["p50_cycle_ms"], 2)))
        print(v, res[v][-1], flush=True)
print(json.dumps(res))
