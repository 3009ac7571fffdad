"""Developer tool: A/B of environment settings on the bench (production and
full-scan p50 of one config), alternating in one GPU session.
python kube-arbitrator_amd/tools/ab_env.py CONFIG 'A=1' 'B=1,C=2' ''  (an empty spec = defaults)"""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    cid = sys.argv[1]
    specs = sys.argv[2:] or [""]
    res = {}
    for rep in range(int(os.environ.get("REPS", "3"))):
        for spec in specs:
            env = dict(os.environ)
            for kv in filter(None, spec.split(",")):
                k, v = kv.split("=", 1)
                env[k] = v
            out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--config", cid, "--steps", "10",
                                  "--warmup", "2", "--no-cpu-baseline", "--no-resident"],
                                 capture_output=True, text=True, timeout=300, env=env, cwd=ROOT)
            d = json.loads(out.stdout.strip().splitlines()[-1])
            fs = d.get("full_scan_mode", {})
            bd = d.get("production_mode", {}).get("breakdown", {})
            r = (round(d["p50_cycle_ms"], 2), round(fs.get("p50_cycle_ms", 0.0), 2), round(bd.get("host_engine_ms", 0), 2),
                 round(bd.get("host_resolve_ms", 0), 2), bd.get("mispredictions"), bd.get("resolve_rechecks"),
                 bd.get("refresh_scans"), round(bd.get("scan_ms", 0), 3))
            res.setdefault(spec or "default", []).append(r)
            print(f"{spec or 'default':40s} prod {r[0]:.2f} ms  full {r[1]:.2f} ms  engine {r[2]:.2f}  resolve {r[3]:.2f}"
                  f"  cuts {r[4]}  rechecks {r[5]}  refreshes {r[6]}  kernel {r[7]} ms", flush=True)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
