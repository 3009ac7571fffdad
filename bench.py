"""Benchmark: kube-batch allocate cycle on MI355X (BASELINE.json metric).

One step = one allocateAction.Execute cycle (allocate.go:41-176) over the
BASELINE config-3 synthetic cluster (5k nodes x 100k pending tasks, 2k gang
PodGroups, 4 proportion queues, default tiers), on a session re-opened from
the same snapshot (the HBM node table is restored with a device copy; the
snapshot itself was uploaded once, untimed). Inputs are resident in HBM when
the timed region starts.

value       = placements/sec (Allocate + Pipeline decisions / wall time), whole job
ms_per_step = mean allocate-cycle wall time; p50_cycle_ms = median
roofline    = the scan kernel (dominant device kernel): algorithmic bytes per
              launch = evaluations x (N x 64 B + 32 B) / HIP-event
              time of the launch, against 8 TB/s HBM3E
cpu_baseline= the kbref oracle (single-threaded C++ restatement of the Go
              allocate path) on one full C3 cycle on this host
N > 1       = independent replicas, one cluster per rank (weak scaling); see DESIGN.md
"""
import argparse
import ctypes
import json
import os
import statistics
import subprocess
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "kube-arbitrator_amd"))

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md chip table)
NODE_RECORD_B = 64     # SURVEY §8(d) algorithmic bytes per node record
TASK_RECORD_B = 32


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def cpu_baseline(fx, budget_note):
    """kbref oracle on the same workload, single thread (kind "port")."""
    ref = os.path.join(ROOT, "oracle", "build", "kbref")
    if not os.path.exists(ref):
        subprocess.run(["make", "-C", os.path.join(ROOT, "oracle")], check=True, capture_output=True)
    with tempfile.TemporaryDirectory() as d:
        src, dst = os.path.join(d, "fx.json"), os.path.join(d, "out.json")
        with open(src, "w") as f:
            json.dump(fx, f)
        subprocess.run(["taskset", "-c", "0", ref, src, "-o", dst], check=True)
        with open(dst) as f:
            out = json.load(f)
    secs = out["stats"]["seconds"]
    n = out["stats"]["decisions"]
    return {"value": n / secs, "unit": "placements/s", "cores": 1, "kind": "port",
            "sample": f"one full {budget_note} allocate cycle ({n} placements, {secs:.2f} s, "
                      f"{out['stats']['predicate_calls']} predicate calls), kbref C++ port, 1 thread"}


def load_pmc_traffic(n_nodes):
    """Per-launch HBM bytes of the scan kernel from the committed PMC profile, if any."""
    p = os.path.join(ROOT, "profiles", "pmc_scan.json")
    if not os.path.exists(p):
        return None
    try:
        d = json.load(open(p))
        if d.get("n_nodes") == n_nodes:
            return d.get("hbm_bytes_per_launch")
    except (OSError, ValueError):
        pass
    return None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--config", type=int, default=3)
    ap.add_argument("--batch", type=int, default=0)
    ap.add_argument("--candidates", type=int, default=0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))

    import torch
    dist = None
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group("nccl", init_method="env://")
        torch.cuda.set_device(local_rank)
    else:
        torch.cuda.set_device(0)

    from kbgpu import _abi, actions, synth  # noqa: F401
    from kbgpu.cache import cache_from_fixture
    from kbgpu.fixture import fixture_tiers
    from kbgpu.framework import open_session

    cid = args.config
    t0 = time.time()
    fx = synth.config_fixture(cid)
    if world > 1 and rank > 0:
        # weak scaling: each rank schedules its own replica cluster
        fx["name"] += f"-replica{rank}"
    cache = cache_from_fixture(fx)
    opts = {"device": local_rank}
    if args.batch:
        opts["batch_tasks"] = args.batch
    if args.candidates:
        opts["candidates"] = args.candidates
    ssn = open_session(cache, fixture_tiers(fx), opts)
    n_nodes = len(ssn.nodes)
    L = _abi.lib()
    cap = max(1, ssn.flat.pending_count)
    buf = (_abi.kbg_decision * cap)()
    nout = ctypes.c_int32(0)
    log(f"[rank {rank}] C{cid}: {n_nodes} nodes, {ssn.flat.pending_count} pending tasks, "
        f"setup {time.time() - t0:.1f}s, session open {ssn.stats().open_ms:.1f} ms")

    def step():
        _abi.check(L.kbg_session_reset(ssn.handle))
        _abi.check(L.kbg_allocate(ssn.handle, buf, cap, ctypes.byref(nout)))
        return nout.value

    for _ in range(args.warmup):
        step()

    cycle_ms, decisions = [], 0
    evals = 0
    scan_ms = 0.0
    launches = 0
    sel_ms = 0.0
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    t_start = time.perf_counter()
    for _ in range(args.steps):
        t1 = time.perf_counter()
        decisions += step()
        cycle_ms.append((time.perf_counter() - t1) * 1e3)
        st = ssn.stats()
        evals += st.evaluations
        scan_ms += st.scan_kernel_ms
        sel_ms += st.select_kernel_ms
        launches += st.scan_launches
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    elapsed = time.perf_counter() - t_start
    st = ssn.stats()

    total_decisions = decisions
    if dist:
        t = torch.tensor([elapsed], dtype=torch.float64, device="cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
        d = torch.tensor([decisions], dtype=torch.float64, device="cuda")
        dist.all_reduce(d, op=dist.ReduceOp.SUM)
        total_decisions = int(d.item())

    algo_bytes = evals * (n_nodes * NODE_RECORD_B + TASK_RECORD_B)
    achieved = algo_bytes / (scan_ms * 1e-3) / 1e9 if scan_ms > 0 else 0.0
    traffic = load_pmc_traffic(n_nodes)
    line = {
        "metric": "task placements/sec + p50 allocate-cycle latency, 5k nodes x 100k pending tasks",
        "value": total_decisions / elapsed,
        "unit": "placements/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": elapsed / args.steps * 1e3,
        "p50_cycle_ms": statistics.median(cycle_ms),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f64",
        "data": "synthetic (seeded BASELINE config generator, kbgpu/synth.py)",
        "config": {"workload": f"C{cid}: {n_nodes} nodes x {ssn.flat.pending_count} pending tasks, "
                               f"{len(ssn.jobs)} gang PodGroups, {len(ssn.queues)} proportion queues, default tiers",
                   "parallelism": "replicas" if world > 1 else "single-gpu",
                   "batch_tasks": opts.get("batch_tasks", 2048), "candidates": opts.get("candidates", 32)},
        "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                     "kernel": "kbg_scan_kernel",
                     "avg_launch_us": scan_ms * 1e3 / max(1, launches),
                     "algo_bytes_per_launch": algo_bytes / max(1, launches)},
        "decisions_per_cycle": decisions // max(1, args.steps),
        "device_breakdown_ms_per_cycle": {"scan": scan_ms / args.steps, "select": sel_ms / args.steps,
                                          "launches": launches / args.steps,
                                          "batches": st.batches, "mispredictions": st.mispredictions,
                                          "truncations": st.truncations, "replayed": st.replayed,
                                          "host_engine": st.engine_ms, "host_resolve": st.resolve_ms,
                                          "device_roundtrips": st.device_ms, "delta_writeback": st.delta_ms},
        "open_ms": st.open_ms,
    }
    if rank == 0 and not args.no_cpu_baseline:
        line["cpu_baseline"] = cpu_baseline(fx, f"C{cid}")
    ssn.close()
    if rank == 0:
        print(json.dumps(line), flush=True)
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
