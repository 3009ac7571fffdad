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
N > 1       = ONE cluster with its node axis sharded over the N GPUs:
              each rank scans its node rows, an RCCL all-gather over xGMI
              publishes the per-shard feasibility bitmaps every batch, every
              rank resolves the identical decision sequence (strong scaling;
              the whole job places decisions_per_cycle per step)
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


# The contract is ONE JSON line on stdout. Libraries write there too (RCCL
# prints a version banner when a communicator comes up), so file descriptor 1
# is pointed at stderr for the whole run and the result line goes to a
# duplicate of the original stdout.
_RESULT_FD = None


def _capture_stdout():
    global _RESULT_FD
    sys.stdout.flush()
    _RESULT_FD = os.dup(1)
    os.dup2(2, 1)


def emit(line):
    data = (json.dumps(line) + "\n").encode()
    if _RESULT_FD is None:
        sys.stdout.write(data.decode())
        sys.stdout.flush()
    else:
        os.write(_RESULT_FD, data)


def cpu_baseline(fx, budget_note, threads=1):
    """kbref oracle on the same workload (kind "port"): 1 thread (SURVEY 8(d)
    B-ref, the Go allocate loop is single-goroutine), or `threads` threads
    evaluating each task's node loop in parallel blocks with the FitDelta map
    built once per job (B-omp, the fair multi-core CPU baseline); both return
    the same decisions."""
    ref = os.path.join(ROOT, "oracle", "build", "kbref")
    if not os.path.exists(ref):
        subprocess.run(["make", "-C", os.path.join(ROOT, "oracle")], check=True, capture_output=True)
    with tempfile.TemporaryDirectory() as d:
        src, dst = os.path.join(d, "fx.json"), os.path.join(d, "out.json")
        with open(src, "w") as f:
            json.dump(fx, f)
        cpus = ",".join(str(c) for c in range(threads))
        subprocess.run(["taskset", "-c", cpus, ref, "--threads", str(threads), src, "-o", dst], check=True)
        with open(dst) as f:
            out = json.load(f)
    secs = out["stats"]["seconds"]
    n = out["stats"]["decisions"]
    how = "1 thread" if threads == 1 else f"{threads} threads (OpenMP node loop)"
    return {"value": n / secs, "unit": "placements/s", "cores": threads, "kind": "port",
            "sample": f"one full {budget_note} allocate cycle ({n} placements, {secs:.2f} s, "
                      f"{out['stats']['predicate_calls']} predicate calls), kbref C++ port, {how}"}


def omp_threads():
    return max(1, min(16, len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else os.cpu_count() or 1))


def load_pmc_traffic(n_nodes, mode):
    """Per-launch HBM bytes (read + write) of the scan kernel in `mode`
    ("full_scan" / "grouped") from the committed rocprofv3 PMC summary of this
    same bench command (profiles/pmc_scan.json), if it matches the workload."""
    p = os.path.join(ROOT, "profiles", "pmc_scan.json")
    if not os.path.exists(p):
        return None
    try:
        d = json.load(open(p))
        if d.get("n_nodes") == n_nodes:
            return (d.get(mode) or {}).get("hbm_bytes_per_launch")
    except (OSError, ValueError):
        pass
    return None


def main():
    _capture_stdout()
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--config", type=int, default=3)
    ap.add_argument("--batch", type=int, default=0)
    ap.add_argument("--candidates", type=int, default=0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--comm", action="store_true",
                    help="open the session through the RCCL sharded entry point even at N=1 (rehearsal)")
    ap.add_argument("--dist-backend", default="nccl", help="nccl (RCCL) on MI355X; gloo to rehearse on one GPU")
    args = ap.parse_args()

    import torch
    from kbgpu import dist as kdist
    rank, world, local_rank = kdist.env_rank()
    # KBG_BENCH_DEVICE pins every rank to one device (rehearsal on a 1-GPU box only)
    device = int(os.environ.get("KBG_BENCH_DEVICE", local_rank))
    torch.cuda.set_device(device)
    kdist.init(args.dist_backend)

    from kbgpu import _abi, actions, synth  # noqa: F401
    from kbgpu.cache import cache_from_fixture
    from kbgpu.fixture import fixture_tiers
    from kbgpu.framework import open_session

    cid = args.config
    t0 = time.time()
    fx = synth.config_fixture(cid)  # every rank: the same cluster
    cache = cache_from_fixture(fx)
    base_opts = {"device": device}
    comm = None
    if world > 1 or args.comm:
        comm = kdist.ShardComm(device)
        base_opts["comm"] = comm
    if args.batch:
        base_opts["batch_tasks"] = args.batch
    if args.candidates:
        base_opts["candidates"] = args.candidates
    L = _abi.lib()

    def run_mode(full_scan, steps, warmup, barrier):
        ssn = open_session(cache, fixture_tiers(fx), dict(base_opts, full_scan=full_scan))
        cap = max(1, ssn.flat.pending_count)
        buf = (_abi.kbg_decision * cap)()
        nout = ctypes.c_int32(0)

        def step():
            _abi.check(L.kbg_session_reset(ssn.handle))
            _abi.check(L.kbg_allocate(ssn.handle, buf, cap, ctypes.byref(nout)))
            return nout.value

        for _ in range(warmup):
            step()
        agg = {"cycle_ms": [], "decisions": 0, "evals": 0, "visits": 0, "scan_ms": 0.0, "sel_ms": 0.0,
               "launches": 0}
        if barrier:
            kdist.barrier()
        torch.cuda.synchronize()
        t_start = time.perf_counter()
        for _ in range(steps):
            t1 = time.perf_counter()
            agg["decisions"] += step()
            agg["cycle_ms"].append((time.perf_counter() - t1) * 1e3)
            st = ssn.stats()
            agg["evals"] += st.evaluations
            agg["visits"] += st.node_visits
            agg["scan_ms"] += st.scan_kernel_ms
            agg["sel_ms"] += st.select_kernel_ms
            agg["launches"] += st.scan_launches
        torch.cuda.synchronize()
        agg["elapsed"] = time.perf_counter() - t_start
        if barrier:
            kdist.barrier()
        agg["stats"] = ssn.stats()
        agg["n_nodes"] = len(ssn.nodes)
        agg["pending"] = ssn.flat.pending_count
        agg["jobs"] = len(ssn.jobs)
        agg["queues"] = len(ssn.queues)
        ssn.close()
        return agg

    def roofline(agg, mode):
        # per rank: every evaluation row streams this shard's node records (N/R x 64 B) + its 32 B task record
        algo = agg["visits"] * NODE_RECORD_B + agg["evals"] * TASK_RECORD_B
        ach = algo / (agg["scan_ms"] * 1e-3) / 1e9 if agg["scan_ms"] > 0 else 0.0
        return {"bound": "hbm", "achieved": ach, "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": ach / HBM_PEAK_GBS,
                "traffic": load_pmc_traffic(agg["n_nodes"], mode) if comm is None else None, "kernel": "kbg_scan_kernel",
                "avg_launch_us": agg["scan_ms"] * 1e3 / max(1, agg["launches"]),
                "algo_bytes_per_launch": algo / max(1, agg["launches"]),
                "evaluations_per_launch": agg["evals"] / max(1, agg["launches"])}

    log(f"[rank {rank}] C{cid} setup {time.time() - t0:.1f}s")
    # the process's first session open pays the HIP runtime / code-object
    # initialisation; the sessions measured below are opened after it
    warm = open_session(cache, fixture_tiers(fx), dict(base_opts))
    open_ms_first = warm.stats().open_ms
    warm.close()
    if fx.get("actions"):
        contended_bench(args, fx, cache, base_opts, comm, rank, world, cid, open_ms_first)
        return
    prod = run_mode(0, args.steps, args.warmup, True)      # production: grouped shapes
    full = run_mode(1, max(1, min(3, args.steps)), 1, False)  # SURVEY roofline rule: every task scans all N
    decisions = prod["decisions"]
    elapsed, total_decisions = kdist.aggregate(prod["elapsed"], decisions, sharded=world > 1)
    st = prod["stats"]
    n_nodes = prod["n_nodes"]

    def breakdown(agg):
        s2 = agg["stats"]
        return {"scan_ms": s2.scan_kernel_ms, "select_ms": s2.select_kernel_ms, "launches": s2.scan_launches,
                "evaluations": s2.evaluations, "batches": s2.batches, "mispredictions": s2.mispredictions,
                "truncations": s2.truncations, "replayed": s2.replayed, "host_engine_ms": s2.engine_ms,
                "host_resolve_ms": s2.resolve_ms, "device_roundtrip_ms": s2.device_ms,
                "delta_writeback_ms": s2.delta_ms, "exchange_ms": s2.exchange_ms, "shards": s2.shards,
                "cycle_ms": s2.allocate_ms}

    line = {
        "metric": "task placements/sec + p50 allocate-cycle latency, 5k nodes x 100k pending tasks",
        "value": total_decisions / elapsed,
        "unit": "placements/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": elapsed / args.steps * 1e3,
        "p50_cycle_ms": statistics.median(prod["cycle_ms"]),
        "higher_is_better": True,
        "scaling": "strong" if world > 1 else "weak",
        "vs_baseline": None,
        "dtype": "f64",
        "data": "synthetic (seeded BASELINE config generator, kbgpu/synth.py)",
        "config": {"workload": f"C{cid}: {n_nodes} nodes x {prod['pending']} pending tasks, "
                               f"{prod['jobs']} gang PodGroups, {prod['queues']} proportion queues, default tiers",
                   "parallelism": f"node-axis shards x{world} (RCCL all-gather)" if world > 1 else "single-gpu",
                   "batch_tasks": base_opts.get("batch_tasks", 8192),
                   "candidates": base_opts.get("candidates", 32)},
        "roofline": roofline(full, "full_scan"),
        "roofline_note": "scan kernel in full-scan mode (every task evaluation scans all N nodes, SURVEY 8d rule); "
                         "the production mode groups identical (class, request) shapes per batch",
        "full_scan_mode": {"placements_per_s": full["decisions"] / full["elapsed"],
                           "p50_cycle_ms": statistics.median(full["cycle_ms"]), "breakdown": breakdown(full)},
        "production_mode": {"roofline": roofline(prod, "grouped"), "breakdown": breakdown(prod)},
        "decisions_per_cycle": decisions // max(1, args.steps),
        "open_ms": st.open_ms,
        "open_ms_first_in_process": open_ms_first,
    }
    if rank == 0 and not args.no_cpu_baseline:
        line["cpu_baseline"] = cpu_baseline(fx, f"C{cid}")
        line["cpu_baseline_omp"] = cpu_baseline(fx, f"C{cid}", omp_threads())
    if rank == 0:
        emit(line)
    if comm is not None:
        comm.close()
    kdist.shutdown()


def contended_bench(args, fx, cache, base_opts, comm, rank, world, cid, open_ms_first):
    """C5: one step = one scheduling cycle of the fixture's actions ("reclaim,
    allocate, backfill, preempt") through the C ABI on a session reset to the
    snapshot. value = (pipelines + allocations) / s; evictions are reported
    beside them. The dominant device kernel is the victim scan (one launch per
    reclaimer / preemptor task, one thread per node); its algorithmic bytes per
    launch are N x 64 B (node record) + R x 32 B (the Running task records the
    scan walks, R = running session tasks), DESIGN.md §5."""
    import torch
    from kbgpu import _abi
    from kbgpu import dist as kdist
    from kbgpu.api import RUNNING
    from kbgpu.fixture import fixture_tiers
    from kbgpu.framework import open_session

    L = _abi.lib()
    ssn = open_session(cache, fixture_tiers(fx), dict(base_opts))
    cap = max(1, ssn.flat.pending_all)
    buf = (_abi.kbg_decision * cap)()
    nout = ctypes.c_int32(0)
    nev = ctypes.c_int32(0)
    entries = {"reclaim": L.kbg_reclaim, "allocate": L.kbg_allocate, "backfill": L.kbg_backfill,
               "preempt": L.kbg_preempt}
    acts = [entries[a] for a in fx["actions"]]
    phase = {"reclaim_ms": [], "allocate_ms": [], "backfill_ms": [], "preempt_ms": []}

    def step():
        _abi.check(L.kbg_session_reset(ssn.handle))
        for fn in acts:
            _abi.check(fn(ssn.handle, buf, cap, ctypes.byref(nout)))
        _abi.check(L.kbg_evictions_get(ssn.handle, None, 0, ctypes.byref(nev)))
        return nout.value, nev.value

    for _ in range(args.warmup):
        step()
    cyc, dec, ev, vscans, vms, vtries, vevals = [], 0, 0, 0, 0.0, 0, 0
    kdist.barrier()
    torch.cuda.synchronize()
    t_start = time.perf_counter()
    for _ in range(args.steps):
        t1 = time.perf_counter()
        d, e = step()
        cyc.append((time.perf_counter() - t1) * 1e3)
        dec += d
        ev += e
        st = ssn.stats()
        vscans += st.victim_scans
        vms += st.victim_kernel_ms
        vtries += st.victim_tries
        vevals += st.victim_host_evals
        for k in phase:
            phase[k].append(getattr(st, k))
    torch.cuda.synchronize()
    elapsed_local = time.perf_counter() - t_start
    kdist.barrier()
    st = ssn.stats()
    n_nodes = len(ssn.nodes)
    running = sum(1 for t in ssn.flat.task_objs if t.status == RUNNING)
    pending = ssn.flat.pending_all
    ssn.close()
    elapsed, total = kdist.aggregate(elapsed_local, dec, sharded=world > 1)
    nodes_per_rank = n_nodes / max(1, world)
    algo = nodes_per_rank * NODE_RECORD_B + running / max(1, world) * TASK_RECORD_B
    launch_us = vms * 1e3 / max(1, vscans)
    ach = algo / (launch_us * 1e-6) / 1e9 if launch_us > 0 else 0.0
    line = {
        "metric": "task placements/sec + p50 scheduling-cycle latency, contended cluster (reclaim/preempt)",
        "value": total / elapsed,
        "unit": "placements/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": elapsed / args.steps * 1e3,
        "p50_cycle_ms": statistics.median(cyc),
        "higher_is_better": True,
        "scaling": "strong" if world > 1 else "weak",
        "vs_baseline": None,
        "dtype": "f64",
        "data": "synthetic (seeded BASELINE config generator, kbgpu/synth.py contended_config)",
        "config": {"workload": f"C{cid}: {n_nodes} nodes, {running} running + {pending} pending tasks "
                               f"(~95% CPU), actions {', '.join(fx['actions'])}, default tiers",
                   "parallelism": f"node-axis shards x{world} (RCCL min-reduce of the victim-scan stop node)"
                                  if world > 1 else "single-gpu"},
        "roofline": {"bound": "hbm", "achieved": ach, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": ach / HBM_PEAK_GBS, "traffic": None, "kernel": "kbg_victim_kernel",
                     "avg_launch_us": launch_us, "algo_bytes_per_launch": algo},
        "decisions_per_cycle": dec // max(1, args.steps),
        "evictions_per_cycle": ev // max(1, args.steps),
        "victim_scans_per_cycle": vscans // max(1, args.steps),
        "victim_tries_per_cycle": vtries // max(1, args.steps),
        "victim_host_evals_per_cycle": vevals // max(1, args.steps),
        "phase_ms_p50": {k: statistics.median(v) for k, v in phase.items()},
        "open_ms": st.open_ms,
        "open_ms_first_in_process": open_ms_first,
    }
    if rank == 0 and not args.no_cpu_baseline:
        line["cpu_baseline"] = cpu_baseline(fx, f"C{cid}")
        line["cpu_baseline"]["sample"] = line["cpu_baseline"]["sample"].replace("allocate cycle", "cycle (" +
                                                                                ", ".join(fx["actions"]) + ")")
    if rank == 0:
        emit(line)
    if comm is not None:
        comm.close()
    kdist.shutdown()


if __name__ == "__main__":
    main()
