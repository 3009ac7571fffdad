"""Benchmark: kube-batch allocate cycle on MI355X (BASELINE.json metric).

One step = one allocateAction.Execute cycle (allocate.go:41-176) over the
BASELINE config-3 synthetic cluster (5k nodes x 100k pending tasks, 2k gang
PodGroups, 4 proportion queues, default tiers), on a session re-opened from
the same snapshot (the HBM node table is restored with a device copy; the
snapshot itself was uploaded once, untimed). Inputs are resident in HBM when
the timed region starts.

value       = placements/sec (Allocate + Pipeline decisions / wall time), whole job,
              production mode (identical (class, request) shapes share a scan row)
ms_per_step = mean allocate-cycle wall time; p50_cycle_ms = median
roofline    = the dominant kernel (kbg_firstfit_kernel, full-scan mode: every
              task evaluation scans the whole node table on the device)
              against the ceiling that binds it, VALU issue: PMC wave64 VALU
              instructions per launch (profiles/pmc_scan.json, scaled to this
              run's rows x words) / average launch time (HIP events on the
              library's stream), peak 1024 SIMDs x 2.4 GHz / 4 cycles; traffic
              = PMC HBM bytes per launch with traffic_frac_of_peak against 8
              TB/s; equivalent_8d = SURVEY §8(d) bytes per task evaluation (N x
              64 B + 32 B) x rows / launch time (on-chip reuse, above 1)
cycle_roofline_8d = BASELINE's north-star form: the same bytes per allocate
              cycle / p50 cycle wall time
scan_kernel = the dominant kernel against its physical ceilings: PMC HBM bytes
              and PMC VALU wave instructions per launch over its HIP-event time
cpu_baseline= the kbref oracle on this host, CPU model stated: B-ref (1 thread),
              B-omp (the best of 4 ... 64 threads and every CPU the job can
              use — affinity mask capped by the cgroup quota — the sweep
              beside it), B-faithful (the per-call podLister walk, 20 s
              budget); C3 runs 20 s samples, C4 60 s samples
parity      = the decision log of the LAST timed cycle of each mode, replayed
              through the session (actions.replay) and hashed with the node /
              job / queue states exactly as the parity tests do
              (kbgpu.digest), against the oracle's digest of the same seeded
              session committed under tests/golden/digest_c<config>.json (no
              oracle runs here); a mismatch exits non-zero after the line
--gpus N    = N ranks: under torchrun its WORLD_SIZE must be N; without a
              launcher bench.py starts the N rank processes itself
N > 1       = ONE cluster with its node axis sharded over the N GPUs (SURVEY §8e,
              DESIGN.md §7), the scan service: rank 0 runs the single-GPU
              pipeline (ordering engine, in-order commit); each of its scans is
              an RCCL broadcast of the launch and the commits since the last
              one, every rank scans its own node rows, an RCCL sum-reduce over
              xGMI joins the ranks' word masks; the other ranks replay rank 0's
              commits and every rank returns the identical decision log (strong
              scaling; the whole job places decisions_per_cycle per step).
              KBG_OWNER_RESOLVE=1: the owner-resolve protocol instead
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
SIMDS = 256 * 4        # 256 CUs x 4 SIMDs
CLOCK_GHZ = 2.4        # peak engine clock
VALU_CYC = 4           # issue cycles of one wave64 VALU instruction on a SIMD (fp64 compare, lane moves)
VALU_PEAK_GIPS = SIMDS * CLOCK_GHZ / VALU_CYC  # chip-wide wave64 VALU issue ceiling, G instructions/s
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


def cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


_JOB_CPUS = None


def job_cpus():
    """The CPUs this process may run on (the GPU box gives a job a share of
    the host), as at the first call: the CPU baselines pin this process to one
    of them meanwhile."""
    global _JOB_CPUS
    if _JOB_CPUS is None:
        _JOB_CPUS = sorted(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else \
            list(range(os.cpu_count() or 1))
    return list(_JOB_CPUS)


def cpu_quota():
    """The CPU time the job's cgroup may use, in CPUs (cgroup v2 cpu.max or v1
    cfs quota / period), None when unlimited. A shared box can show every host
    CPU in the affinity mask while a quota caps the job far below it: threads
    past the quota only time-slice."""
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, per = f.read().split()[:2]
            return None if q == "max" else int(q) / int(per)
    except (OSError, ValueError):
        pass
    try:
        with open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us") as f:
            q = int(f.read())
        with open("/sys/fs/cgroup/cpu/cpu.cfs_period_us") as f:
            per = int(f.read())
        return None if q <= 0 else q / per
    except (OSError, ValueError):
        return None


def usable_cpus():
    """CPUs the job can run threads on at once: its affinity mask, capped by the cgroup quota."""
    n = len(job_cpus())
    q = cpu_quota()
    return max(1, min(n, int(q))) if q else n


def omp_sweep():
    """B-omp thread counts (the node loop parallelised over all
    host cores, stated): 4, 8, 16, 32, 64 and every CPU the job can use less
    two, none above that. Past the cgroup quota threads only time-slice, and
    the two left over keep the bench process and the HIP runtime's own threads
    off the team's CPUs (round 5's 16-thread run on a 16-CPU quota collapsed
    to a quarter of its 8-thread rate sharing them)."""
    n = usable_cpus()
    top = max(1, n - 2) if n > 4 else n
    return sorted({t for t in (4, 8, 16, 32, 64) if t < top} | {top})


def spawn_ranks(n):
    """`--gpus N` without a launcher: N child processes of this script, rank r
    on GPU r (RANK / LOCAL_RANK / WORLD_SIZE / MASTER_* in their environment,
    rendezvous on 127.0.0.1), started before this process touches a GPU; the
    parent only waits for them (no exec). A rank that fails ends the others,
    so none is left blocked in a collective. Rank 0 prints the result line on
    the inherited stdout."""
    import signal
    import socket
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env))
    log(f"bench: started {n} ranks (pids {', '.join(str(p.pid) for p in procs)})")
    rc = 0
    live = list(procs)
    while live:
        for p in list(live):
            c = p.poll()
            if c is None:
                continue
            live.remove(p)
            if c != 0 and rc == 0:
                rc = c
                log(f"bench: rank pid {p.pid} exited with {c}; stopping the other ranks")
                for q in live:
                    q.send_signal(signal.SIGTERM)
        time.sleep(0.05)
    return rc


_FX_FILES = {}


def fixture_file(fx):
    """The fixture as JSON on disk, written once per process for every baseline run."""
    key = id(fx)
    if key not in _FX_FILES:
        d = tempfile.mkdtemp(prefix="kbg_bench_")
        path = os.path.join(d, "fx.json")
        with open(path, "w") as f:
            json.dump(fx, f)
        _FX_FILES[key] = path
    return _FX_FILES[key]


def cpu_baseline(fx, label, threads=1, faithful=False, budget=0.0):
    """kbref oracle on the same workload (kind "port"), SURVEY §8(d):
    B-ref     1 thread (the Go allocate loop is single-goroutine), podLister
              walk elided under the proven-true condition;
    B-omp     `threads` threads evaluating each task's node loop (a persistent
              team, 64-node chunks in node order, stopping at the first fit),
              the fair multi-core baseline;
    B-faithful 1 thread replaying the podLister's per-call O(allocated pods)
              walk of predicates.go:70-89 (F7), under a wall-clock budget.
    All produce the decisions the device path makes (tested). With a budget
    the rate is over the placements reached within it. None on failure (the
    bench line is never lost to a baseline)."""
    ref = os.path.join(ROOT, "oracle", "build", "kbref")
    log(f"cpu baseline {label}: {threads} thread(s){', faithful' if faithful else ''}"
        f"{f', {budget:.0f} s budget' if budget else ''}")
    try:
        if not os.path.exists(ref):
            subprocess.run(["make", "-C", os.path.join(ROOT, "oracle")], check=True, capture_output=True)
        src = fixture_file(fx)
        with tempfile.TemporaryDirectory() as d:
            dst = os.path.join(d, "out.json")
            # the team on the job's last CPUs, away from this process (pinned to
            # the first one below while the baseline runs)
            mine = job_cpus()
            cpus = ",".join(str(c) for c in (mine[-threads:] if len(mine) > threads else mine))
            cmd = ["taskset", "-c", cpus, ref, "--threads", str(threads)]
            if faithful:
                cmd.append("--faithful")
            if budget:
                cmd += ["--budget", str(budget)]
            subprocess.run(cmd + [src, "-o", dst], check=True, timeout=max(600, 3 * budget))
            with open(dst) as f:
                out = json.load(f)
    except (subprocess.CalledProcessError, subprocess.TimeoutExpired, OSError, ValueError) as e:
        log(f"cpu baseline ({label}, {threads} threads) failed: {e}")
        return None
    st = out["stats"]
    secs, n = st["seconds"], st["decisions"]
    how = ("B-faithful: 1 thread, podLister walk per predicate call" if faithful else
           "B-ref: 1 thread" if threads == 1 else
           f"B-omp: {threads} threads (one persistent team for the run; each task's node loop in 64-node chunks "
           f"handed out in node order, stopping at the first fit)")
    scope = (f"first {n} placements within a {budget:.0f} s budget" if out["status"] == "budget"
             else f"one full cycle ({n} placements)")
    return {"value": n / secs if secs > 0 else 0.0, "unit": "placements/s", "cores": threads, "kind": "port",
            "cpu_model": cpu_model(), "host_cpus_visible": os.cpu_count(), "job_cpus": len(job_cpus()),
            "cgroup_cpu_quota": cpu_quota(),
            "sample": f"{label}: {scope}, {secs:.2f} s, {st['predicate_calls']} predicate calls, kbref C++ port, {how}"}


def golden_digest(cid):
    """The oracle's digest of BASELINE config `cid` (tests/golden/make_digests.py), if committed."""
    p = os.path.join(ROOT, "tests", "golden", f"digest_c{cid}.json")
    if not os.path.exists(p):
        return None
    with open(p) as f:
        return json.load(f)


def log_sha(decs, evictions=()):
    """sha256 of a cycle's raw decision log (task, node, kind, dispatched_at)
    and evictions (task, by, action) as the library returned them."""
    import hashlib
    return hashlib.sha256(json.dumps([[list(d) for d in decs], [list(e) for e in evictions]],
                                     separators=(",", ":")).encode()).hexdigest()


def evictions_list(ssn):
    """The session's evictions of the cycle as (task, by, action) index triples."""
    from kbgpu import _abi
    L = _abi.lib()
    n = ctypes.c_int32(0)
    _abi.check(L.kbg_evictions_get(ssn.handle, None, 0, ctypes.byref(n)))
    buf = (_abi.kbg_eviction * max(1, n.value))()
    _abi.check(L.kbg_evictions_get(ssn.handle, buf, n.value, ctypes.byref(n)))
    return [(buf[i].task, buf[i].by, buf[i].action) for i in range(n.value)]


def parity_verdict(cid, digests):
    """{mode: digest} of the timed cycles against the golden digest of the
    config: every mode must match it."""
    from kbgpu.digest import digest_mismatches
    ref = golden_digest(cid)
    out = {"golden": f"tests/golden/digest_c{cid}.json" if ref else None,
           "checked": "the last timed cycle of each mode: decision log (task, job, node, kind, dispatched_at), binds, "
                      "evictions, node and job states bit-exact; drf / proportion shares within 1e-12 relative"}
    ok = True
    for mode, dg in digests.items():
        if ref is None:
            out[mode] = "no golden digest for this config"
            continue
        bad = digest_mismatches(ref, dg)
        out[mode] = True if not bad else {"mismatch": bad}
        ok = ok and not bad
    out["ok"] = ok if ref is not None else None
    return out


def load_pmc(n_nodes, mode):
    """A kernel's per-launch PMC figures from the committed rocprofv3 summary
    of this same bench command (profiles/pmc_scan.json), if it matches the
    workload: the scan kernel in `mode` "full_scan" / "grouped", or the
    victim kernel ("victim", C5)."""
    p = os.path.join(ROOT, "profiles", "pmc_scan.json")
    if not os.path.exists(p):
        return None
    try:
        d = json.load(open(p))
        sec = d.get(mode)
        if sec and sec.get("n_nodes", d.get("n_nodes")) == n_nodes:
            return dict(sec, source=d.get("source"), n_nodes=n_nodes)
        other = d.get("by_nodes", {}).get(str(n_nodes), {})  # other workloads' profiles (C4)
        if other.get(mode):
            return dict(other[mode], source=other.get("source"), n_nodes=n_nodes)
    except (OSError, ValueError):
        pass
    return None


def valu_ceiling(pmc, avg_us, rows=None):
    """The VALU-issue ceiling of a kernel: its PMC wave instructions at 4
    cycles each spread over every SIMD of the chip at the peak clock. With
    `rows`, the profiled count is scaled from the profiled command's rows per
    launch to this run's (the instructions grow with the rows)."""
    insts = pmc["valu_insts_per_launch"]
    scaled = bool(rows and pmc.get("rows_per_launch"))
    if scaled:
        insts = insts / pmc["rows_per_launch"] * rows
    floor_us = insts * VALU_CYC / (SIMDS * CLOCK_GHZ * 1e3)
    out = {"wave_insts_per_launch": insts, "issue_floor_us": floor_us,
           "frac": floor_us / avg_us if avg_us > 0 else None,
           "model": f"{VALU_CYC} cycles per wave64 VALU instruction per SIMD, {SIMDS} SIMDs at {CLOCK_GHZ} GHz"}
    if scaled:
        out["scaled_from_rows_per_launch"] = pmc["rows_per_launch"]
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=30)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", type=int, default=3)
    ap.add_argument("--batch", type=int, default=0)
    ap.add_argument("--candidates", type=int, default=0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-faithful", action="store_true", help="skip the 60 s B-faithful CPU baseline")
    ap.add_argument("--no-resident", action="store_true", help="skip the resident-session (kbg_session_update) lines")
    ap.add_argument("--comm", action="store_true",
                    help="open the session through the RCCL sharded entry point even at N=1 (rehearsal)")
    ap.add_argument("--dist-backend", default="nccl", help="nccl (RCCL) on MI355X; gloo to rehearse on one GPU")
    ap.add_argument("--transport", default="rccl", choices=("rccl", "host"),
                    help="the shards' communicator: rccl (one rank per GPU, xGMI) or host (kbg_comm_init_host: "
                         "shared memory between the rank processes; with KBG_BENCH_DEVICE=0 and --dist-backend gloo "
                         "the N-rank path rehearses on one GPU)")
    ap.add_argument("--dry-run", action="store_true",
                    help="launch, rendezvous and report without touching a GPU (CPU test of --gpus)")
    args = ap.parse_args()
    # --gpus N is authoritative: without a launcher start N ranks, under one
    # its world size must agree
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(spawn_ranks(args.gpus))
    if "WORLD_SIZE" in os.environ and int(os.environ["WORLD_SIZE"]) != args.gpus:
        log(f"bench: --gpus {args.gpus} but the launcher started WORLD_SIZE={os.environ['WORLD_SIZE']} ranks")
        sys.exit(2)
    _capture_stdout()

    import torch
    from kbgpu import dist as kdist
    rank, world, local_rank = kdist.env_rank()
    if args.dry_run:
        kdist.init("gloo")
        log(f"bench: rank {rank} of {world} (local rank {local_rank}) up, dry run")
        kdist.barrier()
        _, ranks = kdist.aggregate(0.0, 1, sharded=False)
        if rank == 0:
            emit({"metric": "dry run", "value": None, "n_gpus": world, "ranks_reporting": ranks, "dry_run": True})
        kdist.shutdown()
        return
    # KBG_BENCH_DEVICE pins every rank to one device (rehearsal on a 1-GPU box only)
    device = int(os.environ.get("KBG_BENCH_DEVICE", local_rank))
    torch.cuda.set_device(device)
    kdist.init(args.dist_backend)

    from kbgpu import _abi, actions, synth  # noqa: F401
    from kbgpu.actions import decision_list, replay
    from kbgpu.cache import FakeBinder, cache_from_fixture
    from kbgpu.digest import digest_outputs
    from kbgpu.fixture import fixture_tiers, session_output
    from kbgpu.framework import open_session

    cid = args.config
    t0 = time.time()
    fx = synth.config_fixture(cid)  # every rank: the same cluster
    cache = cache_from_fixture(fx)
    base_opts = {"device": device}
    comm = None
    rccl_ranks = None  # ranks the RCCL communicator itself reports (ncclCommCount); None: no communicator (N=1)
    if world > 1 or args.comm:
        if args.transport == "host":
            name = kdist.broadcast_bytes(f"bench{os.getpid()}-{time.time_ns() % 10**9}".encode() if rank == 0 else b"")
            comm = kdist.HostComm(name.decode(), rank, world, device)
        else:
            comm = kdist.ShardComm(device)
        base_opts["comm"] = comm
        rccl_ranks, rccl_rank = comm.ranks()
        if rccl_ranks != world or rccl_rank != rank:
            log(f"bench: the RCCL communicator reports rank {rccl_rank} of {rccl_ranks}, the launcher {rank} of {world}")
            sys.exit(2)
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
               "launches": 0, "task_evals": 0, "steps": steps, "alloc_ms": []}
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
            agg["task_evals"] += st.task_evaluations
            agg["alloc_ms"].append(st.allocate_ms)
        torch.cuda.synchronize()
        agg["elapsed"] = time.perf_counter() - t_start
        if barrier:
            kdist.barrier()
        agg["stats"] = ssn.stats()
        # parity of the last timed cycle: its log (still in `buf`, the
        # session not reset since) replayed through the session's host
        # objects, then digested with the library's node / job / queue states
        decs = decision_list(buf, nout.value)
        agg["log_sha256"] = log_sha(decs)
        binder = FakeBinder()
        cache.binder = binder
        replay(ssn, decs, "allocate")
        agg["digest"] = digest_outputs(session_output(ssn, binder.binds))
        agg["n_nodes"] = len(ssn.nodes)
        agg["words"] = (((agg["n_nodes"] + 63) // 64) + world - 1) // world  # 64-node words a rank's launch walks
        agg["pending"] = ssn.flat.pending_count
        agg["jobs"] = len(ssn.jobs)
        agg["queues"] = len(ssn.queues)
        ssn.close()
        return agg

    def cycle_roofline(agg, mode):
        """unit = one reference task evaluation (every task the
        allocate loop pops, placed or not); algorithmic bytes per unit = N x
        64 B (node records) + 32 B (task record); achieved = bytes per cycle /
        median cycle wall time. Whole job: the cycle covers the cluster on all
        ranks, the peak is N GPUs' HBM."""
        units = agg["task_evals"] / max(1, agg["steps"])
        per_cycle = units * (agg["n_nodes"] * NODE_RECORD_B + TASK_RECORD_B)
        t = statistics.median(agg["alloc_ms"]) * 1e-3  # allocate Execute's own wall time (kbg_stats.allocate_ms)
        ach = per_cycle / t / 1e9
        peak = HBM_PEAK_GBS * world
        pmc = load_pmc(agg["n_nodes"], mode) if comm is None else None
        traffic = None
        if pmc and pmc.get("hbm_bytes_per_launch") is not None:  # measured HBM bytes of the scan launches of a cycle
            traffic = pmc["hbm_bytes_per_launch"] * agg["launches"] / max(1, agg["steps"])
        out = {"bound": "hbm", "achieved": ach, "peak": peak, "unit": "GB/s", "frac": ach / peak,
               "traffic": traffic, "scope": "allocate cycle",
               "definition": "SURVEY 8(d): task evaluations x (N x 64 B + 32 B) per allocate cycle / p50 wall time "
                             "of kbg_allocate (allocate Execute); traffic = PMC HBM bytes of the cycle's scan launches",
               "task_evaluations_per_cycle": units, "algo_bytes_per_cycle": per_cycle, "p50_cycle_ms": t * 1e3}
        if ach <= peak:
            return out
        # The 8(d) byte count exceeds what HBM could deliver in the cycle (C4:
        # each wave keeps its 64 node rows in registers across the workgroup's
        # rows, so a node record is not re-read per evaluation): the roofline
        # is then the physical one, the measured HBM bytes of the cycle's scan
        # launches over the cycle, and the 8(d) figure is kept beside it.
        eq = {k: out[k] for k in ("achieved", "frac", "task_evaluations_per_cycle", "algo_bytes_per_cycle")}
        eq["note"] = "SURVEY 8(d) byte count / cycle: above the HBM peak, not a fraction of anything physical"
        phys = traffic / t / 1e9 if traffic is not None else None
        out.update({"achieved": phys, "frac": phys / peak if phys is not None else None,
                    "definition": "PMC HBM bytes (2 x FETCH_SIZE + WRITE_SIZE) of the cycle's scan launches / p50 "
                                  "wall time of kbg_allocate", "equivalent_8d": eq})
        return out

    def pmc_scaled(pmc, rows, words):
        """The profiled kernel's PMC figures per launch, scaled from the
        profiled command's rows per launch (and 64-node words per launch: a
        sharded rank walks its own words) to this run's: VALU instructions grow
        with rows x words."""
        f = 1.0
        if rows and pmc.get("rows_per_launch"):
            f *= rows / pmc["rows_per_launch"]
        pw = pmc.get("words_per_launch") or (pmc.get("n_nodes", 5000) + 63) // 64
        if words and pw:
            f *= words / pw
        return f

    def kernel_roofline(agg, mode):
        """The contract's roofline of the dominant kernel, kbg_firstfit_kernel
        in full-scan mode (every row is one task evaluation scanning all N
        nodes, SURVEY 8(d) cursor rule), against the ceiling that binds it.
        The kernel holds a wave's 64 node records in registers for every row of
        its workgroup and the node table is L2-resident, so HBM is far from
        binding (traffic_frac_of_peak); what bounds a launch is VALU issue:
        achieved = PMC wave64 VALU instructions per launch (profiles/pmc_scan.json,
        scaled to this run's rows and words per launch) / the launch's average
        duration (HIP events around the fused launches on the library's
        stream, over the timed steps), peak = 1024 SIMDs x 2.4 GHz / 4 cycles
        per wave64 instruction. The SURVEY 8(d) byte count (N x 64 B + 32 B per
        task evaluation) over the same launch time is kept as equivalent_8d:
        it charges a node read per (row, node) pair, i.e. on-chip reuse, and
        is not a fraction of a physical peak."""
        launches = max(1, agg["launches"])
        rows = agg["evals"] / launches
        avg_s = agg["scan_ms"] * 1e-3 / launches
        words = agg["words"]
        per_launch = rows * (agg["n_nodes"] * NODE_RECORD_B + TASK_RECORD_B)
        eq = {"achieved": per_launch / avg_s / 1e9 if avg_s > 0 else 0.0, "peak": HBM_PEAK_GBS, "unit": "GB/s",
              "algo_bytes_per_launch": per_launch,
              "definition": "SURVEY 8(d) bytes per task evaluation (N x 64 B + 32 B) x rows per launch / average "
                            "launch time: counts a node record per (row, node) pair, above the HBM peak because "
                            "the kernel reuses each node record on chip for every row"}
        eq["frac"] = eq["achieved"] / HBM_PEAK_GBS
        out = {"bound": "valu", "achieved": None, "peak": VALU_PEAK_GIPS, "unit": "G wave64 VALU instructions/s",
               "frac": None, "traffic": None, "kernel": "kbg_firstfit_kernel (full-scan mode)",
               "avg_launch_us": avg_s * 1e6, "rows_per_launch": rows, "words_per_launch": words,
               "timing": "HIP events on the library stream around every fused launch of the timed full-scan steps "
                         "(kbg_stats.scan_kernel_ms; the production mode samples one launch in four)",
               "equivalent_8d": eq}
        pmc = load_pmc(agg["n_nodes"], mode)
        if pmc:
            f = pmc_scaled(pmc, rows, words)
            if pmc.get("valu_insts_per_launch") is not None and avg_s > 0:
                insts = pmc["valu_insts_per_launch"] * f
                out["achieved"] = insts / avg_s / 1e9
                out["frac"] = out["achieved"] / VALU_PEAK_GIPS
                out["valu_insts_per_launch"] = insts
                out["issue_floor_us"] = insts * VALU_CYC / (SIMDS * CLOCK_GHZ * 1e3)
            if pmc.get("hbm_bytes_per_launch") is not None:
                out["traffic"] = pmc["hbm_bytes_per_launch"] * f
                out["traffic_frac_of_peak"] = out["traffic"] / avg_s / 1e9 / HBM_PEAK_GBS if avg_s > 0 else None
            if pmc.get("wait_any_share") is not None:  # share of the waves' lifetime parked at s_waitcnt / barriers
                out["wait_any_share"] = pmc["wait_any_share"]
            out["pmc_scale"] = f
            out["pmc_source"] = pmc.get("source")
            out["definition"] = ("achieved = PMC SQ_INSTS_VALU per launch (scaled by pmc_scale to this run's rows x "
                                 "words per launch) / average launch time; peak = 1024 SIMDs x 2.4 GHz / 4 cycles "
                                 "per wave64 VALU instruction; traffic = PMC HBM bytes per launch "
                                 "(2 x FETCH_SIZE + WRITE_SIZE)")
        else:  # no profile of this workload: the physical figure is unknown, the 8(d) one stays beside it
            out["definition"] = "no PMC profile of this workload committed under profiles/: achieved unmeasured"
        return out

    def scan_kernel(agg, mode):
        """The dominant device kernel against its physical ceilings: HBM
        (PMC-measured bytes per launch) and VALU issue (PMC-measured wave
        instructions per launch at 4 cycles each on one of 1024 SIMDs). The
        algorithmic GB/s figure counts every (row, node) visit as a 64-B node
        read; the node table is L2-resident and each wave keeps its 64 nodes in
        registers across the workgroup's rows, so that figure is reuse, not
        bandwidth, and is not a fraction of any peak."""
        launches = max(1, agg["launches"])
        algo = agg["visits"] * NODE_RECORD_B + agg["evals"] * TASK_RECORD_B
        avg_us = agg["scan_ms"] * 1e3 / launches
        out = {"kernel": "kbg_firstfit_kernel", "avg_launch_us": avg_us, "launches_per_cycle": launches / max(1, agg["steps"]),
               "rows_per_launch": agg["evals"] / launches, "algo_bytes_per_launch": algo / launches,
               "algo_reuse_gbs": algo / (agg["scan_ms"] * 1e-3) / 1e9 if agg["scan_ms"] > 0 else 0.0}
        pmc = load_pmc(agg["n_nodes"], mode) if comm is None else None
        if pmc:
            if pmc.get("hbm_bytes_per_launch") is not None:
                b = pmc["hbm_bytes_per_launch"]
                out["hbm"] = {"bytes_per_launch": b, "achieved_gbs": b / (avg_us * 1e-6) / 1e9,
                              "peak_gbs": HBM_PEAK_GBS, "frac": b / (avg_us * 1e-6) / 1e9 / HBM_PEAK_GBS}
            if pmc.get("valu_insts_per_launch") is not None:
                out["valu"] = valu_ceiling(pmc, avg_us, agg["evals"] / launches)
            out["pmc_source"] = pmc.get("source")
        return out

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
    full = run_mode(1, max(1, min(10, args.steps)), 2, False)  # SURVEY roofline rule: every task scans all N
    decisions = prod["decisions"]
    elapsed, total_decisions = kdist.aggregate(prod["elapsed"], decisions, sharded=world > 1)
    tp = "RCCL" if comm is None or comm.transport == "rccl" else "host shared-memory"
    st = prod["stats"]
    n_nodes = prod["n_nodes"]

    def breakdown(agg):
        s2 = agg["stats"]
        return {"allocate_ms_p50": statistics.median(agg["alloc_ms"]), "resolve_steps": s2.resolve_steps,
                "resolve_rechecks": s2.resolve_rechecks, "overlapped_batches": s2.overlapped,
                "scan_ms": s2.scan_kernel_ms, "select_ms": s2.select_kernel_ms, "launches": s2.scan_launches,
                "evaluations": s2.evaluations, "batches": s2.batches, "mispredictions": s2.mispredictions,
                "truncations": s2.truncations, "replayed": s2.replayed, "host_engine_ms": s2.engine_ms,
                "host_resolve_ms": s2.resolve_ms, "device_roundtrip_ms": s2.device_ms,
                "delta_writeback_ms": s2.delta_ms, "exchange_ms": s2.exchange_ms, "shards": s2.shards,
                "owner_rounds": s2.owner_rounds, "refresh_scans": s2.refresh_scans,
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
                   "parallelism": ((f"node-axis shards x{world} (owner-resolve: batch broadcast, {tp} sum/min-reduce "
                                    f"of availability and packed winners)") if os.environ.get("KBG_OWNER_RESOLVE") == "1"
                                   else (f"node-axis shards x{world} (scan service: rank 0 commits, {tp} broadcast of "
                                         f"each launch, every rank scans its rows, {tp} sum-reduce of the word masks)"))
                                  if world > 1 else "single-gpu",
                   "batch_tasks": base_opts.get("batch_tasks", 8192),
                   "candidates": base_opts.get("candidates", 32)},
        "roofline": kernel_roofline(full, "full_scan"),
        "roofline_note": "full-scan mode (every task evaluation scans all N nodes on the device, SURVEY 8(d) cursor "
                         "rule); bound = VALU issue (PMC), HBM traffic and the 8(d) byte figure beside it; `value` "
                         "is the production mode, which groups identical (class, request) shapes",
        "rccl_ranks": rccl_ranks,
        "comm_transport": comm.transport if comm is not None else None,
        "cycle_roofline_8d": cycle_roofline(full, "full_scan"),
        "scan_kernel": scan_kernel(full, "full_scan"),
        "full_scan_mode": {"placements_per_s": full["decisions"] / full["elapsed"],
                           "p50_cycle_ms": statistics.median(full["cycle_ms"]), "breakdown": breakdown(full)},
        "production_mode": {"equivalent_8d": {("equiv_frac" if k == "frac" else k): v
                                              for k, v in cycle_roofline(prod, "grouped").items()
                                              if k not in ("bound", "peak", "unit")},
                            "equivalent_8d_note": "the 8(d) byte count over the production cycle: grouping skips "
                                                  "work, so this is not a roofline claim",
                            "scan_kernel": scan_kernel(prod, "grouped"), "breakdown": breakdown(prod)},
        "decisions_per_cycle": decisions // max(1, args.steps),
        "open_ms": st.open_ms,
        "open_ms_first_in_process": open_ms_first,
        "parity": dict(parity_verdict(cid, {"production": prod["digest"], "full_scan": full["digest"]}),
                       log_sha256={"production": prod["log_sha256"], "full_scan": full["log_sha256"]}),
    }
    if world == 1 and not args.no_resident:
        line["resident_session"] = resident_bench(cache, fx, base_opts)
    if world == 1 and not args.no_cpu_baseline:  # the CPU baseline is an N=1 figure
        # bounded samples where a full cycle takes longer than ~30 s of CPU
        # (C3's failing tasks walk every node, C4 is 500k tasks)
        budget = {1: 0.0, 2: 0.0, 3: 20.0}.get(cid, 60.0)
        mask = job_cpus()
        if hasattr(os, "sched_setaffinity") and len(mask) > 2:
            os.sched_setaffinity(0, {mask[0]})  # this process (and its idle runtime threads) off the team's CPUs
        line["cpu_baseline"] = cpu_baseline(fx, f"C{cid}", 1, budget=budget)
        sweep = [cpu_baseline(fx, f"C{cid}", t, budget=budget) for t in omp_sweep()]
        sweep = [b for b in sweep if b]
        if sweep:
            line["cpu_baseline_omp"] = max(sweep, key=lambda b: b["value"])
            line["cpu_baseline_omp_sweep"] = [{"cores": b["cores"], "value": b["value"], "sample": b["sample"]}
                                              for b in sweep]
        if not args.no_faithful:
            line["cpu_baseline_faithful"] = cpu_baseline(fx, f"C{cid}", 1, faithful=True, budget=20.0)
        if hasattr(os, "sched_setaffinity") and len(mask) > 2:
            os.sched_setaffinity(0, set(mask))
    if rank == 0:
        emit(line)
    if comm is not None:
        comm.close()
    kdist.shutdown()
    if line["parity"]["ok"] is False:
        log(f"bench: PARITY MISMATCH against {line['parity']['golden']}: {line['parity']}")
        sys.exit(3)


def resident_bench(cache, fx, base_opts, steps=5, churn=0.01, seed=5):
    """Resident session (kbg_session_update, include/kbgpu.h) on the same
    cluster: open once, run a cycle, confirm every Allocate decision's bind
    as a cache event (the pod Running on its node), then `steps` cycles of
    churn — `churn` x pods complete (Running -> Succeeded, they leave their
    nodes) and as many new pods arrive for random jobs (copies of a job's pod
    spec and request) — each an update plus an allocate cycle. Times are the
    library's own (kbg_stats.update_ms / allocate_ms); the events are built
    in numpy, outside the timed calls."""
    import random
    from kbgpu import _abi
    from kbgpu.fixture import fixture_tiers
    from kbgpu.framework import open_session
    L = _abi.lib()
    ssn = open_session(cache, fixture_tiers(fx), dict(base_opts))
    rng = random.Random(seed)
    tasks = ssn.flat.arrays["tasks"]
    T = len(ssn.flat.task_objs)
    cap = T + int(T * churn * (steps + 1)) + 16
    buf = (_abi.kbg_decision * cap)()
    n = ctypes.c_int32(0)
    _abi.check(L.kbg_allocate(ssn.handle, buf, cap, ctypes.byref(n)))
    first_ms = ssn.stats().allocate_ms
    running = {}  # task -> node
    evs = (_abi.kbg_event * max(1, n.value))()
    k = 0
    for i in range(n.value):
        d = buf[i]
        if d.kind == _abi.KIND_ALLOCATE:
            e = evs[k]
            e.kind, e.task, e.status, e.node = _abi.EV_POD_UPDATE, d.task, 1 << 5, d.node  # Running
            running[d.task] = d.node
            k += 1
    _abi.check(L.kbg_session_update(ssn.handle, evs, k))
    bind_ms = ssn.stats().update_ms
    out = {"open_ms": ssn.stats().open_ms, "first_cycle_allocate_ms": first_ms, "bind_events": k,
           "bind_update_ms": bind_ms, "churn_events_per_step": 0, "churn_update_ms": [], "churn_allocate_ms": [],
           "churn_placements": []}
    keep = []
    jobs_of = {}
    for t in range(T):
        jobs_of.setdefault(int(tasks[t]["job"]), t)
    job_ids = sorted(jobs_of)
    binds = []  # (task, node) of the last cycle's Allocate decisions, confirmed in the next update
    for step in range(steps):
        m = int(len(running) * churn)
        done = rng.sample(sorted(running), m)
        evs = (_abi.kbg_event * (len(binds) + 2 * m))()
        i = 0
        for t, nd in binds:
            evs[i].kind, evs[i].task, evs[i].status, evs[i].node = _abi.EV_POD_UPDATE, t, 1 << 5, nd  # Running
            running[t] = nd
            i += 1
        for t in done:
            if t not in running:
                continue
            evs[i].kind, evs[i].task, evs[i].status, evs[i].node = _abi.EV_POD_UPDATE, t, 1 << 7, running.pop(t)
            i += 1
        for a in range(m):
            base = jobs_of[job_ids[rng.randrange(len(job_ids))]]
            src = tasks[base]
            e = evs[i]
            e.kind, e.job, e.spec, e.status, e.node = _abi.EV_POD_ADD, int(src["job"]), int(src["spec"]), 1, -1
            e.priority = int(src["priority"])
            e.resource = _abi.kbg_resource(*[float(x) for x in src["resreq"]])
            keep += [f"churn-{step}-{a}".encode(), f"churn/{step}-{a}".encode()]
            e.uid, e.pod_key = keep[-2], keep[-1]
            i += 1
        _abi.check(L.kbg_session_update(ssn.handle, evs, i))
        out["churn_update_ms"].append(ssn.stats().update_ms)
        out["churn_events_per_step"] = i
        _abi.check(L.kbg_allocate(ssn.handle, buf, cap, ctypes.byref(n)))
        out["churn_allocate_ms"].append(ssn.stats().allocate_ms)
        out["churn_placements"].append(n.value)
        binds = [(buf[j].task, buf[j].node) for j in range(n.value) if buf[j].kind == _abi.KIND_ALLOCATE]
    # one structural update (ABI 13): a node and a PodGroup with 8 pods join, the last job's PodGroup
    # leaves — the session rebuilds from its own updated snapshot — then an allocate cycle
    nd0 = ssn.flat.arrays["nodes"][0]
    spec = _abi.kbg_node_spec(b"bench-new-node", None, 0, 0, None)
    evs = (_abi.kbg_event * 11)()
    evs[0].kind, evs[0].node_spec = _abi.EV_NODE_ADD, ctypes.pointer(spec)
    evs[0].resource = _abi.kbg_resource(*[float(x) for x in nd0["allocatable"]])
    evs[0].max_task_num = int(nd0["max_task_num"])
    evs[1].kind, evs[1].name, evs[1].queue, evs[1].min_available = _abi.EV_JOB_ADD, b"bench/new-job", 0, 8
    new_job = len(ssn.jobs)
    src = tasks[jobs_of[job_ids[0]]]
    for a in range(8):
        e = evs[2 + a]
        e.kind, e.job, e.spec, e.status, e.node = _abi.EV_POD_ADD, new_job, int(src["spec"]), 1, -1
        e.priority = int(src["priority"])
        e.resource = _abi.kbg_resource(*[float(x) for x in src["resreq"]])
        keep += [f"struct-{a}".encode(), f"bench/struct-{a}".encode()]
        e.uid, e.pod_key = keep[-2], keep[-1]
    evs[10].kind, evs[10].job = _abi.EV_JOB_DELETE, job_ids[-1]
    _abi.check(L.kbg_session_update(ssn.handle, evs, 11))
    out["structural_events"] = 11
    out["structural_update_ms"] = ssn.stats().update_ms
    _abi.check(L.kbg_allocate(ssn.handle, buf, cap, ctypes.byref(n)))
    out["structural_allocate_ms"] = ssn.stats().allocate_ms
    ssn.close()
    out["churn_update_ms_p50"] = statistics.median(out["churn_update_ms"])
    out["churn_allocate_ms_p50"] = statistics.median(out["churn_allocate_ms"])
    out["note"] = ("kbg_session_update replaces a session open per cycle (open_ms): binds of the first cycle, then "
                   f"{churn:.0%} completions + {churn:.0%} new pods + the last cycle's binds per update, each "
                   "followed by an allocate cycle; structural_update_ms: one update in which a node and a PodGroup "
                   "with 8 pods join and a PodGroup leaves (the session rebuilds from its own updated snapshot)")
    return out


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
    from kbgpu.actions import decision_list
    from kbgpu.cache import FakeBinder
    from kbgpu.digest import digest_outputs
    from kbgpu.fixture import fixture_tiers, session_output
    from kbgpu.framework import get_action, open_session

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
    # parity: the last timed cycle's raw log, then one more cycle on the reset
    # session through the framework's actions (the same entry points, each
    # action's decisions and evictions replayed through the session) whose
    # log must be the timed one and whose digest must be the oracle's
    timed_sha = log_sha(decision_list(buf, nout.value), evictions_list(ssn))
    binder = FakeBinder()
    cache.binder = binder
    _abi.check(L.kbg_session_reset(ssn.handle))
    for name in fx["actions"]:
        get_action(name).execute(ssn)
    verify_sha = log_sha(ssn.decisions, evictions_list(ssn))
    digest = digest_outputs(session_output(ssn, binder.binds))
    ssn.close()
    elapsed, total = kdist.aggregate(elapsed_local, dec, sharded=world > 1)
    nodes_per_rank = n_nodes / max(1, world)
    algo = nodes_per_rank * NODE_RECORD_B + running / max(1, world) * TASK_RECORD_B
    launch_us = vms * 1e3 / max(1, vscans)
    ach = algo / (launch_us * 1e-6) / 1e9 if launch_us > 0 else 0.0
    pmc = load_pmc(n_nodes, "victim") if comm is None else None
    # both physical ceilings of the victim kernel; `bound` is the one it is closest to
    roof = {"bound": "hbm", "achieved": ach, "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": ach / HBM_PEAK_GBS,
            "traffic": pmc["hbm_bytes_per_launch"] if pmc else None, "kernel": "kbg_victim_kernel",
            "avg_launch_us": launch_us, "algo_bytes_per_launch": algo,
            "definition": "N x 64 B + R x 32 B per launch (DESIGN.md §5) / average launch time (HIP events, one "
                          "launch in 16)"}
    if pmc:
        roof["valu"] = valu_ceiling(pmc, launch_us)
        roof["pmc_source"] = pmc.get("source")
        roof["traffic_frac_of_peak"] = pmc["hbm_bytes_per_launch"] / (launch_us * 1e-6) / 1e9 / HBM_PEAK_GBS
        vf = roof["valu"].get("frac")
        if vf is not None and vf > roof["frac"]:
            hbm = {k: roof[k] for k in ("achieved", "peak", "unit", "frac", "definition")}
            insts = roof["valu"]["wave_insts_per_launch"]
            roof.update({"bound": "valu", "achieved": insts / (launch_us * 1e-6) / 1e9, "peak": VALU_PEAK_GIPS,
                         "unit": "G wave64 VALU instructions/s", "frac": vf, "hbm_algorithmic": hbm,
                         "definition": "PMC SQ_INSTS_VALU per launch / average launch time; peak = 1024 SIMDs x "
                                       "2.4 GHz / 4 cycles per wave64 instruction"})
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
        "roofline": roof,
        "rccl_ranks": comm.ranks()[0] if comm is not None else None,
        "decisions_per_cycle": dec // max(1, args.steps),
        "evictions_per_cycle": ev // max(1, args.steps),
        "victim_scans_per_cycle": vscans // max(1, args.steps),
        "victim_tries_per_cycle": vtries // max(1, args.steps),
        "victim_host_evals_per_cycle": vevals // max(1, args.steps),
        "phase_ms_p50": {k: statistics.median(v) for k, v in phase.items()},
        "open_ms": st.open_ms,
        "open_ms_first_in_process": open_ms_first,
    }
    par = parity_verdict(cid, {"cycle": digest})
    par["timed_cycle_log_sha256"] = timed_sha
    par["verify_cycle_log_equal"] = verify_sha == timed_sha
    par["checked"] = ("the last timed cycle's raw log (decisions and evictions) equals that of one more cycle on the "
                      "reset session through the framework's actions, whose outputs (" + par["checked"] + ") match "
                      "the golden digest")
    if not par["verify_cycle_log_equal"]:
        par["ok"] = False
    line["parity"] = par
    if world == 1 and not args.no_cpu_baseline:
        line["cpu_baseline"] = cpu_baseline(fx, f"C{cid} ({', '.join(fx['actions'])})")
    if rank == 0:
        emit(line)
    if comm is not None:
        comm.close()
    kdist.shutdown()
    if par["ok"] is False:
        log(f"bench: PARITY MISMATCH: {par}")
        sys.exit(3)


if __name__ == "__main__":
    main()
