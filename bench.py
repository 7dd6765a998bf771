#!/usr/bin/env python3
"""Benchmark: fast_consensus() hot path on MI355X (BASELINE.json metric).

  python bench.py [--gpus N] [--steps K] [--warmup W] [--config lfr1m|lfr100k|lfr100k_lpm|lfr1k|sbm4m]

One step = one whole fast_consensus(G, algorithm, n_p, tau, delta) call as §8(d) metric (1)
defines it: graph upload from host arrays (PCIe + device ingest + CSR build) -> every
consensus iteration -> the final pass -> the n_p final labelings landed in a host array.
value = partition*edges/s = (sum_iter n_p*m_iter + n_p*m_final) / wall, aggregated over all
ranks (replicas are sharded: strong scaling, n_p fixed).  The loop alone (graph already
resident) is reported beside it as `loop_ms_per_step`.

--gpus N > 1 without a torch.distributed launcher: this script starts N ranks under
torch.distributed.run itself (one per GPU, RCCL) and exits with their status.  Under a
launcher, --gpus must equal WORLD_SIZE (a mismatch exits non-zero, never a mislabelled line).
Progress goes to stderr; rank 0 prints ONE JSON line on stdout.
"""
import argparse
import json
import math
import os
import socket
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "consensus wall time + partition·edges/sec, LFR 1M nodes n_p=64, 1/2/4/8 GPUs"
HBM_PEAK_GBS = 8000.0   # MI355X_MICROARCH.md: HBM3E 8 TB/s peak (spec)
GATHER_LINE_CEILING_GBS = 7168.0   # measured: 56 G L2-miss requests/s x 128 B (profiles/r02_micro_gather.json)

CONFIGS = {
    # BASELINE.json configs[3] (C4): the metric's workload
    "lfr1m": dict(kind="lfr", n=1_000_000, mu=0.5, algo="louvain", n_p=64, tau=0.2, delta=0.02,
                  desc="LFR n=1,000,000 mu=0.5 tau1=3 tau2=1.5 avg_deg~27.5 max_deg=50 comm 20-100, louvain n_p=64"),
    # configs[2] (C3)
    "lfr100k": dict(kind="lfr", n=100_000, mu=0.5, algo="louvain", n_p=64, tau=0.2, delta=0.02,
                    desc="LFR n=100,000 mu=0.5, louvain n_p=64"),
    "lfr100k_lpm": dict(kind="lfr", n=100_000, mu=0.5, algo="lpm", n_p=64, tau=0.8, delta=0.02,
                        desc="LFR n=100,000 mu=0.5, lpm n_p=64"),
    # configs[1] (C2)
    "lfr1k": dict(kind="lfr", n=1_000, mu=0.4, algo="louvain", n_p=20, tau=0.2, delta=0.02,
                  desc="LFR n=1,000 mu=0.4, louvain n_p=20"),
    # the leiden branch (fast_consensus.py:204-258) on the C4 / C3 graphs
    "lfr1m_leiden": dict(kind="lfr", n=1_000_000, mu=0.5, algo="leiden", n_p=64, tau=0.2, delta=0.02,
                         desc="LFR n=1,000,000 mu=0.5, leiden n_p=64"),
    "lfr100k_leiden": dict(kind="lfr", n=100_000, mu=0.5, algo="leiden", n_p=64, tau=0.2, delta=0.02,
                           desc="LFR n=100,000 mu=0.5, leiden n_p=64"),
    # the infomap branch (fast_consensus.py:260-310 with :268) on the C3 graph, default tau 0.6 (:426)
    "lfr100k_infomap": dict(kind="lfr", n=100_000, mu=0.5, algo="infomap", n_p=64, tau=0.6, delta=0.02,
                            desc="LFR n=100,000 mu=0.5, infomap n_p=64"),
    "lfr1m_infomap": dict(kind="lfr", n=1_000_000, mu=0.5, algo="infomap", n_p=64, tau=0.6, delta=0.02,
                          desc="LFR n=1,000,000 mu=0.5, infomap n_p=64"),
    # configs[4] (C5)
    "sbm4m": dict(kind="sbm", n=4_000_000, algo="lpm", n_p=128, tau=0.8, delta=0.02,
                  desc="SBM n=4,000,000 blocks of 100, ~40M edges, lpm n_p=128"),
}


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def make_graph(cfg, seed):
    from fastconsensus_amd import synth
    if cfg["kind"] == "lfr":
        u, v, planted = synth.lfr(cfg["n"], cfg["mu"], seed=seed)
    else:
        u, v = synth.sbm(cfg["n"], seed=seed)
        planted = None
    return cfg["n"], u, v, planted


# ------------------------------------------------------------------------------- CPU baseline
def host_cpu_share():
    """CPUs this process may use: its affinity set, capped by a cgroup CPU quota (a GPU box
    grants each GPU a share of the machine; os.cpu_count() shows the whole machine)."""
    n = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    for path in ("/sys/fs/cgroup/cpu.max",):
        try:
            q, p = open(path).read().split()[:2]
            if q != "max":
                n = min(n, max(1, math.ceil(int(q) / int(p))))
        except (OSError, ValueError):
            pass
    try:
        q = int(open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us").read())
        p = int(open("/sys/fs/cgroup/cpu/cpu.cfs_period_us").read())
        if q > 0:
            n = min(n, max(1, math.ceil(q / p)))
    except (OSError, ValueError):
        pass
    return n


def cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cpu_baseline(n, u, v, cfg, seed):
    """Reference-semantics CPU port (oracle/, kind 'port') on every host core this process may
    use: ONE full consensus iteration (fast_consensus.py:141-202 louvain / :260-310 lpm) --
    the sequential python-louvain level-0 / igraph-LPA restatement per replica (replicas in
    parallel over threads), the O(m*n_p) consensus rule, threshold, check, closure over
    L = m attempts (O(L): the reference's O(N)-per-sample NodeView conversion is NOT
    reproduced) and isolate repair.  Bounded sample: the CD runs `threads` replicas (one
    per thread, all in parallel); the per-iteration time for n_p replicas scales the CD and
    consensus parts by ceil(n_p / threads) and n_p / threads."""
    from oracle import oracle as orc
    threads = host_cpu_share()
    n_p = cfg["n_p"]
    reps = max(1, min(n_p, threads))
    g = orc.EdgeGraph.from_lines(n, np.stack([u, v], 1))
    if cfg["algo"] == "leiden":
        # the leiden branch on integer nodes is n_p Leiden runs on G (fc_run, capi.cpp)
        t0 = time.perf_counter()
        orc.cd_batch(orc.LEIDEN, reps, g, seed=seed, nthreads=threads)
        cd_s = time.perf_counter() - t0
        full_s = cd_s * math.ceil(n_p / reps)
        return {"value": n_p * g.m / full_s, "unit": "partition·edges/s", "cores": threads, "kind": "port",
                "cpu_model": cpu_model(), "host_cpus_visible": os.cpu_count(), "iteration_s": full_s,
                "sample_s": cd_s,
                "sample": "%d sequential Leiden runs (orc_leiden, the leidenalg restatement) in parallel on %d "
                          "threads (%s) %.2fs; value = n_p*m / (that time x ceil(n_p/threads)=%d) at n_p=%d"
                          % (reps, threads, cpu_model(), cd_s, math.ceil(n_p / reps), n_p)}
    algo = 0 if cfg["algo"] == "louvain" else 1          # the loop: louvain, or lpm (lpm, infomap)
    cd_algo = orc.INFOMAP if cfg["algo"] == "infomap" else algo
    t = {}
    t0 = time.perf_counter()
    lab, _ = orc.cd_batch(cd_algo, reps, g, seed=seed, nthreads=threads)
    t["cd"] = time.perf_counter() - t0
    t0 = time.perf_counter()
    w = orc.consensus(algo, g, lab, reps)
    t["consensus"] = time.perf_counter() - t0
    t0 = time.perf_counter()
    keep = orc.threshold(w, cfg["tau"], reps)
    kept = orc.EdgeGraph(n, g.u[keep], g.v[keep], w[keep], g.age[keep])
    orc.check(kept.w, reps, cfg["delta"])
    t["threshold"] = time.perf_counter() - t0
    t0 = time.perf_counter()
    pairs = orc.closure_sample_pairs(kept, g.m, seed, 0, orc.closure_rounds(algo))
    cu, cv, cw, cf = orc.closure_from_pairs(algo, kept, pairs, lab, reps)
    closure = orc.EdgeGraph(n, cu, cv, cw, (np.int64(1) << orc.AGE_ITER_SHIFT) + cf)
    t["closure"] = time.perf_counter() - t0
    t0 = time.perf_counter()
    parts = [kept, closure]
    if algo == 0:
        ru, rv, rw, rx = orc.repair(g, kept.degrees() + closure.degrees())
        parts.append(orc.EdgeGraph(n, ru, rv, rw, (np.int64(1) << orc.AGE_ITER_SHIFT) + orc.AGE_REPAIR_OFFSET + rx))
    new = orc.concat(parts)
    orc.check(new.w, reps, cfg["delta"])
    t["repair_swap"] = time.perf_counter() - t0
    sample_s = sum(t.values())
    full_s = (t["cd"] * math.ceil(n_p / reps) + t["consensus"] * n_p / reps + t["threshold"] + t["closure"]
              + t["repair_swap"])
    return {"value": n_p * g.m / full_s, "unit": "partition·edges/s", "cores": threads, "kind": "port",
            "cpu_model": cpu_model(), "host_cpus_visible": os.cpu_count(),
            "iteration_s": full_s, "sample_s": sample_s,
            "sample": "ONE full consensus iteration of the reference-semantics C port on %d threads (the CPU "
                      "share of this process: affinity/cgroup quota; %d CPUs visible; %s): %d sequential %s "
                      "level-0 replicas in parallel %.2fs, consensus %.2fs, threshold+check %.2fs, closure over "
                      "L=%d attempts %.2fs, repair+swap %.2fs (n=%d, m=%d). value = n_p*m / one iteration at "
                      "n_p=%d (CD scaled by ceil(n_p/threads)=%d, consensus by n_p/threads): %.1fs per iteration"
                      % (threads, os.cpu_count() or 0, cpu_model(), reps, cfg["algo"], t["cd"], t["consensus"],
                         t["threshold"], g.m, t["closure"], t["repair_swap"], n, g.m, n_p,
                         math.ceil(n_p / reps), full_s)}


def load_traffic(config, kernel="k_decide_light"):
    """HBM bytes per launch of the decide kernel `kernel` (k_decide_light, or the k_rl_decide
    family) from profiles/pmc_<config>.json, only when that profile was taken on a library built
    from the same sources as the one being timed (csrc_hash); returns (bytes or None, note)."""
    from fastconsensus_amd.build import built_hash
    p = os.path.join(ROOT, "profiles", "pmc_%s.json" % config)
    if not os.path.exists(p):
        return None, "no PMC profile for %s" % config
    with open(p) as f:
        d = json.load(f)
    lib, prof = built_hash(), d.get("csrc_hash")
    if not lib or prof != lib:
        return None, "PMC profile %s is from csrc %s, the timed library from %s: traffic not attached" % (
            os.path.basename(p), prof, lib)
    key = "rl_decide_hbm_bytes_per_launch" if kernel == "k_rl_decide" else "decide_hbm_bytes_per_launch"
    return d.get(key), "traffic of %s from %s (csrc %s)" % (kernel, os.path.basename(p), prof)


def load_lv_traffic(config, kernel):
    """Leiden / Infomap: HBM bytes per launch of `kernel` from a same-hash PMC profile."""
    from fastconsensus_amd.build import built_hash
    p = os.path.join(ROOT, "profiles", "pmc_%s.json" % config)
    if not os.path.exists(p):
        return None, "no PMC profile for %s" % config
    with open(p) as f:
        d = json.load(f)
    lib, prof = built_hash(), d.get("csrc_hash")
    if not lib or prof != lib:
        return None, "PMC profile %s is from csrc %s, the timed library from %s: traffic not attached" % (
            os.path.basename(p), prof, lib)
    t = d.get("lv_hbm_bytes_per_launch", {}).get(kernel)
    return t, ("traffic of %s from %s (csrc %s)" % (kernel, os.path.basename(p), prof)) if t else \
        "no %s counters in %s" % (kernel, os.path.basename(p))


# ------------------------------------------------------------------------------- launcher
def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def launch_ranks(n):
    """Start n ranks of this script under torch.distributed.run (a child process: nothing in
    this parent touches the GPU) and return their exit status."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(n),
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")   # dmabuf IPC only on this pool (RCCL)
    log("[launcher] %s" % " ".join(cmd))
    return subprocess.call(cmd, env=env)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--config", default="lfr1m", choices=sorted(CONFIGS))
    ap.add_argument("--seed", type=int, default=42)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--buckets", type=int, default=0)
    ap.add_argument("--chunk", type=int, default=-1, help="CD visit-order chunk (engine option; -1 = default)")
    ap.add_argument("--dist-backend", default="nccl", help="nccl (RCCL) in production; gloo to rehearse N>1 on one GPU")
    ap.add_argument("--prune", type=int, default=-1, help="CD vertex pruning (engine option; -1 = default)")
    ap.add_argument("--relabel", type=int, default=-1, help="internal vertex numbering (engine option; -1 = default)")
    ap.add_argument("--store", type=int, default=-1, help="label storage order (engine option; -1 = default)")
    ap.add_argument("--coarsen", type=int, default=-1, help="experimental coarse rounds, largest g (engine option)")
    ap.add_argument("--opt", action="append", default=[], metavar="NAME=VALUE",
                    help="experiment: any engine option (fastconsensus_amd._lib option names), repeatable")
    ap.add_argument("--n-p", type=int, default=0, help="experiment: override the config's n_p")
    ap.add_argument("--no-pin-out", action="store_true",
                    help="leave the preallocated output array pageable (default: page-locked at allocation)")
    ap.add_argument("--gather-out", action="store_true",
                    help="N>1: all-gather the labelings to rank 0 and download there (default: one shared-memory "
                         "host array, each rank writes its rows)")
    ap.add_argument("--resident", action="store_true",
                    help="experiment: time the loop only (graph loaded once before timing)")
    ap.add_argument("--engine-model", action="store_true",
                    help="TEST HOOK (launcher tests on CPU): the oracle-backed CPU model of the engine "
                         "replaces the HIP engine; the line is marked and carries no throughput claim")
    args = ap.parse_args()
    cfg = dict(CONFIGS[args.config])
    if args.n_p > 0:
        cfg["n_p"] = args.n_p
        cfg["desc"] += " (n_p overridden: %d)" % args.n_p

    if "WORLD_SIZE" not in os.environ:
        if args.gpus > 1:
            sys.exit(launch_ranks(args.gpus))
        world = 1
    else:
        world = int(os.environ["WORLD_SIZE"])
        if world != args.gpus:
            log("bench.py: --gpus %d but WORLD_SIZE=%d: refusing to report a mislabelled line" % (args.gpus, world))
            sys.exit(2)
    rank = int(os.environ.get("RANK", "0"))

    import torch
    import torch.distributed as dist

    model = args.engine_model
    if model:
        local, dev = 0, "cpu"
    else:
        local = int(os.environ.get("LOCAL_RANK", "0"))
        local = local % max(1, torch.cuda.device_count())   # rehearsal: several ranks may share one GPU
        dev = "cuda:%d" % local
    backend = "gloo" if model else args.dist_backend
    if world > 1:
        if not model:
            torch.cuda.set_device(local)
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)
        ws = dist.get_world_size()
        one = torch.ones(1, dtype=torch.int32, device=dev)
        dist.all_reduce(one)                       # the collective path itself agrees on the world
        log("[rank %d] process group: backend=%s world_size=%d all_reduce(1)=%d"
            % (rank, dist.get_backend(), ws, int(one.item())))
        if ws != args.gpus or int(one.item()) != args.gpus:
            log("bench.py: process group reports %d ranks, --gpus %d" % (ws, args.gpus))
            sys.exit(2)

    from fastconsensus_amd.core import ALGORITHMS
    from fastconsensus_amd.distributed import run_sharded

    t0 = time.time()
    n, u, v, planted = make_graph(cfg, args.seed)
    log("[rank %d] graph n=%d m=%d generated in %.1fs" % (rank, n, len(u), time.time() - t0))
    if model:
        from tests.cpu_engine import OracleEngine
        eng = OracleEngine(seed=args.seed)
    else:
        import fastconsensus_amd as fc
        eng = fc.Engine(device=local, seed=args.seed)
        from fastconsensus_amd.core import store_order_pays
        from fastconsensus_amd.distributed import shard
        r0, r1 = shard(cfg["n_p"], rank, world)
        eng.set_option("store", store_order_pays(r1 - r0, ALGORITHMS[cfg["algo"]],
                                                int(dict(kv.split("=", 1) for kv in args.opt).get("cd_engine", 2))))
        from fastconsensus_amd.core import relabel_for
        eng.set_option("relabel", relabel_for(ALGORITHMS[cfg["algo"]]))
        if args.buckets:
            eng.set_params(buckets=args.buckets)
        for name in ("chunk", "prune", "relabel", "store", "coarsen"):
            val = getattr(args, name)
            if val >= 0:
                eng.set_option(name, val)
        for kv in args.opt:
            name, val = kv.split("=", 1)
            eng.set_option(name, int(val))
    algo = ALGORITHMS[cfg["algo"]]

    # the final labelings land in ONE host array, allocated and faulted in before timing: a
    # fresh 256 MB array costs ~20 ms of OS page zeroing on first touch, which is the
    # allocator's cost, not the path's; the PCIe download itself stays inside every step
    host_out = np.zeros((cfg["n_p"], n), np.int32) if rank == 0 else None
    # N > 1: one shared-memory host array for the node; each rank downloads its own replica
    # rows over its own PCIe link (no device all-gather, no n_p*n download through rank 0)
    shared = None
    if world > 1 and not args.gather_out:
        from fastconsensus_amd.distributed import SharedOutput, shard as _shard
        shared = SharedOutput(cfg["n_p"], n)
        if shared.array is None:
            log("[rank %d] /dev/shm cannot hold the labelings: all-gather to rank 0 instead" % rank)
            shared = None
        else:
            a0, a1 = _shard(cfg["n_p"], rank, world)
            shared.array[a0:a1] = 0        # fault this rank's pages in before timing
            host_out = shared.array

    # the output array is page-locked at allocation (like its first touch: the allocator's cost),
    # so each step's download is one DMA; --no-pin-out measures the pageable copy
    # (one GPU only: the shared-memory array of N > 1 stays pageable)
    pinned = None
    if not model and not args.no_pin_out and host_out is not None and world == 1:
        from fastconsensus_amd.core import PinnedHost
        pinned = PinnedHost(host_out)
        log("[rank %d] output array pinned: %s" % (rank, pinned.ok))

    def sync():
        if not model:
            torch.cuda.synchronize()

    def step(load, seed):
        """(stats, load seconds, loop seconds) of one fast_consensus call with engine seed
        `seed` (the run's randomness -- numbering, CD orders, closure -- and so its iteration
        count vary with it; SURVEY §8(d): several seeds, each step its own)."""
        if model:
            eng.seed = seed
        elif load:
            eng.set_option("seed", seed)
        t = time.perf_counter()
        if load:
            eng.load_graph(n, u, v)            # §8(d) metric (1): upload + ingest are inside the call
        t1 = time.perf_counter()
        if world == 1 and not model:
            _, st = eng.run(algo, cfg["n_p"], cfg["tau"], cfg["delta"], out=host_out)
        else:
            _, st = run_sharded(eng, algo, cfg["n_p"], cfg["tau"], cfg["delta"], device=dev, out=host_out,
                                out_shared=shared is not None)
        sync()
        t2 = time.perf_counter()
        return st, t1 - t, t2 - t1

    if args.resident:
        eng.load_graph(n, u, v)
        sync()
    m0 = len(u)
    for w in range(args.warmup):
        st, tl, tr = step(not args.resident, args.seed + 1000 + w)
        m0 = eng.graph_info()[2]
        log("[rank %d] warmup %d: load %.1f ms + loop %.1f ms, iterations=%d exit=%d m_final=%d" %
            (rank, w, 1e3 * tl, 1e3 * tr, st["iterations"], st["exit_check"], st["m_final"]))
    if not model:
        eng.set_timing(True)
        eng.collect_timing()  # reset the event log
    if world > 1:
        dist.barrier()
    sync()
    t_start = time.perf_counter()
    pe_total, iters, m_finals, load_s, loop_s = 0, [], [], 0.0, 0.0
    per_step = []
    for k in range(args.steps):
        st, tl, tr = step(not args.resident, args.seed + k)
        per_step.append({"seed": args.seed + k, "ms": 1e3 * (tl + tr), "iterations": st["iterations"],
                         "partition_edges": st["partition_edges"]})
        pe_total += st["partition_edges"]
        iters.append(st["iterations"])
        m_finals.append(st["m_final"])
        load_s += tl
        loop_s += tr
        log("[rank %d] step %d: load %.1f ms + loop %.1f ms, iterations=%d exit=%d m_final=%d" %
            (rank, k, 1e3 * tl, 1e3 * tr, st["iterations"], st["exit_check"], st["m_final"]))
    sync()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t_start
    m0 = eng.graph_info()[2]
    tim = eng.collect_timing() if not model else None
    if not model:
        eng.set_timing(False)
    if world > 1:
        tt = torch.tensor([elapsed, load_s, loop_s], dtype=torch.float64, device=dev)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        elapsed, load_s, loop_s = (float(x) for x in tt.tolist())
    value = pe_total / elapsed

    roof, phases = None, None
    if tim is not None:
        # roofline of the dominant kernel, measured with HIP events on the engine's stream over
        # the timed region; bytes = the algorithmic model.  Two decide kernels share the CD
        # batches of the hybrid engine (the default): the replica-lane k_rl_decide family (full
        # sweeps) and cd.hip's k_decide_light (filtered sweeps); the one with more time is
        # reported, both are listed under "kernels"
        kern = {}
        for key, name in (("decide", "k_decide_light"), ("rl_decide", "k_rl_decide")):
            n_l = tim["%s_launches" % key]
            if n_l:
                a_s = tim["%s_ms" % key] / n_l / 1e3
                b_l = tim["%s_bytes" % key] / n_l
                ach = b_l / a_s / 1e9 if a_s > 0 else 0.0
                kern[name] = {"launches": n_l, "avg_us": a_s * 1e6, "algorithmic_bytes_per_launch": b_l,
                              "achieved": ach, "frac": ach / HBM_PEAK_GBS, "ms_per_step": tim["%s_ms" % key] / args.steps}
        dom = max(kern, key=lambda k: kern[k]["ms_per_step"]) if kern else "k_decide_light"
        kd = kern.get(dom, {"launches": 0, "avg_us": 0.0, "algorithmic_bytes_per_launch": 0.0, "achieved": 0.0})
        avg_s = kd["avg_us"] / 1e6
        # a line run with --n-p n reads the profile taken at that n_p (tools/pmc_bench.sh, FC_PMC_NP)
        traffic, traffic_note = load_traffic(args.config if args.n_p <= 0 else "%s_np%d" % (args.config, args.n_p),
                                             dom)
        roof = {"bound": "hbm", "achieved": kd["achieved"], "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": kd["achieved"] / HBM_PEAK_GBS, "traffic": traffic, "traffic_note": traffic_note,
                "kernel": "%s<%s>" % (dom, "true" if algo != 1 else "false"),
                "note": (None if cfg["algo"] in ("louvain", "lpm") else
                         "the %s CD runs its own kernels (leiden.hip); this roofline covers the Louvain-engine "
                         "decide launches only" % cfg["algo"]),
                "launches": kd["launches"], "avg_us": kd["avg_us"],
                "algorithmic_bytes_per_launch": kd["algorithmic_bytes_per_launch"], "kernels": kern,
                # line traffic (PMC, L2 misses x 128 B) per second of decide time, against the
                # measured ceiling of random 4-B gathers that miss L2 (tools/micro/gather.hip:
                # ~56 G requests/s x 128 B, whether or not the Infinity Cache holds the line)
                "traffic_rate_gbs": (traffic / avg_s / 1e9) if (traffic and avg_s > 0) else None,
                "gather_line_ceiling_gbs": GATHER_LINE_CEILING_GBS}
        if cfg["algo"] in ("leiden", "infomap"):
            # the CD's own dominant kernel (leiden.hip): k_lv_decide or k_lv_heavy, whichever took
            # longer in the timed region; both are reported
            lv = {}
            for k in ("decide", "heavy"):
                n_l = tim["lv_%s_launches" % k]
                if n_l:
                    a_s = tim["lv_%s_ms" % k] / n_l / 1e3
                    b_l = tim["lv_%s_bytes" % k] / n_l
                    ach = b_l / a_s / 1e9 if a_s > 0 else 0.0
                    lv["k_lv_" + k] = {"launches": n_l, "avg_us": a_s * 1e6, "algorithmic_bytes_per_launch": b_l,
                                       "achieved": ach, "frac": ach / HBM_PEAK_GBS,
                                       "ms_per_step": tim["lv_%s_ms" % k] / args.steps}
            if lv:
                dom = max(lv, key=lambda k: lv[k]["ms_per_step"])
                traffic, traffic_note = load_lv_traffic(args.config, dom)
                roof = {"bound": "hbm", "achieved": lv[dom]["achieved"], "peak": HBM_PEAK_GBS, "unit": "GB/s",
                        "frac": lv[dom]["frac"], "traffic": traffic, "traffic_note": traffic_note, "kernel": dom,
                        "note": "the %s CD's dominant kernel by time in the timed region; level 0 of Leiden runs the "
                                "Louvain engine (k_decide_light: %d launches, %.1f ms per step)"
                                % (cfg["algo"], tim["decide_launches"], tim["decide_ms"] / args.steps),
                        "launches": lv[dom]["launches"], "avg_us": lv[dom]["avg_us"],
                        "algorithmic_bytes_per_launch": lv[dom]["algorithmic_bytes_per_launch"], "kernels": lv}
        phases = {k: tim[k] / args.steps for k in ("cd_ms", "consensus_ms", "closure_ms", "rebuild_ms", "decide_ms",
                                                    "rl_decide_ms", "lv_decide_ms", "lv_heavy_ms")}

    if rank == 0:
        cpu = None
        if world == 1 and not args.no_cpu_baseline and not model:
            t = time.perf_counter()
            cpu = cpu_baseline(n, u, v, cfg, args.seed)
            log("[rank 0] cpu baseline %.3g %s in %.1fs" % (cpu["value"], cpu["unit"], time.perf_counter() - t))
        result = {
            "metric": METRIC, "value": value, "unit": "partition·edges/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": 1e3 * elapsed / args.steps,
            "higher_is_better": True, "scaling": "strong", "vs_baseline": None, "dtype": "int32",
            "data": "synthetic (native LFR/SBM generator, graph seed %d; engine seed %d + step index)"
                    % (args.seed, args.seed),
            "config": {"workload": cfg["desc"], "n": n, "m": m0, "algorithm": cfg["algo"], "n_p": cfg["n_p"],
                       "tau": cfg["tau"], "delta": cfg["delta"], "parallelism": "replica-sharded x%d" % world,
                       "iterations": iters, "m_final": m_finals,
                       "step": ("loop only, graph resident before timing (--resident)" if args.resident else
                                "fast_consensus() end to end: host edge arrays -> PCIe upload + device ingest "
                                "-> every iteration + final pass -> n_p labelings in a preallocated host array")},
            "consensus_wall_ms": 1e3 * elapsed / args.steps,
            "load_ms_per_step": 1e3 * load_s / args.steps,
            "per_step": per_step,
            "step_value_median": float(np.median([p["partition_edges"] / p["ms"] * 1e3 for p in per_step])),
            "step_value_min": float(np.min([p["partition_edges"] / p["ms"] * 1e3 for p in per_step])),
            "loop_ms_per_step": 1e3 * loop_s / args.steps,
            "output_array": ("page-locked at allocation" if pinned is not None and pinned.ok else "pageable"),
            "dist": {"backend": backend if world > 1 else None, "world_size": world,
                     "labels_out": (None if world == 1 else
                                    "shared host array, each rank its rows" if shared is not None else
                                    "all-gather, rank 0 downloads")},
            "roofline": roof,
            "cpu_baseline": cpu,
            "phase_ms_per_step_rank0": phases,
        }
        if model:
            result["engine"] = "cpu-model (TEST HOOK: oracle-backed model of the engine, not the product)"
            result["value"] = None
        print(json.dumps(result))
    if pinned is not None:
        pinned.release()
    if shared is not None:
        host_out = None            # noqa: F841 (the last view of the shared array)
        shared.close()


if __name__ == "__main__":
    main()
