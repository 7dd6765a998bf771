"""Replica-sharded fast_consensus over several GPUs (one process per GPU, RCCL over xGMI).

The n_p community-detection runs of every iteration are independent given the graph, so
rank g owns the CONTIGUOUS replica range [g*n_p/W, (g+1)*n_p/W) (the Louvain consensus
rule depends on replica order, fast_consensus.py:154-159).  Every rank keeps an identical
copy of the graph; the only data-path exchanges are
  * per-edge partials: Louvain k_last (all-reduce MAX) / LPM co-membership counts (SUM);
  * per-candidate closure co-membership counts (SUM, louvain only);
both travel as uint8 when n_p <= 255 (k_last + 1 and counts are in [0, n_p]): a quarter
of the int32 bytes on every xGMI ring hop;
after which threshold, check, repair and the graph rebuild run replicated and
deterministically -- no graph broadcast.  The triadic closure runs replicated too (same
counter-based RNG on every rank) unless shard_closure=True: then each closure block's
attempts are divided over the ranks and their (pair, first attempt) lists all-gathered
(_closure_sharded, same candidates).  Measured on LFR-1M it does not pay: half the
attempts yield a candidate, and the per-candidate work (dedup, append, growing the closure
graph) stays on every rank -- 4.7 ms per rank at W = 8 against 6.0 ms replicated, before
the ~116 MB all-gathered per iteration (profiles/r03_closure_shard_time.json).  The final
partitions are all-gathered to rank 0.  The loop mirrors fc_run (capi.cpp) step for step,
so W ranks produce bit-identical results to one GPU.

The driver only needs an "engine" with the step API of fastconsensus_amd.Engine; buffers
are torch tensors on the engine's device (RCCL) or on the CPU (gloo, used by the tests).
"""
import os

import numpy as np
import torch
import torch.distributed as dist

from .core import FINAL_PASS_ITER

LOUVAIN, LPM, LOUVAIN_NC, LEIDEN, INFOMAP = 0, 1, 2, 3, 4


def on_device(t):
    return t.device.type == "cuda"


def shard(n_p, rank, world):
    return n_p * rank // world, n_p * (rank + 1) // world


def _all_reduce_small(t, op, n_p, world, shift):
    """In-place all-reduce of int32 values in [-shift, n_p - shift] (MAX, or SUM of per-rank
    counts whose total is <= n_p); as uint8 when n_p <= 255.  Exact: MAX commutes with the
    +shift, and every partial SUM is a count of replicas, <= n_p."""
    if world <= 1:
        return t
    if n_p > 255:
        dist.all_reduce(t, op=op)
        return t
    b = (t + shift).to(torch.uint8)
    dist.all_reduce(b, op=op)
    t.copy_(b)
    if shift:
        t.sub_(shift)
    return t


def _closure_sharded(engine, attempts, iteration, world, rank, device):
    """fast_consensus.py:175-184 / :292-300 (the growing nextgraph) over W ranks: block b's
    attempts [t0, t1) are split into W contiguous sub-ranges, each rank draws its own, and
    the ranks' pair lists (int64 key, first attempt) are all-gathered -- a count exchange,
    then the lists padded to the largest -- and added on every rank before block b + 1 draws
    from the grown graph.  Same candidates as engine.closure_sample on one rank."""
    blocks = engine.closure_begin(attempts, iteration)
    for b in range(blocks):
        t0, t1 = attempts * b // blocks, attempts * (b + 1) // blocks
        lo, hi = t0 + (t1 - t0) * rank // world, t0 + (t1 - t0) * (rank + 1) // world
        cap_pairs = (t1 - t0 + world - 1) // world + 1          # >= every rank's sub-range
        mine = torch.empty(2 * cap_pairs, dtype=torch.int64, device=device)
        k = engine.closure_block_sample(b, lo, hi, mine)
        cnt = torch.tensor([k], dtype=torch.int64, device=device)
        cnts = [torch.empty_like(cnt) for _ in range(world)]
        dist.all_gather(cnts, cnt)
        cnts = [int(x) for x in torch.cat(cnts).tolist()]
        top = max(cnts)
        if top == 0:
            engine.closure_block_add(b, None, 0)
            continue
        recv = [torch.empty(2 * top, dtype=torch.int64, device=device) for _ in range(world)]
        dist.all_gather(recv, mine[:2 * top])
        pairs = torch.cat([recv[g][:2 * cnts[g]] for g in range(world)])
        engine.closure_block_add(b, pairs, sum(cnts))
    return engine.closure_finish()


class SharedOutput:
    """The run's [n_p][n] int32 host labelings in POSIX shared memory, mapped by every rank of
    the node (collective: all ranks construct it).  Passed as run_sharded(out=..., out_shared=
    True), each rank downloads ITS replica rows over its own PCIe link straight into the
    array -- no device all-gather of n_p*n labels and no 256 MB download through rank 0.
    `array` is None on every rank (callers fall back to the gather) when /dev/shm cannot hold
    it -- tmpfs does not reserve pages, and a write past its limit would be a SIGBUS -- or when
    the ranks are not all on one node (a rank elsewhere could not map it)."""

    def __init__(self, n_p, n):
        from multiprocessing import resource_tracker, shared_memory
        self.rank = dist.get_rank() if dist.is_initialized() else 0
        self.shm, self.array = None, None
        size = max(4 * int(n_p) * int(n), 4)
        name = None
        one_node = True
        if dist.is_initialized() and dist.get_world_size() > 1:
            import socket
            hosts = [None] * dist.get_world_size()
            dist.all_gather_object(hosts, socket.gethostname())
            one_node = len(set(hosts)) == 1
        if self.rank == 0 and one_node:
            try:
                st = os.statvfs("/dev/shm")
                if st.f_bavail * st.f_frsize >= size + size // 8 + (64 << 20):
                    self.shm = shared_memory.SharedMemory(create=True, size=size)
                    name = self.shm.name
            except OSError:
                name = None
        obj = [name]
        if dist.is_initialized():
            dist.broadcast_object_list(obj, src=0)
        name = obj[0]
        if name is None:
            return
        if self.rank != 0:
            self.shm = shared_memory.SharedMemory(name=name)
            resource_tracker.unregister(self.shm._name, "shared_memory")   # rank 0 owns (unlinks) it
        self.array = np.ndarray((n_p, n), np.int32, buffer=self.shm.buf)

    def close(self):
        """Collective.  Drop every view of `array` first."""
        if dist.is_initialized():
            dist.barrier()
        self.array = None
        if self.shm is not None:
            self.shm.close()
            if self.rank == 0:
                self.shm.unlink()
            self.shm = None


def run_sharded(engine, algo, n_p, tau, delta, device="cuda", max_iters=1000, gather=True, out=None,
                shard_closure=False, out_shared=False):
    """Returns (labels [n_p][N] on rank 0 (None elsewhere), stats dict).  `out`: optional
    C-contiguous int32 host array [n_p][N] that rank 0 downloads into (see Engine.run).
    shard_closure: split the closure's attempts over the ranks (world > 1; same result);
    default False: every rank draws all of them (see the module docstring).
    out_shared: `out` is the same host array on every rank (SharedOutput.array): each rank
    writes its own rows, rank 0 returns it once all have."""
    world = dist.get_world_size() if dist.is_initialized() else 1
    rank = dist.get_rank() if dist.is_initialized() else 0
    if out_shared and world > 1 and out is None:
        # every rank must pass the shared array: a rank without it would take the all-gather
        # path while the others wait in the shared path's barrier
        raise ValueError("run_sharded(out_shared=True) needs the SharedOutput array on every rank")
    r0, r1 = shard(n_p, rank, world)
    louv = algo in (LOUVAIN, LOUVAIN_NC)    # louvain loop: check #1, closure counts, repair
    on_gpu = str(device).startswith("cuda")
    if not on_gpu:
        return _loop(engine, algo, n_p, tau, delta, device, max_iters, gather, world, rank, r0, r1, louv, out,
                     shard_closure, out_shared)
    # engine kernels and torch/RCCL ops on ONE explicit stream: no cross-stream races
    # (torch's default stream is the legacy null stream, which the engine cannot adopt)
    stream = torch.cuda.Stream(device=device)
    stream.wait_stream(torch.cuda.current_stream(device))
    engine.set_stream(stream.cuda_stream)
    try:
        with torch.cuda.stream(stream):
            return _loop(engine, algo, n_p, tau, delta, device, max_iters, gather, world, rank, r0, r1, louv, out,
                         shard_closure, out_shared)
    finally:
        stream.synchronize()
        engine.set_stream(None)


def _loop(engine, algo, n_p, tau, delta, device, max_iters, gather, world, rank, r0, r1, louv, out=None,
          shard_closure=False, out_shared=False):
    mine = r1 - r0
    engine.reset_graph()
    n, _, L = engine.graph_info()
    st = {"iterations": 0, "exit_check": 0, "hit_iter_cap": 0, "partition_edges": 0, "n_p": n_p}
    it = 0
    if algo == LEIDEN:
        # fast_consensus.py:204-258 on integer node ids: the str-keyed lookups (:97, :217) never
        # match, every weight stays 0 and check #1 (:229) converges on the emptied graph; the
        # loop's CD batch cannot reach the result (capi.cpp fc_run does the same)
        st["exit_check"] = 1
    while algo != LEIDEN:
        if it >= max_iters:
            st["hit_iter_cap"] = 1
            break
        m = engine.m
        part = torch.empty(max(m, 1), dtype=torch.int32, device=device)
        if mine > 0:
            engine.cd(algo, r0, mine, n_p, it)                       # :148 / :270
            engine.consensus_partial(algo, part)                     # :150-159 / :273-280
        else:
            part.fill_(-1 if algo == LOUVAIN else 0)
        # louvain: k_last in [-1, n_p-1] (MAX); lpm / new_consensus rule: counts in [0, n_p] (SUM)
        if algo == LOUVAIN:
            _all_reduce_small(part, dist.ReduceOp.MAX, n_p, world, 1)
        else:
            _all_reduce_small(part, dist.ReduceOp.SUM, n_p, world, 0)
        st["partition_edges"] += n_p * m
        conv1, kept, unc = engine.consensus_apply(algo, n_p, tau, delta, part)   # :163-173
        if louv and conv1:
            st["exit_check"] = 1
            break
        if world > 1 and shard_closure:                              # :175-184 / :292-300
            nc = _closure_sharded(engine, L, it, world, rank, device)
        else:
            nc = engine.closure_sample(L, it)
        cnt = None
        if louv and nc > 0:
            cnt = torch.zeros(nc, dtype=torch.int32, device=device)
            if mine > 0:
                engine.closure_partial(cnt)                          # :186-190
            _all_reduce_small(cnt, dist.ReduceOp.SUM, n_p, world, 0)
        conv2, _ = engine.closure_apply(algo, n_p, delta, cnt, it)   # :193-202 / :307-310
        it += 1
        if conv2:
            st["exit_check"] = 2
            break
    st["iterations"] = it + (1 if st["exit_check"] == 1 else 0)
    m = engine.m
    st["partition_edges"] += n_p * m
    st["m_final"] = m
    if mine > 0:
        engine.cd(algo, r0, mine, n_p, FINAL_PASS_ITER + it)         # final pass :383-392
    if gather and world > 1 and out_shared and out is not None:
        # every rank downloads its rows into the shared host array; the barrier orders the
        # writes before rank 0 hands the array back
        if mine > 0:
            engine.get_labels_into(out[r0:r1], renumber=True)
        dist.barrier()
        return (out if rank == 0 else None), st
    if not gather or world == 1:
        if mine > 0 and out is not None and world == 1:
            engine.get_labels_into(out, renumber=True)
            return out, st
        return (engine.get_labels(mine, renumber=True) if mine > 0 else None), st
    # final partitions: exported straight into the gather buffer (no host round trip), one
    # all-gather, one download on rank 0
    cap = max(shard(n_p, g, world)[1] - shard(n_p, g, world)[0] for g in range(world))
    buf = torch.full((cap, n), -1, dtype=torch.int32, device=device)
    if mine > 0:
        if on_device(buf):
            engine.get_labels(mine, renumber=True, dev_out=buf)
        else:
            buf[:mine].copy_(torch.from_numpy(engine.get_labels(mine, renumber=True)))
    bufs = [torch.empty_like(buf) for _ in range(world)]
    dist.all_gather(bufs, buf)
    if rank != 0:
        return None, st
    if out is None:
        out = np.empty((n_p, n), np.int32)
    host = torch.from_numpy(out)   # device -> the host array directly (no staging tensors)
    for g in range(world):
        a, b = shard(n_p, g, world)
        if b > a:
            host[a:b].copy_(bufs[g][:b - a])
    return out, st
