"""Replica-sharded driver over torch.distributed (gloo, CPU, world_size 2 and 3) gives
bit-identical partitions and graphs to one rank (fastconsensus_amd/distributed.py).
The engine here is the oracle-backed CPU model (tests/cpu_engine.py); on the GPU the
same driver runs the HIP engine over RCCL (tests/test_gpu_parity.py checks world=1)."""
import os
import socket
import tempfile

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from tests import golden_io


def _graph():
    case = golden_io.load("lfr1k_louvain_np20")
    return case.N, case.edges_file


def _sigma(N):
    """A fixed internal numbering (the engine draws one per seed; any permutation works)."""
    return np.random.default_rng(5).permutation(N).astype(np.int32)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, algo, n_p, tau, delta, out_path, shard_closure=False, shared_out=False):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from fastconsensus_amd.distributed import SharedOutput, run_sharded
        from tests.cpu_engine import OracleEngine
        N, e = _graph()
        eng = OracleEngine(seed=17, sigma=_sigma(N))
        eng.load_graph(N, e[:, 0], e[:, 1])
        so = None
        if shared_out:      # every rank writes its rows into one shared host array
            so = SharedOutput(n_p, N)
            assert so.array is not None
            so.array[...] = -9
            host = so.array
        else:
            host = np.full((n_p, N), -9, np.int32) if rank == 0 else None   # rank 0 downloads into it
        labels, st = run_sharded(eng, algo, n_p, tau, delta, device="cpu", max_iters=50, out=host,
                                 shard_closure=shard_closure, out_shared=shared_out)
        if rank == 0:
            assert labels is host
            u, v, w, age = eng.get_graph()
            np.savez(out_path, labels=labels, u=u, v=v, w=w, age=age, iters=st["iterations"],
                     pe=st["partition_edges"])
        else:
            assert labels is None
        if so is not None:
            labels = host = None
            so.close()
    finally:
        dist.destroy_process_group()


def _single(algo, n_p, tau, delta):
    from fastconsensus_amd.distributed import run_sharded
    from tests.cpu_engine import OracleEngine
    N, e = _graph()
    eng = OracleEngine(seed=17, sigma=_sigma(N))
    eng.load_graph(N, e[:, 0], e[:, 1])
    labels, st = run_sharded(eng, algo, n_p, tau, delta, device="cpu", max_iters=50)
    return labels, eng.get_graph(), st


# n_p=10 louvain runs 9 consensus iterations on this graph (closure + repair every time);
# shard_closure: each closure block's attempts split over the ranks, lists all-gathered
# shared_out: the final labelings land in one shared-memory host array, each rank its rows
@pytest.mark.parametrize("world,algo,n_p,tau,shard_closure,shared_out",
                         [(2, 0, 10, 0.2, False, False), (2, 1, 4, 0.8, False, False), (3, 0, 12, 0.2, False, False),
                          (2, 2, 10, 0.2, False, False), (2, 3, 6, 0.2, False, False), (3, 4, 5, 0.6, False, False),
                          (2, 0, 10, 0.2, True, False), (3, 0, 12, 0.2, True, False), (3, 1, 4, 0.8, True, False),
                          (3, 0, 10, 0.2, False, True), (2, 1, 4, 0.8, False, True)])
def test_sharded_equals_single_rank(world, algo, n_p, tau, shard_closure, shared_out):
    ref_labels, ref_graph, ref_st = _single(algo, n_p, tau, 0.02)
    with tempfile.TemporaryDirectory() as d:
        out = os.path.join(d, "r0.npz")
        mp.spawn(_worker, args=(world, _free_port(), algo, n_p, tau, 0.02, out, shard_closure, shared_out),
                 nprocs=world, join=True)
        z = np.load(out)
        np.testing.assert_array_equal(z["labels"], ref_labels)
        for a, b in zip((z["u"], z["v"], z["w"], z["age"]), ref_graph):
            np.testing.assert_array_equal(a, b)
        assert int(z["iters"]) == ref_st["iterations"]
        assert int(z["pe"]) == ref_st["partition_edges"]


def test_shard_ranges_cover_contiguously():
    from fastconsensus_amd.distributed import shard
    for n_p in (1, 5, 64, 128):
        for w in (1, 2, 3, 8):
            ranges = [shard(n_p, r, w) for r in range(w)]
            assert ranges[0][0] == 0 and ranges[-1][1] == n_p
            assert all(ranges[i][1] == ranges[i + 1][0] for i in range(w - 1))


def _reduce_worker(rank, world, port, out_path):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from fastconsensus_amd.distributed import _all_reduce_small
        res = {}
        for n_p in (7, 255, 300):
            rng = np.random.default_rng(100 * rank + n_p)
            # k_last in [-1, n_p-1] (MAX); per-rank counts summing to <= n_p (SUM)
            k = torch.from_numpy(rng.integers(-1, n_p, 1000).astype(np.int32))
            c = torch.from_numpy(rng.integers(0, n_p // world + 1, 1000).astype(np.int32))
            res["max%d" % n_p] = _all_reduce_small(k.clone(), dist.ReduceOp.MAX, n_p, world, 1).numpy()
            res["sum%d" % n_p] = _all_reduce_small(c.clone(), dist.ReduceOp.SUM, n_p, world, 0).numpy()
            res["k%d" % n_p], res["c%d" % n_p] = k.numpy(), c.numpy()
        np.savez(out_path + ".%d.npz" % rank, **res)
    finally:
        dist.destroy_process_group()


def test_small_all_reduce_exact():
    """uint8 collectives (n_p <= 255, k_last shifted by +1) and the int32 fallback give the
    exact int32 MAX / SUM."""
    world = 2
    with tempfile.TemporaryDirectory() as d:
        out = os.path.join(d, "red")
        mp.spawn(_reduce_worker, args=(world, _free_port(), out), nprocs=world, join=True)
        z = [np.load(out + ".%d.npz" % r) for r in range(world)]
        for n_p in (7, 255, 300):
            kmax = np.maximum(z[0]["k%d" % n_p], z[1]["k%d" % n_p])
            csum = z[0]["c%d" % n_p] + z[1]["c%d" % n_p]
            for r in range(world):
                np.testing.assert_array_equal(z[r]["max%d" % n_p], kmax)
                np.testing.assert_array_equal(z[r]["sum%d" % n_p], csum)
                assert z[r]["max%d" % n_p].dtype == np.int32
