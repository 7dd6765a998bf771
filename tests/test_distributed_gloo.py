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


def _worker(rank, world, port, algo, n_p, tau, delta, out_path):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from fastconsensus_amd.distributed import run_sharded
        from tests.cpu_engine import OracleEngine
        N, e = _graph()
        eng = OracleEngine(seed=17, sigma=_sigma(N))
        eng.load_graph(N, e[:, 0], e[:, 1])
        labels, st = run_sharded(eng, algo, n_p, tau, delta, device="cpu", max_iters=50)
        if rank == 0:
            u, v, w, age = eng.get_graph()
            np.savez(out_path, labels=labels, u=u, v=v, w=w, age=age, iters=st["iterations"],
                     pe=st["partition_edges"])
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


# n_p=10 louvain runs 9 consensus iterations on this graph (closure + repair every time)
@pytest.mark.parametrize("world,algo,n_p,tau", [(2, 0, 10, 0.2), (2, 1, 4, 0.8), (3, 0, 12, 0.2), (2, 2, 10, 0.2)])
def test_sharded_equals_single_rank(world, algo, n_p, tau):
    ref_labels, ref_graph, ref_st = _single(algo, n_p, tau, 0.02)
    with tempfile.TemporaryDirectory() as d:
        out = os.path.join(d, "r0.npz")
        mp.spawn(_worker, args=(world, _free_port(), algo, n_p, tau, 0.02, out), nprocs=world, join=True)
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
