"""The replica-sharded driver on the device: W ranks, each with a REAL HIP engine, sharing the
box's one MI355X over gloo (fastconsensus_amd/distributed.py; the reference's
per-iteration loop fast_consensus.py:141-202 / :260-310 and final pass :383-392).

Each rank runs `tests/mr_worker.py` as its own process: its contiguous replica shard through
fc_cd / fc_consensus_partial at a non-zero offset, the uint8 MAX / SUM all-reduces on device
tensors (`_all_reduce_small`), the replicated threshold / closure / repair / rebuild, and the
final labelings either into one shared host array (`SharedOutput`, each rank its own rows,
`get_labels_into`) or through the device all-gather to rank 0 (`--gather-out`).  The closure is
replicated or split over the ranks (`shard_closure`).  Required: the labelings, iterations,
partition_edges and final graph bit-identical to ONE rank's native fc_run, and the final graph
identical on every rank.  The workers are child processes (subprocess), never an exec of this
process."""
import os
import socket
import subprocess
import sys
import tempfile

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
WORKER = os.path.join(ROOT, "tests", "mr_worker.py")


@pytest.fixture(scope="module")
def fcmod():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import fastconsensus_amd as fc
    return fc


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _one_rank(fc, algo, n_p, tau, graph, seed, opts):
    from tests.mr_worker import graph as load
    n, u, v = load(graph)
    with fc.Engine(device=0, seed=seed) as eng:
        for k, val in opts.items():
            eng.set_option(k, val)
        eng.load_graph(n, u, v)
        labels, st = eng.run(algo, n_p, tau, 0.02)
        return labels, st, eng.get_graph()


def _ranks(world, algo, n_p, tau, graph, seed, shard_closure, shared_out, opts, d):
    port = _free_port()
    prefix = os.path.join(d, "r")
    env = dict(os.environ, OMP_NUM_THREADS="2")
    procs = []
    for r in range(world):
        cmd = [sys.executable, "-u", WORKER, "--rank", str(r), "--world", str(world), "--port", str(port),
               "--algo", str(algo), "--n-p", str(n_p), "--tau", str(tau), "--graph", graph, "--seed", str(seed),
               "--out", prefix]
        cmd += ["--shard-closure"] if shard_closure else []
        cmd += ["--shared-out"] if shared_out else []
        for k, val in opts.items():
            cmd += ["--opt", "%s=%d" % (k, val)]
        procs.append(subprocess.Popen(cmd, env=env, cwd=ROOT, stdout=subprocess.PIPE, stderr=subprocess.STDOUT))
    outs = []
    try:
        for p in procs:
            outs.append(p.communicate(timeout=240)[0].decode(errors="replace"))
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
                p.wait()
    for r, (p, o) in enumerate(zip(procs, outs)):
        assert p.returncode == 0, "rank %d exited %s:\n%s" % (r, p.returncode, o[-3000:])
    return [np.load(prefix + "_%d.npz" % r) for r in range(world)]


# (world, algo, n_p, tau, graph, shard_closure, shared_out, options)
# C3 louvain / lpm (BASELINE configs[2]; lpm on the sparse LFR-100k where LPA's ties matter);
# the last cases force the hybrid's replica-lane kernels at this size (rl_min_vertices=1), so
# a shard's replica-lane batch starts at replica 32 / 21 / 42, and run 3 ranks (ragged shards)
CASES = [
    (2, 0, 64, 0.2, "c3", False, True, {}),
    (2, 0, 64, 0.2, "c3", True, False, {}),
    (2, 1, 64, 0.8, "c3sparse", False, False, {}),
    (2, 1, 64, 0.8, "c3sparse", True, True, {}),
    (2, 0, 64, 0.2, "c3", False, True, {"rl_min_vertices": 1}),
    (3, 0, 64, 0.2, "c3", True, True, {"rl_min_vertices": 1}),
    (3, 1, 64, 0.8, "c3sparse", False, False, {"rl_min_vertices": 1}),
    (2, 2, 20, 0.2, "lfr1k", False, True, {}),
]


@pytest.mark.timeout(600)
@pytest.mark.parametrize("world,algo,n_p,tau,graph,shard_closure,shared_out,opts", CASES)
def test_sharded_hip_engine_equals_one_rank(fcmod, world, algo, n_p, tau, graph, shard_closure, shared_out, opts):
    seed = 77
    labels, st, g1 = _one_rank(fcmod, algo, n_p, tau, graph, seed, opts)
    with tempfile.TemporaryDirectory() as d:
        z = _ranks(world, algo, n_p, tau, graph, seed, shard_closure, shared_out, opts, d)
        print("world %d algo %d %s: iterations %d exit %d m_final %d (one rank: %d / %d / %d)" % (
            world, algo, graph, int(z[0]["iters"]), int(z[0]["exit"]), int(z[0]["m_final"]), st["iterations"],
            st["exit_check"], st["m_final"]))
        assert int(z[0]["iters"]) == st["iterations"]
        assert int(z[0]["exit"]) == st["exit_check"]
        assert int(z[0]["pe"]) == st["partition_edges"]
        assert int(z[0]["m_final"]) == st["m_final"]
        np.testing.assert_array_equal(z[0]["labels"], labels)
        for r in range(world):                   # replicated state: the same graph on every rank
            for key, exp in zip(("u", "v", "w", "age"), g1):
                np.testing.assert_array_equal(z[r][key], exp, err_msg="rank %d %s" % (r, key))
