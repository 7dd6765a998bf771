#!/usr/bin/env python3
"""One rank of the replica-sharded driver with a REAL HIP engine (test infrastructure).

tests/test_gpu_sharded.py starts `world` of these as child processes on the one MI355X of a
box (gloo: RCCL refuses two ranks on one device), each with its own fc.Engine on cuda:0, and
compares what they produce with one rank's native fc_run.  Every rank writes
<out>_<rank>.npz: its final graph (replicated state: must be identical on every rank) and
its stats; rank 0 adds the labelings it returns.

    python tests/mr_worker.py --rank R --world W --port P --algo A --n-p NP --tau T
                              --graph c3|c3sparse|lfr1k --seed S [--shard-closure] [--shared-out]
                              [--opt name=value ...] --out PREFIX
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402


def graph(name):
    """(n, u, v) of the named test graph (the same bytes in every process)."""
    if name == "lfr1k":
        from tests import golden_io
        case = golden_io.load("lfr1k_louvain_np20")
        return case.N, case.edges_file[:, 0].copy(), case.edges_file[:, 1].copy()
    from fastconsensus_amd import synth
    kw = {"avg_deg": 8, "max_deg": 25} if name == "c3sparse" else {}
    u, v, _ = synth.lfr(100_000, 0.5, seed=42, **kw)
    return 100_000, u, v


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rank", type=int, required=True)
    ap.add_argument("--world", type=int, required=True)
    ap.add_argument("--port", type=int, required=True)
    ap.add_argument("--algo", type=int, required=True)
    ap.add_argument("--n-p", type=int, required=True)
    ap.add_argument("--tau", type=float, required=True)
    ap.add_argument("--graph", required=True)
    ap.add_argument("--seed", type=int, required=True)
    ap.add_argument("--shard-closure", action="store_true")
    ap.add_argument("--shared-out", action="store_true")
    ap.add_argument("--opt", action="append", default=[])
    ap.add_argument("--out", required=True)
    a = ap.parse_args()
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(a.port)
    import torch
    import torch.distributed as dist
    dist.init_process_group("gloo", rank=a.rank, world_size=a.world)
    try:
        import fastconsensus_amd as fc
        from fastconsensus_amd.distributed import SharedOutput, run_sharded
        n, u, v = graph(a.graph)
        with fc.Engine(device=0, seed=a.seed) as eng:
            for kv in a.opt:
                k, val = kv.split("=")
                eng.set_option(k, int(val))
            eng.load_graph(n, u, v)
            so = None
            if a.shared_out:
                so = SharedOutput(a.n_p, n)
                assert so.array is not None, "shared output unavailable"
                so.array[...] = -9
                host = so.array
            else:
                host = np.full((a.n_p, n), -9, np.int32) if a.rank == 0 else None
            labels, st = run_sharded(eng, a.algo, a.n_p, a.tau, 0.02, device="cuda", max_iters=1000, out=host,
                                     shard_closure=a.shard_closure, out_shared=a.shared_out)
            torch.cuda.synchronize()
            gu, gv, gw, gage = eng.get_graph()
            rec = dict(u=gu, v=gv, w=gw, age=gage, iters=st["iterations"], pe=st["partition_edges"],
                       exit=st["exit_check"], m_final=st["m_final"])
            if a.rank == 0:
                assert labels is host
                rec["labels"] = np.array(labels)
            else:
                assert labels is None
            np.savez(a.out + "_%d.npz" % a.rank, **rec)
            labels = host = None
            if so is not None:
                so.close()
    finally:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
