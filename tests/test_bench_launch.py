"""bench.py's launcher contract on CPU (no GPU): `--gpus N` starts N ranks under
torch.distributed.run itself, `n_gpus` is the world size the process group reports, the
sharded run is bit-identical to one rank, and a --gpus / WORLD_SIZE mismatch exits non-zero
instead of printing a mislabelled line.  The engine is bench.py's --engine-model test hook
(the oracle-backed CPU model, tests/cpu_engine.py): this checks the launcher, not speed."""
import json
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(ROOT, "bench.py")


def _run(args, env_extra=None):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env.update(env_extra or {})
    p = subprocess.run([sys.executable, BENCH, "--engine-model", "--config", "lfr1k", "--steps", "1",
                        "--warmup", "0"] + args, capture_output=True, text=True, env=env, cwd=ROOT, timeout=600)
    return p


def _line(p):
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [x for x in p.stdout.splitlines() if x.startswith("{")]
    assert len(lines) == 1, p.stdout
    return json.loads(lines[0])


def test_gpus2_launches_two_ranks_bit_identical():
    one = _line(_run(["--gpus", "1"]))
    two = _line(_run(["--gpus", "2"]))
    assert one["n_gpus"] == 1 and two["n_gpus"] == 2
    assert two["dist"] == {"backend": "gloo", "world_size": 2, "labels_out": "shared host array, each rank its rows"}
    assert two["config"]["iterations"] == one["config"]["iterations"]
    assert two["config"]["m_final"] == one["config"]["m_final"]
    gat = _line(_run(["--gpus", "2", "--gather-out"]))
    assert gat["dist"]["labels_out"] == "all-gather, rank 0 downloads"
    assert gat["config"]["m_final"] == one["config"]["m_final"]
    assert two["config"]["parallelism"] == "replica-sharded x2"
    # the test hook never claims a throughput
    assert one["value"] is None and "TEST HOOK" in one["engine"]


def test_gpus_world_size_mismatch_exits_nonzero():
    p = _run(["--gpus", "1"], {"WORLD_SIZE": "2", "RANK": "0", "LOCAL_RANK": "0"})
    assert p.returncode == 2
    assert not [x for x in p.stdout.splitlines() if x.startswith("{")]
    assert "mislabelled" in p.stderr


def test_cpu_baseline_full_iteration_small():
    """The CPU baseline times one FULL consensus iteration (CD + consensus + threshold +
    closure + repair) of the reference-semantics port and reports cores and CPU model."""
    sys.path.insert(0, ROOT)
    import bench
    from fastconsensus_amd import synth
    cfg = dict(bench.CONFIGS["lfr1k"])
    u, v, _ = synth.lfr(cfg["n"], cfg["mu"], seed=3)
    cpu = bench.cpu_baseline(cfg["n"], u, v, cfg, seed=3)
    assert cpu["kind"] == "port" and cpu["cores"] == bench.host_cpu_share() >= 1
    assert cpu["value"] > 0 and cpu["iteration_s"] > 0 and cpu["cpu_model"]
    for part in ("consensus", "closure over", "repair+swap", "ONE full consensus iteration"):
        assert part in cpu["sample"]
    assert np.isfinite(cpu["value"])
