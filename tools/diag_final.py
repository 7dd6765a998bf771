#!/usr/bin/env python3
"""Diagnostic (GPU box): one fast_consensus run of bench's lfr1m workload with engine seed S,
then the final graph (node ids, weights), the engine numbering, the final labels of the first
replicas and the run stats into gpurun_out/final_graph_S.npz -- replayed on the CPU twin to
study the final pass's sweep count.
    python tools/diag_final.py [seed] [config]"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
import fastconsensus_amd as fc  # noqa: E402
from fastconsensus_amd.core import ALGORITHMS  # noqa: E402

seed = int(sys.argv[1]) if len(sys.argv) > 1 else 42
config = sys.argv[2] if len(sys.argv) > 2 else "lfr1m"
cfg = bench.CONFIGS[config]
n, u, v, _ = bench.make_graph(cfg, 42)
eng = fc.Engine(device=0, seed=seed)
eng.set_option("seed", seed)
eng.load_graph(n, u, v)
sigma = eng.node_map()
lab, st = eng.run(ALGORITHMS[cfg["algo"]], cfg["n_p"], cfg["tau"], cfg["delta"])
gu, gv, gw, gage = eng.get_graph()
os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
np.savez_compressed(os.path.join(ROOT, "gpurun_out", "final_graph_%d.npz" % seed), u=gu, v=gv, w=gw, sigma=sigma,
                    lab=lab[:4])
print(json.dumps({k: (int(x) if isinstance(x, (int, np.integer)) else x) for k, x in st.items()}))
it = st["iterations"] - (1 if st["exit_check"] == 1 else 0)
eng.set_timing(True)
eng.collect_timing()
eng.cd(ALGORITHMS[cfg["algo"]], 0, cfg["n_p"], cfg["n_p"], 0x40000000 + it)
t = eng.collect_timing()
print("final pass replay: it=%d sweeps/replica %.2f cd_ms %.2f same_labels %s" % (
    it, t["cd_sweeps"] / cfg["n_p"], t["cd_ms"], bool(np.array_equal(eng.get_labels(cfg["n_p"])[:4], lab[:4]))))
