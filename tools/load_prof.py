"""Wall time of fc_load_graph (host arrays -> resident graph) per phase (FC_TRACE=1)."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ.setdefault("FC_TRACE", "1")
import fastconsensus_amd as fc  # noqa: E402
from fastconsensus_amd import synth  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000
u, v, _ = synth.lfr(n, 0.5, seed=42)
for store in (1, 0):
    eng = fc.Engine(seed=42)
    eng.set_option("store", store)
    for rep in range(3):
        t = time.perf_counter()
        eng.load_graph(n, u, v)
        print("store=%d load %d: %.1f ms" % (store, rep, 1e3 * (time.perf_counter() - t)), file=sys.stderr, flush=True)
    eng.close()
