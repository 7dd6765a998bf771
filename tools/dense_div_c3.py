"""A/B helper (GPU box): the C3 louvain consensus NMI distribution over 40 seeds with FC_OPT_DENSE_DIV = argv[1],
against the reference loop (refsem_lfr100k_louvain_np64.json) through tests/dist_gates.py."""
import sys, os, time, json
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import fastconsensus_amd as fc
from fastconsensus_amd import synth
from tests import dist_gates, golden_io
dd = int(sys.argv[1])
u, v, planted = synth.lfr(100_000, 0.5, seed=42)
with open(golden_io.GOLDEN + "/refsem_lfr100k_louvain_np64.json") as f:
    ref = json.load(f)
got = []
t = time.time()
for seed in range(300, 340):
    with fc.Engine(seed=seed) as eng:
        eng.set_option("dense_div", dd)
        eng.load_graph(100_000, u, v)
        labels, st = eng.run(0, 64, 0.2, 0.02)
    got.append(float(np.mean([dist_gates.nmi(planted, l) for l in labels])))
got = np.array(got)
print("dense_div", dd, "time %.1f s" % (time.time() - t), flush=True)
try:
    dist_gates.check(got, ref["nmi"], 0.0005, "C3 louvain dd%d" % dd, ks=True, p10_slack=0.0005)
    print("GATES PASS")
except AssertionError as ex:
    print("GATES FAIL", ex)
