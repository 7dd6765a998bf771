#!/usr/bin/env python3
"""A/B of CD-kernel variants on one graph (GPU box).  Each variant is a library path (variant
builds from tools/build_variant.sh; `base` = the in-tree library) run in its own process:

    python tools/cd_ab.py [--config lfr1m] [--algo 0] [--reps 3] [--np N] base name1 name2 ...

Per variant: one CD batch of n_p replicas on the input graph (fc_cd, iteration 0) timed with
the engine's HIP events (cd_ms, decide_ms, launches), a whole fc_run, and a hash of the
labelings -- variants that claim identical semantics must print the same hash.
"""
import hashlib
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def child(lib, config, algo, reps, np_over=0):
    os.environ["FC_LIB_PATH"] = lib
    sys.path.insert(0, ROOT)
    import time

    import numpy as np

    import bench
    import fastconsensus_amd as fc
    cfg = dict(bench.CONFIGS[config])
    n, u, v, _ = bench.make_graph(cfg, 42)
    if np_over:
        cfg["n_p"] = np_over
    n_p = cfg["n_p"]
    out = {"lib": lib}
    with fc.Engine(seed=42) as eng:
        # FC_AB_OPTS="name=value;...": engine options of this variant (fc_set_option)
        for kv in filter(None, os.environ.get("FC_AB_OPTS", "").split(";")):
            k, _, val = kv.partition("=")
            eng.set_option(k, int(val))
        loads = []
        for _ in range(3):
            t0 = time.perf_counter()
            eng.load_graph(n, u, v)
            loads.append(1e3 * (time.perf_counter() - t0))
        out["load_ms"] = min(loads)
        eng.cd(algo, 0, n_p, n_p, 0)          # warm (buffers)
        eng.set_timing(True)
        eng.collect_timing()
        cds = []
        for _ in range(reps):
            eng.cd(algo, 0, n_p, n_p, 0)
            t = eng.collect_timing()
            cds.append(t)
        lab = eng.get_labels(n_p)
        out["labels_sha"] = hashlib.sha1(lab.tobytes()).hexdigest()[:16]
        if os.environ.get("FC_AB_CDONLY") == "1":     # PMC passes: the CD batches only
            print(json.dumps(out), flush=True)
            return
        out["cd_ms"] = min(t["cd_ms"] for t in cds)
        out["decide_ms"] = min(t["decide_ms"] for t in cds)
        out["decide_launches"] = cds[0]["decide_launches"]
        out["decide_us_avg"] = 1e3 * out["decide_ms"] / max(1, out["decide_launches"])
        out["rl_decide_ms"] = min(t["rl_decide_ms"] for t in cds)
        out["visits"] = cds[0]["cd_vertex_visits"]
        out["sweeps"] = cds[0]["cd_sweeps"]
        host = np.zeros((n_p, n), np.int32)
        runs = []
        for _ in range(reps):
            t0 = time.perf_counter()
            _, st = eng.run(algo, n_p, cfg["tau"], cfg["delta"], out=host)
            runs.append(1e3 * (time.perf_counter() - t0))
            out["iterations"] = st["iterations"]
        out["run_ms"] = min(runs)
        out["run_sha"] = hashlib.sha1(host.tobytes()).hexdigest()[:16]
        # one CD batch on the run's final (weighted consensus) graph
        eng.collect_timing()
        cds = []
        for _ in range(reps):
            eng.cd(algo, 0, n_p, n_p, 7)
            cds.append(eng.collect_timing())
        out["w_cd_ms"] = min(t["cd_ms"] for t in cds)
        out["w_decide_ms"] = min(t["decide_ms"] for t in cds)
        out["w_rl_decide_ms"] = min(t["rl_decide_ms"] for t in cds)
        out["w_labels_sha"] = hashlib.sha1(eng.get_labels(n_p).tobytes()).hexdigest()[:16]
    print(json.dumps(out), flush=True)


def main():
    args = sys.argv[1:]
    if args and args[0] == "--child":
        child(args[1], args[2], int(args[3]), int(args[4]), int(args[5]))
        return
    config, algo, reps, np_over = "lfr1m", 0, 3, 0
    while args and args[0].startswith("--"):
        k, val = args[0], args[1]
        args = args[2:]
        if k == "--config":
            config = val
        elif k == "--algo":
            algo = int(val)
        elif k == "--reps":
            reps = int(val)
        elif k == "--np":
            np_over = int(val)
    for spec in args or ["base"]:
        # name[@ENV=VAL,ENV=VAL]: a variant library and engine environment switches
        name, _, envs = spec.partition("@")
        env = dict(os.environ)
        for kv in filter(None, envs.split(",")):
            k, _, v = kv.partition("=")
            env[k] = v
        lib = os.path.join(ROOT, "fastconsensus_amd", "lib",
                           "libfastconsensus_amd.so" if name == "base" else name + "/libfastconsensus_amd.so")
        print("variant", spec, flush=True)
        rc = subprocess.call([sys.executable, __file__, "--child", lib, config, str(algo), str(reps), str(np_over)], env=env)
        if rc != 0:
            print("variant %s failed rc=%d" % (name, rc), flush=True)
            sys.exit(rc)


if __name__ == "__main__":
    main()
