#!/usr/bin/env python3
"""A/B of Leiden / Infomap kernel variants (GPU box): per variant library, whole fc_run calls on
one graph, best-of-reps wall time and a hash of the labelings (variants claiming identical
decisions must print the same hash).

    python tools/lv_ab.py [--config lfr1m_leiden] [--reps 2] base name1[@ENV=VAL,...] ...
"""
import hashlib
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def child(lib, config, reps):
    os.environ["FC_LIB_PATH"] = lib
    sys.path.insert(0, ROOT)
    import numpy as np

    import bench
    import fastconsensus_amd as fc
    from fastconsensus_amd import core
    cfg = dict(bench.CONFIGS[config])
    n, u, v, planted = bench.make_graph(cfg, 42)
    algo = core.algo_id(cfg["algo"])
    host = np.zeros((cfg["n_p"], n), np.int32)
    out = {"lib": lib, "config": config}
    with fc.Engine(seed=42) as eng:
        # FC_AB_OPTS="name=value;...": engine options of this variant (fc_set_option)
        for kv in filter(None, os.environ.get("FC_AB_OPTS", "").split(";")):
            k, _, val = kv.partition("=")
            eng.set_option(k, int(val))
        eng.load_graph(n, u, v)
        eng.run(algo, cfg["n_p"], cfg["tau"], cfg["delta"], out=host)      # warm
        runs = []
        for _ in range(reps):
            eng.load_graph(n, u, v)
            t0 = time.perf_counter()
            _, st = eng.run(algo, cfg["n_p"], cfg["tau"], cfg["delta"], out=host)
            runs.append(1e3 * (time.perf_counter() - t0))
        out["run_ms"] = min(runs)
        out["runs_ms"] = [round(x, 1) for x in runs]
        out["labels_sha"] = hashlib.sha1(host.tobytes()).hexdigest()[:16]
        # quality of one CD batch on the input graph (variants that change the random streams
        # are compared by it): mean NMI to the planted communities, and for infomap the mean
        # two-level codelength
        from tests import dist_gates
        eng.reset_graph()
        eng.cd(algo, 0, 8, 8, 0)
        lab = eng.get_labels(8)
        out["cd_nmi"] = round(float(np.mean([dist_gates.nmi(planted, x) for x in lab])), 5)
        if cfg["algo"] == "infomap":
            from tests.test_infomap import codelength
            e = np.stack([u, v], 1).astype(np.int64)
            out["cd_codelength"] = round(float(np.mean([codelength(n, e, x) for x in lab])), 5)
        out["final_nmi"] = round(float(np.mean([dist_gates.nmi(planted, x) for x in host[:8]])), 5)
    print(json.dumps(out), flush=True)


def main():
    args = sys.argv[1:]
    if args and args[0] == "--child":
        child(args[1], args[2], int(args[3]))
        return
    config, reps = "lfr1m_leiden", 2
    while args and args[0].startswith("--"):
        k, val = args[0], args[1]
        args = args[2:]
        if k == "--config":
            config = val
        elif k == "--reps":
            reps = int(val)
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
        rc = subprocess.call([sys.executable, __file__, "--child", lib, config, str(reps)], env=env)
        if rc != 0:
            print("variant %s failed rc=%d" % (name, rc), flush=True)
            sys.exit(rc)


if __name__ == "__main__":
    main()
