"""The C-ABI library loads and exports every symbol include/*.h declares (no GPU needed),
and the product path fails loudly without a GPU (no CPU fallback)."""
import ctypes
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_symbols():
    names = set()
    for fn in os.listdir(os.path.join(ROOT, "include")):
        if fn.endswith(".h"):
            src = open(os.path.join(ROOT, "include", fn)).read()
            src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
            names |= set(re.findall(r"\b(fc_[a-z_]+)\s*\(", src))
    return names


def test_header_declares_expected_surface():
    names = declared_symbols()
    for must in ("fc_create", "fc_run", "fc_consensus_partial", "fc_consensus_apply", "fc_closure_apply",
                 "fc_last_error"):
        assert must in names


def test_library_exports_every_declared_symbol():
    from fastconsensus_amd import _lib
    from fastconsensus_amd.build import build
    build(verbose=False)
    L = ctypes.CDLL(_lib.LIB_PATH)
    missing = [n for n in sorted(declared_symbols()) if not hasattr(L, n)]
    assert not missing, missing
    assert set(_lib.SYMBOLS) == declared_symbols()
    _lib.load()
    assert b"gfx950" in _lib.load().fc_version()


def test_no_gpu_fails_loudly():
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    import fastconsensus_amd as fc
    with pytest.raises(fc.FastConsensusError) as ei:
        fc.Engine(seed=1)
    assert ei.value.code == -2


def test_product_package_never_imports_oracle():
    pkg = os.path.join(ROOT, "fastconsensus_amd")
    for dirpath, _, files in os.walk(pkg):
        for fn in files:
            if fn.endswith((".py", ".cpp", ".hip", ".h")):
                src = open(os.path.join(dirpath, fn)).read()
                for pat in (r"^\s*(from|import)\s+oracle", r"fcoracle", r"\borc_[a-z]", r"oracle\.oracle"):
                    assert not re.search(pat, src, flags=re.M), (fn, pat)


def test_cpu_twin_defaults_match_engine_defaults():
    """orc.engine_cd / OracleEngine defaults are the engine's (fc_ctx.h), so a bare call of the
    twin is the bit-exact target of a bare Engine.cd."""
    import inspect
    from oracle import oracle as orc
    from tests.cpu_engine import OracleEngine
    src = open(os.path.join(ROOT, "fastconsensus_amd", "csrc", "fc_ctx.h")).read()
    eng = {k: int(re.search(r"\b%s = (\d+)" % k, src).group(1)) for k in ("max_sweeps", "chunk", "prune", "coarsen", "prune_mark", "dense_div")}
    # buckets: 0 in the context = cd_buckets' per-algorithm default (Louvain 16, LPA 32), which the
    # twin restates (orc.cd_buckets; engine_cd / OracleEngine default None)
    assert int(re.search(r"\bbuckets = (\d+)", src).group(1)) == 0
    bl, bp = (int(x) for x in re.search(r"CD_BUCKETS_LOUVAIN = (\d+), CD_BUCKETS_LPA = (\d+)", src).groups())
    assert (orc.BUCKETS_LOUVAIN, orc.BUCKETS_LPA) == (bl, bp)
    assert orc.cd_buckets(orc.LOUVAIN) == bl and orc.cd_buckets(orc.LOUVAIN_NC) == bl and orc.cd_buckets(orc.LPM) == bp
    assert inspect.signature(orc.engine_cd).parameters["buckets"].default is None
    assert inspect.signature(OracleEngine.__init__).parameters["buckets"].default is None
    # the default CD engine is the hybrid (FC_OPT_CD_ENGINE=2): the twin's shared=2
    assert int(re.search(r"\bcd_engine = (\d+)", src).group(1)) == 2
    eng["shared"] = 2
    twin = inspect.signature(orc.engine_cd).parameters
    model = inspect.signature(OracleEngine.__init__).parameters
    for k, v in eng.items():
        assert twin[k].default == v, k
        if k in model:
            assert model[k].default == v, k
    assert int(re.search(r"\bclosure_rounds = (\d+)", src).group(1)) == 0      # 0: per algorithm
    m = re.search(r"CLOSURE_ROUNDS_LOUVAIN = (\d+), CLOSURE_ROUNDS_LPM = (\d+)", src)
    assert (orc.CLOSURE_ROUNDS_LOUVAIN, orc.CLOSURE_ROUNDS_LPM) == (int(m.group(1)), int(m.group(2)))
    assert [orc.closure_rounds(a) for a in (0, 1, 2, 4)] == [int(m.group(1)), int(m.group(2)), int(m.group(1)),
                                                            int(m.group(2))]
    assert inspect.signature(orc.closure_sample_pairs).parameters["rounds"].default == orc.CLOSURE_ROUNDS_LOUVAIN
