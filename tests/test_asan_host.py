"""ASan/UBSan host builds (SURVEY.md §5 auxiliaries): the C-ABI's host code (capi.cpp,
gen.cpp; tests/asan/build.sh) driven through every argument check, error path, the native
edge-list parser and the generators; and the C oracle (fc_oracle.c, gcc -fsanitize=address)
replaying a golden run.  CPU only: no device code runs."""
import os
import shutil
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _asan_clean(p):
    out = p.stdout + p.stderr
    assert "AddressSanitizer" not in out and "runtime error:" not in out, out[-4000:]


@pytest.mark.skipif(not os.path.exists("/opt/rocm/bin/hipcc"), reason="hipcc absent")
@pytest.mark.skipif(not os.path.exists(os.path.join(ROOT, "tests", "asan", "build.sh")),
                    reason="tests/asan/ not shipped (it is CPU-only and listed in .gpurunignore)")
def test_capi_host_code_under_asan(tmp_path):
    from fastconsensus_amd.build import build
    build(verbose=False)                                   # the regular device objects
    subprocess.run(["bash", os.path.join(ROOT, "tests", "asan", "build.sh")], check=True, capture_output=True)
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:halt_on_error=1", UBSAN_OPTIONS="halt_on_error=1")
    p = subprocess.run([os.path.join(ROOT, "tests", "asan", "_build", "asan_driver"),
                        os.path.join(ROOT, "tests", "golden"), str(tmp_path)], capture_output=True, text=True,
                       env=env, timeout=300)
    _asan_clean(p)
    assert p.returncode == 0 and "ASAN DRIVER: clean" in p.stdout, p.stdout + p.stderr


@pytest.mark.skipif(shutil.which("gcc") is None, reason="gcc absent")
def test_oracle_under_asan(tmp_path):
    lib = str(tmp_path / "libfcoracle_asan.so")
    subprocess.run(["gcc", "-O1", "-g", "-shared", "-fPIC", "-fopenmp", "-fsanitize=address,undefined",
                    "-fno-omit-frame-pointer", "-o", lib, os.path.join(ROOT, "oracle", "fc_oracle.c"), "-lm"],
                   check=True)
    libasan = subprocess.run(["gcc", "-print-file-name=libasan.so"], capture_output=True, text=True).stdout.strip()
    code = ("import sys; sys.path.insert(0, %r)\n"
            "from oracle import oracle as orc\n"
            "orc.LIB_PATH = %r; orc.build = lambda: None\n"
            "from tests import golden_io\n"
            "import numpy as np\n"
            "for name in ('karate_louvain_np50', 'lfr1k_lpm_np20'):\n"
            "    c = golden_io.load(name)\n"
            "    g, tr, fin = orc.replay(c.algo, c.N, c.edges_file, c.n_p, c.tau, c.delta, c.cd_batches, c.pair_batches)\n"
            "    kept = tr[0]['kept']\n"
            "    pairs = orc.closure_sample_pairs(kept, g[0].m, 3, 0)\n"
            "    lab, sw = orc.engine_cd(c.algo, g[0], 3, 0, 0, 5)\n"
            "    lab2, _ = orc.cd_batch(c.algo, 2, g[0], seed=5, nthreads=2)\n"
            "print('oracle under asan ok')\n" % (ROOT, lib))
    # libasan must come first; whatever the environment already preloads stays after it
    pre = ":".join(x for x in (libasan, os.environ.get("LD_PRELOAD", "")) if x)
    env = dict(os.environ, LD_PRELOAD=pre, ASAN_OPTIONS="detect_leaks=0:halt_on_error=1",
               UBSAN_OPTIONS="halt_on_error=1", OMP_NUM_THREADS="2")
    p = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, env=env, timeout=600, cwd=ROOT)
    _asan_clean(p)
    assert p.returncode == 0 and "oracle under asan ok" in p.stdout, p.stdout + p.stderr
