"""Guard against tree contents the GPU pool refuses (round 2's driver GPU run was refused for a bare
sanitizer flag on a hipcc link line in tests/asan/build.sh).  Scans every tracked file that gpurun
ships (i.e. not matched by .gpurunignore) for:

* a `-fsanitize=` not directly preceded by `-Xarch_host` (unless the statement carries
  `-fno-gpu-sanitize` and no `-Xarch_` option at all);
* XNACK-on settings;
* a hardware-queue override above 32;
* rocprofv3 counter collection combined with trace domains.

CPU only; this file itself is listed in .gpurunignore."""
import fnmatch
import os
import re
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SCANNED = (".sh", ".py", ".hip", ".cpp", ".c", ".h", ".mk", "Makefile")


def _ignore_patterns():
    pats = []
    with open(os.path.join(ROOT, ".gpurunignore")) as f:
        for line in f:
            line = line.strip()
            if line and not line.startswith("#"):
                pats.append(line)
    return pats


def _ignored(path, pats):
    for p in pats:
        if p.startswith("./"):
            top = p[2:].rstrip("/")
            if path == top or path.startswith(top + "/") or fnmatch.fnmatch(path, top):
                return True
        elif fnmatch.fnmatch(os.path.basename(path), p) or fnmatch.fnmatch(path, p):
            return True
    return False


def _shipped_files():
    try:
        out = subprocess.run(["git", "ls-files", "-co", "--exclude-standard"], cwd=ROOT, capture_output=True,
                             text=True, check=True).stdout.split()
    except (OSError, subprocess.CalledProcessError):
        pytest.skip("git unavailable")
    pats = _ignore_patterns()
    return [p for p in out if p.endswith(SCANNED) and not _ignored(p, pats) and os.path.isfile(os.path.join(ROOT, p))]


def _statements(text):
    """Shell-ish statements: backslash continuations joined."""
    return text.replace("\\\n", " ").splitlines()


SAN_OK = re.compile(r"-Xarch_host[\"',\s]+-fsanitize=")


def _bad_sanitizer(stmt):
    n = stmt.count("-fsanitize=")
    if n == 0:
        return False
    if len(SAN_OK.findall(stmt)) == n:
        return False
    return not ("-fno-gpu-sanitize" in stmt and "-Xarch_" not in stmt)


def test_gpurunignore_covers_cpu_only_helpers():
    pats = _ignore_patterns()
    for p in ("tests/asan/build.sh", "tests/test_asan_host.py", "tests/test_pool_rules.py"):
        assert _ignored(p, pats), p
    for p in ("fastconsensus_amd/lib/libfastconsensus_amd.so", "fastconsensus_amd/csrc/cd.hip", "bench.py",
              "tests/test_gpu_parity.py", "oracle/fc_oracle.c", "__graft_entry__.py"):
        assert not _ignored(p, pats), p


def test_no_gpu_sanitizer_or_xnack_in_shipped_tree():
    bad = []
    xnack_on = re.compile(r"HSA_XNACK\s*=\s*[\"']?1|xnack\+")
    queues = re.compile(r"GPU_MAX_HW_QUEUES\D{0,4}(\d+)")
    trace_domains = ("--sys-trace", "--runtime-trace", "--hip-trace", "--hsa-trace", "--memory-copy-trace",
                     "--scratch-memory-trace", "--marker-trace", " -s ", " -r ")
    for p in _shipped_files():
        with open(os.path.join(ROOT, p), errors="replace") as f:
            text = f.read()
        for i, st in enumerate(_statements(text)):
            if _bad_sanitizer(st):
                bad.append("%s: bare sanitizer: %s" % (p, st.strip()[:160]))
            if xnack_on.search(st):
                bad.append("%s: xnack on: %s" % (p, st.strip()[:160]))
            for q in queues.findall(st):
                if int(q) > 32:
                    bad.append("%s: hw queues %s" % (p, q))
            if "rocprofv3" in st and ("--pmc" in st or " -i " in st) and any(d in st + " " for d in trace_domains):
                bad.append("%s: pmc with trace domains: %s" % (p, st.strip()[:160]))
    assert not bad, "\n".join(bad)


def test_scanner_flags_the_round2_line():
    assert _bad_sanitizer('$HIPCC --offload-arch=gfx950 -fsanitize=address -fsanitize=undefined -g -o x')
    assert not _bad_sanitizer('$HIPCC -Xarch_host -fsanitize=address -Xarch_host -fsanitize=undefined -o x')
    assert not _bad_sanitizer('hipcc -fsanitize=address -fno-gpu-sanitize -o x')
    assert _bad_sanitizer('hipcc -fsanitize=address -fno-gpu-sanitize -Xarch_host -O2 -o x')
    assert not _bad_sanitizer('["gcc", "-Xarch_host", "-fsanitize=address"]')
