"""Build libfastconsensus_amd.so (HIP for gfx950) in-tree with hipcc.

    python -m fastconsensus_amd.build      # or __graft_entry__.build()
"""
import concurrent.futures as cf
import hashlib
import os
import subprocess
import sys

PKG = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(PKG, "csrc")
OUT_DIR = os.path.join(PKG, "lib")
LIB = os.path.join(OUT_DIR, "libfastconsensus_amd.so")
SRC_HASH = LIB + ".srchash"     # the source hash the library was built from (profiles are matched to it)
BUILD_REC = os.path.join(OUT_DIR, "BUILD.json")   # what the last build() did (provenance record)
SOURCES = ["graph.hip", "consensus.hip", "cd.hip", "cd_rl.hip", "leiden.hip", "capi.cpp", "gen.cpp"]
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = "gfx950"
FLAGS = ["-O3", "-fPIC", "-std=c++17", "--offload-arch=" + ARCH, "-Wall", "-Wno-unused-function",
         "-I" + os.path.join(os.path.dirname(PKG), "include")]


def _obj(src):
    return os.path.join(OUT_DIR, "obj", src + ".o")


def _deps():
    return [os.path.join(CSRC, f) for f in os.listdir(CSRC)] + \
        [os.path.join(os.path.dirname(PKG), "include", "fastconsensus_amd.h")]


def source_hash():
    """sha256 (16 hex) over the library's sources and header, by name, and the compile flags and
    target: what a PMC profile under profiles/ records (bench.py attaches traffic only from a
    profile of the same code), and what the library embeds (fc_build_hash, compiled into
    capi.cpp), so a binary built from other sources OR other flags is detected."""
    h = hashlib.sha256()
    # the flags without the include path (absolute, so it differs between checkouts)
    h.update(" ".join([f for f in FLAGS if not f.startswith("-I")] + ["--offload-arch=" + ARCH]).encode())
    for d in sorted(_deps(), key=os.path.basename):
        if os.path.isfile(d):
            h.update(os.path.basename(d).encode())
            with open(d, "rb") as f:
                h.update(f.read())
    return h.hexdigest()[:16]


def built_hash():
    """Source hash recorded when the library was linked (None if unknown)."""
    try:
        with open(SRC_HASH) as f:
            return f.read().strip() or None
    except OSError:
        return None


def _compile(src):
    """-> (object path, whether it was compiled now)"""
    path = os.path.join(CSRC, src)
    obj = _obj(src)
    newest = max(os.path.getmtime(d) for d in _deps())
    stamp = obj + ".hash"                       # capi.cpp embeds the source hash (fc_build_hash)
    fresh = os.path.exists(obj) and os.path.getmtime(obj) >= newest
    if fresh and src == "capi.cpp":
        try:
            with open(stamp) as f:
                fresh = f.read().strip() == source_hash()
        except OSError:
            fresh = False
    if fresh:
        return obj, False
    lang = ["-x", "hip"] if src.endswith(".hip") else []
    cmd = [HIPCC] + FLAGS + lang + ["-c", path, "-o", obj]
    if src == "capi.cpp":   # the library reports what it was built from (fc_build_hash)
        cmd += ['-DFC_BUILD_HASH="%s"' % source_hash()]
    subprocess.check_call(cmd)
    if src == "capi.cpp":
        with open(stamp, "w") as f:
            f.write(source_hash() + "\n")
    return obj, True


def _record(compiled, linked):
    """BUILD.json: the build mode of the last build() -- which objects were compiled, whether the
    library was relinked -- and the source hash it stands for."""
    import json
    import time
    try:
        ver = subprocess.run([HIPCC, "--version"], capture_output=True, text=True, timeout=60).stdout
        ver = next((l.strip() for l in ver.splitlines() if "HIP version" in l), ver.strip()[:80])
    except (OSError, subprocess.SubprocessError):
        ver = None
    rec = {"source_hash": source_hash(), "built_hash": built_hash(), "arch": ARCH, "hipcc": ver,
           "compiled": compiled, "relinked": linked,
           "build_mode": "compiled" if compiled else ("relinked" if linked else "up-to-date"),
           "utc": time.strftime("%Y-%m-%dT%H:%M:%SZ", time.gmtime())}
    with open(BUILD_REC, "w") as f:
        json.dump(rec, f, indent=1)
    return rec


def build(verbose=True, jobs=None):
    os.makedirs(os.path.join(OUT_DIR, "obj"), exist_ok=True)
    jobs = jobs or min(len(SOURCES), max(1, (os.cpu_count() or 4) // 2), 8)
    with cf.ThreadPoolExecutor(jobs) as ex:
        res = list(ex.map(_compile, SOURCES))
    objs = [o for o, _ in res]
    compiled = [src for src, (_, c) in zip(SOURCES, res) if c]
    if os.path.exists(LIB) and os.path.getmtime(LIB) >= max(os.path.getmtime(o) for o in objs) \
            and built_hash() == source_hash():
        _record(compiled, False)
        return LIB
    cmd = [HIPCC, "--offload-arch=" + ARCH, "-shared", "-fPIC", "-o", LIB] + objs
    subprocess.check_call(cmd)
    with open(SRC_HASH, "w") as f:
        f.write(source_hash() + "\n")
    _record(compiled, True)
    if verbose:
        print("built", LIB, file=sys.stderr)
    return LIB


if __name__ == "__main__":
    build()
