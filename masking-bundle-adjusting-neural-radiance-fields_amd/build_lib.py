"""Build libmarf.so (all HIP sources, gfx950 only) in-tree: lib/libmarf.so.

    python build_lib.py [--force]
    python build_lib.py --variant libmarf_<name>.so "<extra hipcc flags>"   (A/B variants, MARF_LIB=...)

The library is rebuilt when any source under csrc/ or include/ is newer than it.  Every build
embeds a hash of those sources (marker MARF_SOURCE_HASH=<sha1>); marf_hip.lib() compares it with
the sources next to it before loading, so an out-of-date binary is never loaded silently.
"""
import hashlib
import glob
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
LIB = os.path.join(HERE, "lib", "libmarf.so")
# diagnostic variant with in-kernel phase stamps (tools/phase_stamps.py); never loaded by default
LIB_STAMPS = os.path.join(HERE, "lib", "libmarf_stamps.so")
SOURCES = ["marf_lie.hip", "marf_mlp.hip", "marf_wgrad.hip", "marf_step.hip", "marf_step2.hip", "marf_misc.hip", "marf_edge.hip", "marf_abi.hip", "marf_prof.hip", "marf_comm.hip"]
FLAGS = ["--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-shared",
         # exact fp32 operation order for the bit-exact prologue (no implicit FMA contraction)
         "-ffp-contract=off", "-fno-slp-vectorize", "-Wall", "-Wno-unused-function"]


def source_hash():
    """sha1 over the names and contents of csrc/* and include/*.h (what every build compiles)."""
    h = hashlib.sha1()
    deps = sorted(glob.glob(os.path.join(HERE, "csrc", "*")) + glob.glob(os.path.join(ROOT, "include", "*.h")))
    for d in deps:
        h.update(os.path.relpath(d, ROOT).encode())
        with open(d, "rb") as f:
            h.update(f.read())
    return h.hexdigest()


def embedded_hash(lib_path):
    """The source hash a built library carries (None if it has no marker)."""
    with open(lib_path, "rb") as f:
        data = f.read()
    i = data.find(b"MARF_SOURCE_HASH=")
    if i < 0:
        return None
    return data[i + 17:i + 57].decode(errors="replace")


def _stale():
    if not os.path.exists(LIB):
        return True
    t = os.path.getmtime(LIB)
    deps = glob.glob(os.path.join(HERE, "csrc", "*")) + glob.glob(os.path.join(ROOT, "include", "*.h"))
    return any(os.path.getmtime(d) > t for d in deps)


def build(force=False, verbose=True, stamps=False):
    if stamps:
        extra = os.environ.get("MARF_EXTRA_FLAGS", "").split()
        name = os.environ.get("MARF_LIB_NAME")  # diagnostic variants side by side
        path = os.path.join(HERE, "lib", name) if name else LIB_STAMPS
        return _compile(path, ["-DMARF_STAMPS"] + extra, verbose)
    if not force and not _stale():
        return LIB
    return _compile(LIB, [], verbose)


OBJ_CACHE = os.path.join(HERE, "build", "obj")  # compiled translation units, keyed by their inputs


def _unit_key(src, cflags):
    """sha1 of one translation unit's compile: hipcc flags (less the library hash, which only
    marf_abi.hip embeds), its source and every header under csrc/ and include/."""
    h = hashlib.sha1()
    flags = [f for f in cflags if not f.startswith("-DMARF_SOURCE_HASH") or src == "marf_abi.hip"]
    h.update(" ".join(flags).encode())
    deps = [os.path.join(HERE, "csrc", src)] + sorted(glob.glob(os.path.join(HERE, "csrc", "*.h")) +
                                                      glob.glob(os.path.join(ROOT, "include", "*.h")))
    for d in deps:
        h.update(os.path.relpath(d, ROOT).encode())
        with open(d, "rb") as f:
            h.update(f.read())
    return h.hexdigest()[:16]


def _compile(lib_path, extra, verbose):
    """One hipcc process per translation unit (in parallel; units whose inputs are unchanged come
    from build/obj), then one link."""
    import shutil
    import tempfile
    hipcc = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
    os.makedirs(os.path.dirname(lib_path), exist_ok=True)
    os.makedirs(OBJ_CACHE, exist_ok=True)
    tmp = f"{lib_path}.tmp.{os.getpid()}"  # per process: concurrent builders never share a file
    if verbose:
        print("[marf] building", lib_path, flush=True)
    jobs = max(1, min(len(SOURCES), int(os.environ.get("MAX_JOBS", os.cpu_count() or 4))))
    with tempfile.TemporaryDirectory() as td:
        objs, procs, logs, cached = [], [], [], []
        cflags = [f for f in FLAGS if f != "-shared"] + [f'-DMARF_SOURCE_HASH="{source_hash()}"'] + list(extra)
        for src in SOURCES:
            key = _unit_key(src, cflags)
            keep = os.path.join(OBJ_CACHE, f"{src[:-4]}-{key}.o")
            cached.append(keep)
            obj = os.path.join(td, src.replace(".hip", ".o"))
            objs.append(obj)
            if os.path.exists(keep):
                shutil.copyfile(keep, obj)
                procs.append(None)
                logs.append(None)
                continue
            # compiler output to a file, not a pipe: a pipe nobody drains blocks a verbose compile
            log = open(obj + ".log", "w+")
            logs.append(log)
            procs.append(subprocess.Popen([hipcc] + cflags + ["-c", os.path.join(HERE, "csrc", src), "-o", obj],
                                          stdout=log, stderr=subprocess.STDOUT))
            while sum(p is not None and p.poll() is None for p in procs) >= jobs:
                procs[[p is not None and p.poll() is None for p in procs].index(True)].wait()
        errs = []
        for src, p, log, obj, keep in zip(SOURCES, procs, logs, objs, cached):
            if p is None:
                continue
            p.wait()
            log.seek(0)
            out = log.read()
            log.close()
            if p.returncode != 0:
                errs.append(f"{src}:\n{out}")
            else:
                shutil.copyfile(obj, keep + f".tmp.{os.getpid()}")
                os.replace(keep + f".tmp.{os.getpid()}", keep)
        if errs:
            raise RuntimeError("hipcc failed:\n" + "\n".join(errs))
        r = subprocess.run([hipcc, "--offload-arch=gfx950", "-shared", "-fPIC"] + objs + ["-o", tmp],
                           capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError("hipcc link failed:\n" + r.stdout + r.stderr)
    os.replace(tmp, lib_path)
    return lib_path


if __name__ == "__main__":
    if "--variant" in sys.argv:  # A/B builds: --variant libmarf_<x>.so "-DFLAG=..." (loaded via MARF_LIB)
        i = sys.argv.index("--variant")
        _compile(os.path.join(HERE, "lib", sys.argv[i + 1]), sys.argv[i + 2].split() if len(sys.argv) > i + 2 else [], True)
    else:
        build(force="--force" in sys.argv, stamps="--stamps" in sys.argv)
