"""In-tree build of libccsc.so for gfx950 (hipcc, parallel object compiles).

Usage:  python -m ccsc_code_iccv2017_amd.build [--force]
The shared library lands next to this file so it travels with the repo
snapshot to the GPU box (it is git-ignored, not gpurun-ignored).
"""
from __future__ import annotations

import concurrent.futures as cf
import hashlib
import os
import subprocess
import sys
from pathlib import Path

PKG = Path(__file__).resolve().parent
CSRC = PKG / "csrc"
OBJ = PKG.parent / "build" / "obj"
LIB = PKG / "libccsc.so"
ROCM = Path(os.environ.get("ROCM_PATH", "/opt/rocm"))
HIPCC = str(ROCM / "bin" / "hipcc")
ARCH = "gfx950"
CFLAGS = ["-O3", "-std=c++17", "-fPIC", f"--offload-arch={ARCH}", "-Wall", "-Wno-unused-function"]


def _sources():
    return sorted(list(CSRC.glob("*.hip")) + list(CSRC.glob("*.cpp")))


def _deps():
    return sorted(list(CSRC.glob("*.hpp")) + [PKG.parent / "include" / "ccsc.h"])


def source_hash() -> str:
    """sha256 over the names and contents of every source and header the library is built
    from (written next to the library as libccsc.srchash; tools/check_lib.py compares)."""
    h = hashlib.sha256()
    for p in sorted(_sources() + _deps(), key=lambda q: q.name):
        h.update(p.name.encode())
        h.update(p.read_bytes())
    return h.hexdigest()


def _needs(target: Path, inputs) -> bool:
    if not target.exists():
        return True
    t = target.stat().st_mtime
    return any(p.stat().st_mtime > t for p in inputs)


def _compile(src: Path, force: bool) -> Path:
    obj = OBJ / (src.name + ".o")
    if force or _needs(obj, [src] + _deps()):
        cmd = [HIPCC] + CFLAGS + ["-c", str(src), "-o", str(obj)]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"hipcc failed for {src.name}:\n{r.stderr[-6000:]}")
    return obj


def build(force: bool = False, jobs: int | None = None) -> Path:
    OBJ.mkdir(parents=True, exist_ok=True)
    srcs = _sources()
    jobs = jobs or min(len(srcs), max(1, min(8, os.cpu_count() or 1)))
    with cf.ThreadPoolExecutor(max_workers=jobs) as ex:
        objs = list(ex.map(lambda s: _compile(s, force), srcs))
    stamp = OBJ / "libccsc.objs"
    sig = "\n".join(f"{o}:{o.stat().st_mtime_ns}" for o in objs)
    libsig = f"{LIB.stat().st_mtime_ns}:{LIB.stat().st_size}" if LIB.exists() else "none"
    # stale if the object set changed or the library was replaced behind our back
    stale = not stamp.exists() or stamp.read_text() != sig + "\n" + libsig
    if force or stale or _needs(LIB, objs):
        cmd = [HIPCC, f"--offload-arch={ARCH}", "-shared", "-o", str(LIB)] + [str(o) for o in objs]
        cmd += [f"-L{ROCM / 'lib'}", "-lrccl", f"-Wl,-rpath,{ROCM / 'lib'}"]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"link failed:\n{r.stderr[-6000:]}")
        stamp.write_text(sig + "\n" + f"{LIB.stat().st_mtime_ns}:{LIB.stat().st_size}")
    # the library is now the link of these sources (a replaced library fails the stamp above)
    LIB.with_suffix(".srchash").write_text(source_hash() + "\n")
    return LIB


PROBE_SRC = PKG.parent / "tools" / "copy_probe.hip"
PROBE = PKG.parent / "tools" / "libcopy_probe.so"


def build_probe(force: bool = False) -> Path:
    """bench.py's streaming-copy probe (tools/copy_probe.hip -> tools/libcopy_probe.so)."""
    if force or _needs(PROBE, [PROBE_SRC]):
        cmd = [HIPCC] + CFLAGS + ["-shared", str(PROBE_SRC), "-o", str(PROBE)]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"hipcc failed for {PROBE_SRC.name}:\n{r.stderr[-6000:]}")
    return PROBE


if __name__ == "__main__":
    print(build(force="--force" in sys.argv))
    print(build_probe(force="--force" in sys.argv))
