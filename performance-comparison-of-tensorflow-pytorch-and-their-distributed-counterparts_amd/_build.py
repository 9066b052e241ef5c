"""In-tree native build for the framework (hipcc, gfx950 only).

Compiles every ``csrc/*.hip`` (device + op-registration host code) with ``hipcc
--offload-arch=gfx950`` and every ``csrc/runtime/*.cpp`` (host-only native runtime: text
pipeline, bucket planner, ...) with ``g++``, then links one shared library
``_native/libpcmp_hip.so`` next to this file.  The library registers its ops in the
``torch.ops.pcmp`` namespace (``TORCH_LIBRARY_FRAGMENT``) and is loaded with
``torch.ops.load_library``.  Objects are rebuilt only when a source or header is newer.

Usage: ``python -c "import pcmp._build as b; b.build()"`` (also called by
``__graft_entry__.build()``).
"""
from __future__ import annotations

import concurrent.futures as cf
import os
import pathlib
import subprocess
import sys
import sysconfig

PKG = pathlib.Path(__file__).resolve().parent
CSRC = PKG / "csrc"
OUT_DIR = PKG / "_native"
OBJ_DIR = PKG.parent / "build" / "obj"
LIB = OUT_DIR / "libpcmp_hip.so"
ARCH = "gfx950"
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")


def _torch_paths():
    import torch
    from torch.utils import cpp_extension as ce
    inc = [
        os.path.join(os.path.dirname(torch.__file__), "include"),
        os.path.join(os.path.dirname(torch.__file__), "include", "torch", "csrc", "api", "include"),
    ]
    libdir = ce.library_paths()[0]
    abi = int(torch._C._GLIBCXX_USE_CXX11_ABI)
    return inc, libdir, abi


def _common_flags(inc, abi):
    py_inc = sysconfig.get_paths()["include"]
    flags = ["-O3", "-std=c++17", "-fPIC", f"-D_GLIBCXX_USE_CXX11_ABI={abi}",
             "-DTORCH_API_INCLUDE_EXTENSION_H", "-DTORCH_EXTENSION_NAME=pcmp_hip",
             "-D__HIP_PLATFORM_AMD__=1", "-DUSE_ROCM=1", "-Wno-unused-result",
             "-Wno-deprecated-declarations", f"-I{py_inc}", f"-I{CSRC}"]
    for d in inc:
        flags.append(f"-I{d}")
    flags.append("-I/opt/rocm/include")
    return flags


def _local_includes(path: pathlib.Path, seen=None) -> set:
    """Local headers (``#include "x.h"``) a source includes, transitively."""
    seen = set() if seen is None else seen
    for line in path.read_text(errors="ignore").splitlines():
        line = line.strip()
        if line.startswith("#include \""):
            name = line.split('"')[1]
            h = (path.parent / name).resolve()
            if not h.exists():   # -I csrc: "runtime/x.h" from csrc/runtime/*.cpp
                h = (CSRC / name).resolve()
            if h.exists() and h not in seen:
                seen.add(h)
                _local_includes(h, seen)
    return seen


def _deps_newer(obj: pathlib.Path, src: pathlib.Path) -> bool:
    if not obj.exists():
        return True
    t = obj.stat().st_mtime
    if src.stat().st_mtime > t:
        return True
    return any(h.stat().st_mtime > t for h in _local_includes(src))


def _compile(cmd, src):
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"compile failed: {src}\n{' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
    return src


def sources():
    return sorted(CSRC.glob("*.hip")) + sorted((CSRC / "runtime").glob("*.cpp"))


def build(verbose: bool = True, jobs: int | None = None) -> pathlib.Path:
    inc, libdir, abi = _torch_paths()
    OBJ_DIR.mkdir(parents=True, exist_ok=True)
    OUT_DIR.mkdir(parents=True, exist_ok=True)
    flags = _common_flags(inc, abi)
    jobs = jobs or min(8, os.cpu_count() or 4)
    todo, objs = [], []
    for src in sources():
        obj = OBJ_DIR / (src.stem + ("_hip.o" if src.suffix == ".hip" else "_cpp.o"))
        objs.append(obj)
        if not _deps_newer(obj, src):
            continue
        if src.suffix == ".hip":
            cmd = [HIPCC, f"--offload-arch={ARCH}", "-munsafe-fp-atomics", "-ffp-contract=fast",
                   *flags, "-x", "hip", "-c", str(src), "-o", str(obj)]
        else:
            cmd = ["g++", *flags, "-fopenmp", "-c", str(src), "-o", str(obj)]
        todo.append((cmd, src))
    if todo:
        with cf.ThreadPoolExecutor(jobs) as ex:
            futs = [ex.submit(_compile, c, s) for c, s in todo]
            for f in cf.as_completed(futs):
                s = f.result()
                if verbose:
                    print(f"[pcmp build] compiled {s.name}", flush=True)
    need_link = bool(todo) or not LIB.exists() or any(o.stat().st_mtime > LIB.stat().st_mtime for o in objs)
    if need_link:
        # link to a temporary name and rename: a reader (a running process, a tree snapshot) sees
        # the old or the new library, never a partly written one
        tmp = LIB.with_name(LIB.name + ".tmp")
        cmd = [HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", str(tmp), *map(str, objs),
               f"-L{libdir}", f"-Wl,-rpath,{libdir}", "-lc10", "-lc10_hip", "-ltorch", "-ltorch_cpu",
               "-ltorch_hip", "-fopenmp"]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"link failed\n{' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
        os.replace(tmp, LIB)
        if verbose:
            print(f"[pcmp build] linked {LIB}", flush=True)
    return LIB


if __name__ == "__main__":
    build()
    sys.exit(0)
