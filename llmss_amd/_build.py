"""In-tree build of the native extension ``llmss_amd._C`` for gfx950.

Every ``csrc/*.hip`` kernel file and the host runtime ``csrc/*.cpp`` are compiled by ``hipcc
--offload-arch=gfx950`` (cross-compiles without a GPU) in parallel into ``build/obj`` and linked
into ``llmss_amd/_C*.so`` (linked against RCCL for the native communicator, csrc/comm.cpp). No torch headers, no hipify, no CUDA compatibility layer: bindings
take raw device pointers and a HIP stream handle (see ``csrc/bindings.cpp``).

Usage: ``python -m llmss_amd._build [--force] [-j N]``.
"""
from __future__ import annotations

import argparse
import concurrent.futures as cf
import glob
import hashlib
import os
import subprocess
import sys
import sysconfig

PKG = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(PKG)
CSRC = os.path.join(PKG, "csrc")
OBJ = os.path.join(ROOT, "build", "obj")
ARCH = os.environ.get("LLMSS_OFFLOAD_ARCH", "gfx950")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")


def ext_path() -> str:
    suffix = sysconfig.get_config_var("EXT_SUFFIX") or ".so"
    return os.path.join(PKG, "_C" + suffix)


def _includes():
    import pybind11

    return [f"-I{pybind11.get_include()}", f"-I{sysconfig.get_paths()['include']}", f"-I{CSRC}"]


def _flags():
    return [
        f"--offload-arch={ARCH}",
        "-O3",
        "-std=c++17",
        "-fPIC",
        "-fvisibility=hidden",
        "-Wno-unused-result",
        "-Wno-unused-variable",
        "-ffp-contract=fast",
        "-munsafe-fp-atomics",
    ]


def _sources():
    return sorted(glob.glob(os.path.join(CSRC, "*.hip")) + glob.glob(os.path.join(CSRC, "*.cpp")))


def _digest(src: str) -> str:
    h = hashlib.sha1()
    for p in [src] + sorted(glob.glob(os.path.join(CSRC, "*.h"))):
        with open(p, "rb") as f:
            h.update(f.read())
    h.update(" ".join(_flags()).encode())
    return h.hexdigest()[:16]


def _compile(src: str, force: bool) -> str:
    base = os.path.basename(src)
    obj = os.path.join(OBJ, base + ".o")
    stamp = obj + ".sha"
    dig = _digest(src)
    if not force and os.path.exists(obj) and os.path.exists(stamp):
        with open(stamp) as f:
            if f.read().strip() == dig:
                return obj
    lang = ["-x", "hip"] if src.endswith(".hip") else []
    cmd = [HIPCC] + _flags() + _includes() + lang + ["-c", src, "-o", obj]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"compile failed: {base}\n{' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
    with open(stamp, "w") as f:
        f.write(dig)
    return obj


def build(force: bool = False, jobs: int = 0, verbose: bool = False) -> str:
    os.makedirs(OBJ, exist_ok=True)
    srcs = _sources()
    jobs = jobs or min(len(srcs), max(1, (os.cpu_count() or 4)), 16)
    with cf.ThreadPoolExecutor(jobs) as ex:
        objs = list(ex.map(lambda s: _compile(s, force), srcs))
    out = ext_path()
    newest = max(os.path.getmtime(o) for o in objs)
    if force or not os.path.exists(out) or os.path.getmtime(out) < newest:
        tmp = out + ".tmp"
        cmd = [HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", tmp] + objs + ["-L/opt/rocm/lib", "-lrccl", "-Wl,-rpath,/opt/rocm/lib", "-lpthread"]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"link failed\n{' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
        os.replace(tmp, out)
    if verbose:
        print(out)
    return out


def is_built() -> bool:
    out = ext_path()
    if not os.path.exists(out):
        return False
    m = os.path.getmtime(out)
    return all(os.path.getmtime(s) <= m for s in _sources() + glob.glob(os.path.join(CSRC, "*.h")))


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--force", action="store_true")
    ap.add_argument("-j", "--jobs", type=int, default=0)
    a = ap.parse_args(argv)
    print(build(a.force, a.jobs, verbose=False))


if __name__ == "__main__":
    sys.exit(main())
