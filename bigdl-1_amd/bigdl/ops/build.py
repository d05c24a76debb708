"""Build ``libbigdl_kernels.so`` in-tree with hipcc for gfx950.

    python -m bigdl.ops.build [--jobs N] [--debug]

Each ``csrc/*.hip`` / ``*.cpp`` is compiled to an object under ``csrc/build/`` (re-used when the
source and headers are older than the object) and linked into ``lib/libbigdl_kernels.so``.
``--debug`` adds ``-DBIGDL_DEBUG`` (device-side bounds asserts) and host ASan/UBSan via
``-Xarch_host`` (GPU sanitizers are not available on the pool).
"""
from __future__ import annotations

import argparse
import concurrent.futures as cf
import glob
import os
import shutil
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
BUILD = os.path.join(CSRC, "build")
LIB = os.path.join(HERE, "lib", "libbigdl_kernels.so")
ARCH = os.environ.get("BIGDL_OFFLOAD_ARCH", "gfx950")


def hipcc() -> str:
    for p in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if p and os.path.exists(p):
            return p
    raise RuntimeError("hipcc not found")


def _needs(src, obj, headers):
    if not os.path.exists(obj):
        return True
    t = os.path.getmtime(obj)
    return any(os.path.getmtime(p) > t for p in [src] + headers)


def compile_one(src, debug=False):
    base = os.path.basename(src).rsplit(".", 1)[0]
    obj = os.path.join(BUILD, base + (".dbg" if debug else "") + ".o")
    headers = glob.glob(os.path.join(CSRC, "*.h"))
    if not _needs(src, obj, headers):
        return obj, None
    cmd = [hipcc(), "-c", "-fPIC", "-O3", "-std=c++17", f"--offload-arch={ARCH}", "-fvisibility=hidden",
           "-munsafe-fp-atomics", "-I", CSRC, src, "-o", obj]
    if src.endswith(".cpp"):
        cmd = [hipcc(), "-c", "-fPIC", "-O3", "-std=c++17", "-fvisibility=hidden", "-I", CSRC, src, "-o", obj]
    if debug:
        cmd[3:3] = ["-DBIGDL_DEBUG", "-g", "-Xarch_host", "-fsanitize=address,undefined"]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        return obj, f"{' '.join(cmd)}\n{r.stdout}\n{r.stderr}"
    return obj, None


def build(jobs: int = 8, debug: bool = False, verbose: bool = True) -> str:
    os.makedirs(BUILD, exist_ok=True)
    os.makedirs(os.path.dirname(LIB), exist_ok=True)
    srcs = sorted(glob.glob(os.path.join(CSRC, "*.hip")) + glob.glob(os.path.join(CSRC, "*.cpp")))
    objs, errs = [], []
    with cf.ThreadPoolExecutor(max_workers=max(1, jobs)) as ex:
        for obj, err in ex.map(lambda s: compile_one(s, debug), srcs):
            objs.append(obj)
            if err:
                errs.append(err)
    if errs:
        raise RuntimeError("HIP compile failed:\n" + "\n\n".join(errs))
    out = LIB if not debug else LIB.replace(".so", "_debug.so")
    if not os.path.exists(out) or any(os.path.getmtime(o) > os.path.getmtime(out) for o in objs):
        cmd = [hipcc(), "-shared", "-fPIC", f"--offload-arch={ARCH}", "-o", out] + objs
        if debug:
            cmd += ["-Xarch_host", "-fsanitize=address,undefined"]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"link failed:\n{' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
    # a kernel template whose host-side instantiation fails substitution gets no launch stub, and hipcc
    # reports no error: the library then fails to load on the GPU box.  Refuse such a link here.
    nm = shutil.which("nm") or "/opt/rocm/lib/llvm/bin/llvm-nm"
    r = subprocess.run([nm, "-D", "--undefined-only", out], capture_output=True, text=True)
    missing = [l.split()[-1] for l in r.stdout.splitlines() if "__device_stub__" in l]
    if missing:
        os.remove(out)
        raise RuntimeError("kernel launch stubs undefined (host-side template substitution failed): " +
                           ", ".join(missing[:6]))
    if verbose:
        print(f"[bigdl.ops.build] {out} ({len(objs)} objects, arch {ARCH})")
    return out


RT_CSRC = os.path.join(os.path.dirname(HERE), "runtime", "csrc")
RT_LIB = os.path.join(os.path.dirname(HERE), "runtime", "lib", "libbigdl_runtime.so")


def build_runtime(verbose: bool = True, debug: bool = False) -> str:
    """Host-only native runtime (threaded batch loader, …): ``runtime/csrc/*.cpp`` → g++ -O3."""
    srcs = sorted(glob.glob(os.path.join(RT_CSRC, "*.cpp")))
    os.makedirs(os.path.dirname(RT_LIB), exist_ok=True)
    if not srcs:
        return RT_LIB
    if os.path.exists(RT_LIB) and all(os.path.getmtime(s) <= os.path.getmtime(RT_LIB) for s in srcs):
        return RT_LIB
    cxx = os.environ.get("CXX") or shutil.which("g++") or "g++"
    cmd = [cxx, "-O3", "-std=c++17", "-shared", "-fPIC", "-pthread", "-fvisibility=hidden", "-o", RT_LIB] + srcs
    if debug:
        cmd[1:1] = ["-g", "-fsanitize=address,undefined", "-fno-omit-frame-pointer"]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"runtime build failed:\n{' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
    if verbose:
        print(f"[bigdl.ops.build] {RT_LIB} ({len(srcs)} sources, host)")
    return RT_LIB


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--jobs", type=int, default=min(8, os.cpu_count() or 1))
    ap.add_argument("--debug", action="store_true")
    a = ap.parse_args()
    build(a.jobs, a.debug)
    build_runtime(debug=a.debug)


if __name__ == "__main__":
    sys.exit(main())
