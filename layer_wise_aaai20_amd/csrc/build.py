"""Build the in-tree HIP extension ``layer_wise_aaai20_amd/_lwaaai_C.so`` for gfx950.

Every ``*.hip`` / ``*.cpp`` under ``csrc/`` is compiled with ``hipcc --offload-arch=gfx950 -c`` and
the objects are linked with the host C++ linker against the HIP runtime *bundled with PyTorch*
(``torch/lib/libamdhip64.so``, soname ``libamdhip64.so.7``) so that exactly one HIP runtime is
loaded in the process. No hipify step, no CUDA sources, no JIT cache: the ``.so`` lands next to the
package and travels with the repo snapshot.

Usage: ``python -m layer_wise_aaai20_amd.csrc.build [--force] [-j N]``
"""
from __future__ import annotations

import argparse
import concurrent.futures as cf
import hashlib
import os
import subprocess
import sys
import sysconfig

HERE = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.dirname(HERE)
# experiment builds: LWAAAI_SO names another output (loaded by ops/_ext.py from the same
# variable), LWAAAI_HIPCC_FLAGS adds compile flags (e.g. -DLW_GLDS=0), objects go to their own dir
OUT = os.environ.get("LWAAAI_SO") or os.path.join(PKG, "_lwaaai_C.so")
EXTRA = os.environ.get("LWAAAI_HIPCC_FLAGS", "").split()
BUILD = os.path.join(HERE, "build" + ("" if not os.environ.get("LWAAAI_SO") else
                                      "_" + os.path.basename(OUT).replace(".so", "")))
ARCH = os.environ.get("LWAAAI_ARCH", "gfx950")


def _hipcc() -> str:
    for c in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc"):
        if c and os.path.exists(c):
            return c
    return "hipcc"


def _torch_paths():
    import torch
    root = os.path.dirname(torch.__file__)
    inc = [os.path.join(root, "include"), os.path.join(root, "include", "torch", "csrc", "api",
                                                       "include")]
    lib = os.path.join(root, "lib")
    abi = int(torch._C._GLIBCXX_USE_CXX11_ABI)
    return inc, lib, abi


def sources():
    return sorted(os.path.join(HERE, f) for f in os.listdir(HERE)
                  if f.endswith((".hip", ".cpp")))


def _digest(paths, flags=()) -> str:
    h = hashlib.sha256()
    for p in sorted(paths):
        with open(p, "rb") as f:
            h.update(p.encode())
            h.update(f.read())
    h.update(ARCH.encode())
    h.update(" ".join(EXTRA + list(flags)).encode())
    return h.hexdigest()[:16]


def _compile(src, inc, abi, bdir=BUILD, flags=(), dig=""):
    """One object; skipped when ``obj.stamp`` holds the digest of (this source, every header,
    the flags) — an edit to one kernel file recompiles that file only."""
    obj = os.path.join(bdir, os.path.basename(src) + ".o")
    ostamp = obj + ".stamp"
    if dig and os.path.exists(obj) and os.path.exists(ostamp):
        with open(ostamp) as f:
            if f.read().strip() == dig:
                return obj
    cmd = [_hipcc(), f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-c", src, "-o", obj,
           f"-D_GLIBCXX_USE_CXX11_ABI={abi}", "-DUSE_ROCM", "-D__HIP_PLATFORM_AMD__=1",
           "-Wno-unused-result", "-Wno-deprecated-declarations", f"-I{HERE}"] + EXTRA + list(flags)
    if src.endswith(".cpp"):
        cmd += [f"-I{p}" for p in inc] + [f"-I{sysconfig.get_paths()['include']}"]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"hipcc failed for {src}:\n{' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
    if dig:
        with open(ostamp, "w") as f:
            f.write(dig)
    return obj


# The fp16 build of the same kernels (csrc/elem16.h: fp16 conversions, v_mfma_f32_16x16x32_f16),
# registered as torch.ops.lwaaai16 and used when the fused path runs the reference's --fp16
# recipe (ops/_ext.py set_half). The communicator (rccl.cpp) lives only in the main library.
OUT16 = os.environ.get("LWAAAI_SO16") or os.path.join(PKG, "_lwaaai16_C.so")
FLAGS16 = ["-DLW_FP16", "-DLW_OPS_NS=lwaaai16"]


def _build_one(out, bdir, flags, srcs, force, jobs, verbose):
    headers = [os.path.join(HERE, f) for f in os.listdir(HERE) if f.endswith(".h")]
    stamp = os.path.join(bdir, "stamp")
    dig = _digest(srcs + headers + [os.path.abspath(__file__)], flags)
    if not force and os.path.exists(out) and os.path.exists(stamp):
        with open(stamp) as f:
            if f.read().strip() == dig:
                if verbose:
                    print(f"[lwaaai] up to date: {out}")
                return out
    os.makedirs(bdir, exist_ok=True)
    inc, lib, abi = _torch_paths()
    jobs = jobs or min(8, len(srcs), os.cpu_count() or 4)
    if verbose:
        print(f"[lwaaai] compiling {len(srcs)} sources for {ARCH} ({' '.join(flags) or 'bf16'}) "
              f"with {jobs} jobs")
    odig = {s: ("" if force else _digest([s] + headers + [os.path.abspath(__file__)], flags))
            for s in srcs}
    with cf.ThreadPoolExecutor(jobs) as ex:
        objs = list(ex.map(lambda s: _compile(s, inc, abi, bdir, flags, odig[s]), srcs))
    tmp = out + ".tmp"
    cmd = ["g++", "-shared", "-o", tmp] + objs + [
        f"-L{lib}", "-lc10", "-lc10_hip", "-ltorch", "-ltorch_cpu", "-ltorch_hip",
        "-l:libamdhip64.so", "-lrccl", f"-Wl,-rpath,{lib}", "-Wl,-z,defs"]   # unresolved symbols fail here
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"link failed:\n{' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
    os.replace(tmp, out)
    with open(stamp, "w") as f:
        f.write(dig)
    if verbose:
        print(f"[lwaaai] built {out}")
    return out


def build(force: bool = False, jobs: int = 0, verbose: bool = True, half: bool = True) -> str:
    """Build the bf16 library (and, with ``half``, its fp16 twin); returns the bf16 one's path."""
    srcs = sources()
    main = _build_one(OUT, BUILD, [], srcs, force, jobs, verbose)
    if half and not os.environ.get("LWAAAI_SO"):
        _build_one(OUT16, os.path.join(HERE, "build_fp16"), FLAGS16,
                   [s for s in srcs if not s.endswith("rccl.cpp")], force, jobs, verbose)
    return main


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--force", action="store_true")
    ap.add_argument("-j", type=int, default=0)
    args = ap.parse_args()
    build(args.force, args.j)
    sys.exit(0)
