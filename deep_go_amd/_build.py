"""In-tree native build: hipcc for the gfx950 kernels, g++ for the CPU engine.

Produces ``deep_go_amd/_native/_dghip<EXT>`` (HIP kernels, pybind11) and
``deep_go_amd/_native/_dgcpu<EXT>`` (Go engine, t7 codec, SGF parser, loader thread
pool).  Built in-tree so the ``.so`` files travel with the repo snapshot to the GPU box.

Usage: ``python -m deep_go_amd._build [--force] [--only hip|cpu] [--sanitize thread|address]``
"""
from __future__ import annotations

import argparse
import concurrent.futures as cf
import os
import subprocess
import sys
import sysconfig
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
PKG = ROOT / "deep_go_amd"
OUT = PKG / "_native"
BUILD = ROOT / "build"
KDIR = ROOT / "csrc" / "kernels"
EDIR = ROOT / "csrc" / "engine"
CDIR = ROOT / "csrc" / "comm"
ARCH = os.environ.get("PYTORCH_ROCM_ARCH", "gfx950")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
CXX = os.environ.get("CXX", "g++")
EXT = sysconfig.get_config_var("EXT_SUFFIX") or ".so"

HIP_SOURCES = ["conv_mfma.hip", "conv_board.hip", "conv_stack2.hip", "conv_layer2.hip", "conv_stack_f8.hip", "conv_wgrad_win.hip", "conv_wgrad_win8.hip", "conv_l1.hip", "conv_fp8.hip", "head.hip", "head_mfma.hip", "elementwise.hip", "bindings.cpp"]
CPU_SOURCES = ["go_engine.cpp", "sgf.cpp", "t7.cpp", "features.cpp", "loader.cpp",
               "bindings.cpp"]


def _pybind_includes():
    import pybind11
    return [f"-I{pybind11.get_include()}", f"-I{sysconfig.get_paths()['include']}"]


def _newer(src: Path, dst: Path, deps=()) -> bool:
    if not dst.exists():
        return True
    t = dst.stat().st_mtime
    return src.stat().st_mtime > t or any(d.stat().st_mtime > t for d in deps)


def _run(cmd):
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"build failed: {' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
    return r


def build_hip(force: bool = False, jobs: int = 8) -> Path:
    BUILD.mkdir(exist_ok=True)
    OUT.mkdir(exist_ok=True)
    target = OUT / f"_dghip{EXT}"
    headers = list(KDIR.glob("*.h"))
    objs, cmds = [], []
    for s in HIP_SOURCES:
        src = KDIR / s
        if not src.exists():
            continue
        obj = BUILD / ("hip_" + s + ".o")
        objs.append(obj)
        if force or _newer(src, obj, headers):
            cmd = [HIPCC, f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC",
                   "-munsafe-fp-atomics", "-Wno-unused-result", "-c", str(src), "-o", str(obj)]
            if s.endswith(".cpp"):
                cmd = [HIPCC, "-O2", "-std=c++17", "-fPIC", *(_pybind_includes()), "-c",
                       str(src), "-o", str(obj)]
            cmds.append(cmd)
    with cf.ThreadPoolExecutor(max_workers=jobs) as ex:
        list(ex.map(_run, cmds))
    if force or cmds or not target.exists():
        _run([HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", "--hip-link", "-o",
              str(target), *map(str, objs)])
    return target


def build_cpu(force: bool = False, jobs: int = 8, sanitize: str | None = None) -> Path:
    BUILD.mkdir(exist_ok=True)
    OUT.mkdir(exist_ok=True)
    suffix = f"_{sanitize}" if sanitize else ""
    target = OUT / f"_dgcpu{suffix}{EXT}"
    headers = list(EDIR.glob("*.h"))
    flags = ["-O3", "-std=c++17", "-fPIC", "-pthread", "-Wall", "-Wno-sign-compare"]
    if sanitize:
        flags = ["-O1", "-g", "-std=c++17", "-fPIC", "-pthread", f"-fsanitize={sanitize}",
                 "-fno-omit-frame-pointer"]
    objs, cmds = [], []
    for s in CPU_SOURCES:
        src = EDIR / s
        obj = BUILD / (f"cpu{suffix}_" + s + ".o")
        objs.append(obj)
        if force or _newer(src, obj, headers):
            cmds.append([CXX, *flags, *(_pybind_includes()), "-c", str(src), "-o", str(obj)])
    with cf.ThreadPoolExecutor(max_workers=jobs) as ex:
        list(ex.map(_run, cmds))
    if force or cmds or not target.exists():
        link = [CXX, "-shared", "-pthread", "-o", str(target), *map(str, objs)]
        if sanitize:
            link.insert(1, f"-fsanitize={sanitize}")
        _run(link)
    return target


def build_comm(force: bool = False) -> Path:
    """_dgcomm: native RCCL communicator (host code; links librccl.so.1 — at run time the copy
    torch already mapped, same SONAME)."""
    BUILD.mkdir(exist_ok=True)
    OUT.mkdir(exist_ok=True)
    target = OUT / f"_dgcomm{EXT}"
    src = CDIR / "comm.cpp"
    kern = CDIR / "oneshot.hip"       # the one-shot IPC all-reduce kernel (small buckets)
    obj = BUILD / "comm_oneshot.hip.o"
    if force or _newer(kern, obj):
        _run([HIPCC, "-O3", "-std=c++17", "-fPIC", f"--offload-arch={ARCH}", "-c", str(kern),
              "-o", str(obj)])
    hobj = BUILD / "comm_host.cpp.o"
    if force or _newer(src, hobj):
        _run([HIPCC, "-O2", "-std=c++17", "-fPIC", f"--offload-arch={ARCH}", "-c",
              *(_pybind_includes()), "-I/opt/rocm/include", str(src), "-o", str(hobj)])
    if force or _newer(hobj, target) or _newer(obj, target):
        _run([HIPCC, "-shared", "-fPIC", f"--offload-arch={ARCH}", str(hobj), str(obj), "-o",
              str(target), "-L/opt/rocm/lib", "-lrccl", "-lamdhip64"])
    return target


def build_all(force: bool = False) -> None:
    build_cpu(force)
    build_hip(force)
    build_comm(force)


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--force", action="store_true")
    ap.add_argument("--only", choices=["hip", "cpu", "comm"])
    ap.add_argument("--sanitize", choices=["thread", "address", "address,undefined"])
    ap.add_argument("-j", type=int, default=min(8, os.cpu_count() or 4))
    a = ap.parse_args(argv)
    if a.only in (None, "cpu"):
        print(build_cpu(a.force, a.j, a.sanitize))
    if a.only in (None, "hip") and not a.sanitize:
        print(build_hip(a.force, a.j))
    if a.only in (None, "comm") and not a.sanitize:
        print(build_comm(a.force))


if __name__ == "__main__":
    main()
