"""Build recipe for the MI355X SPF engine (in-tree, no JIT cache):

  libopenr_spf.so        hipcc --offload-arch=gfx950  csrc/spf_device.hip
  _openr_spf*.so         g++ host C++ (LinkState / SpfSolver / PrefixState)
                         + pybind11 bindings, linked to libopenr_spf.so

Run `python -m openr_amd.build` (or __graft_entry__.build()).  Targets are
rebuilt only when a source is newer than the output.
"""

from __future__ import annotations

import glob
import os
import subprocess
import sys
import sysconfig

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
INC = os.path.join(ROOT, "include")
CSRC = os.path.join(HERE, "csrc")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = os.environ.get("OPENR_SPF_ARCH", "gfx950")

LIB = os.path.join(HERE, "libopenr_spf.so")
EXT = os.path.join(HERE, "_openr_spf" + sysconfig.get_config_var("EXT_SUFFIX"))


def _newer(target, sources):
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(s) > t for s in sources)


def _run(cmd):
    print("[openr_amd.build]", " ".join(cmd), flush=True)
    subprocess.run(cmd, check=True)


def build_device(force=False):
    srcs = [os.path.join(CSRC, "spf_device.hip"), os.path.join(CSRC, "spf_cluster.hip"),
            os.path.join(INC, "openr_spf.h")]
    if force or _newer(LIB, srcs):
        _run(
            [
                HIPCC,
                f"--offload-arch={ARCH}",
                "-O3",
                "-std=c++17",
                "-shared",
                "-fPIC",
                f"-I{INC}",
                "-o",
                LIB,
                srcs[0],
                srcs[1],
                "-L/opt/rocm/lib",
                "-lrccl",
                "-lrocprofiler-sdk-roctx",
                "-Wl,-rpath,/opt/rocm/lib",
            ]
        )
    return LIB


def build_host(force=False):
    import pybind11

    host = sorted(glob.glob(os.path.join(CSRC, "host", "*.cpp")))
    hdrs = sorted(glob.glob(os.path.join(CSRC, "host", "*.h")))
    bind = os.path.join(CSRC, "py", "bindings.cpp")
    if force or _newer(EXT, host + hdrs + [bind, LIB, os.path.join(INC, "openr_spf.h")]):
        _run(
            [
                os.environ.get("CXX", "g++"),
                "-O2",
                "-std=c++17",
                "-shared",
                "-fPIC",
                "-fvisibility=hidden",
                "-pthread",
                f"-I{INC}",
                f"-I{pybind11.get_include()}",
                f"-I{sysconfig.get_paths()['include']}",
                *host,
                bind,
                "-o",
                EXT,
                f"-L{HERE}",
                "-lopenr_spf",
                "-Wl,-rpath,$ORIGIN",
            ]
        )
    return EXT


def build(force=False):
    build_device(force)
    build_host(force)


if __name__ == "__main__":
    build(force="--force" in sys.argv)
