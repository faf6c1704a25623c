"""Build recipe for the CPU oracle (TEST INFRASTRUCTURE ONLY):
oracle/_oracle_ref*.so from oracle/ref_decision.cpp (g++, pybind11).

The reference itself is not built: its Decision path needs folly, fbthrift,
fb303 and glog, which this image does not have ("Oracle").
"""

from __future__ import annotations

import os
import subprocess
import sys
import sysconfig

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
SRC = os.path.join(HERE, "ref_decision.cpp")
DEPS = [
    SRC,
    os.path.join(HERE, "csr_spf.h"),
    os.path.join(ROOT, "openr_amd", "csrc", "host", "Types.h"),
    os.path.join(ROOT, "openr_amd", "csrc", "py", "convert.h"),
]
EXT = os.path.join(HERE, "_oracle_ref" + sysconfig.get_config_var("EXT_SUFFIX"))


def build(force=False):
    import pybind11

    if not force and os.path.exists(EXT):
        t = os.path.getmtime(EXT)
        if all(os.path.getmtime(d) <= t for d in DEPS):
            return EXT
    cmd = [
        os.environ.get("CXX", "g++"),
        "-O2",
        "-std=c++17",
        "-shared",
        "-fPIC",
        "-pthread",
        "-fvisibility=hidden",
        f"-I{pybind11.get_include()}",
        f"-I{sysconfig.get_paths()['include']}",
        SRC,
        "-o",
        EXT,
    ]
    print("[oracle.build]", " ".join(cmd), flush=True)
    subprocess.run(cmd, check=True)
    return EXT


if __name__ == "__main__":
    build(force="--force" in sys.argv)
