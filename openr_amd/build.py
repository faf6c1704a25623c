"""Build recipe for the MI355X SPF engine (in-tree, no JIT cache):

  libopenr_spf.so        the C ABI: hipcc --offload-arch=gfx950
                         csrc/spf_device.hip + csrc/spf_cluster.hip (RCCL, roctx)
  libopenr_decision.so   the host layer (LinkState / PrefixState / SpfSolver /
                         AllNodesRouteTable / PublicationIngest), g++
  decision_consumer      a standalone Decision-style C++ caller
  _openr_spf*.so         pybind11 bindings of the host layer (tests / bench),
                         linked to libopenr_decision.so + libopenr_spf.so

The first three commands are READ from INTEGRATION.md's "Build recipe"
block (the recipe a maintainer follows is the one this repo builds with).
Run `python -m openr_amd.build` (or __graft_entry__.build()).  Targets are
rebuilt only when a source is newer than the output.
"""

from __future__ import annotations

import glob
import os
import re
import shlex
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
DECISION = os.path.join(HERE, "libopenr_decision.so")
CONSUMER = os.path.join(HERE, "decision_consumer")
EXT = os.path.join(HERE, "_openr_spf" + sysconfig.get_config_var("EXT_SUFFIX"))


def recipe(out=HERE, repo=ROOT):
    """INTEGRATION.md's build recipe: {"engine" | "host" | "consumer": argv},
    with $REPO / $OUT substituted."""
    text = open(os.path.join(ROOT, "INTEGRATION.md")).read()
    head = "### Build recipe"
    block = text[text.index(head):].split("```sh\n", 1)[1].split("```", 1)[0]
    cmds, cur = {}, None
    for line in block.splitlines():
        m = re.match(r"# recipe: (\w+)", line)
        if m:
            cur = m.group(1)
            cmds[cur] = ""
            continue
        if cur is not None and line.strip() and not line.lstrip().startswith("#"):
            cmds[cur] += " " + line.strip().rstrip("\\")
    out_cmds = {}
    for k, v in cmds.items():
        v = v.replace("$REPO", repo).replace("$OUT", out)
        out_cmds[k] = shlex.split(v)
    if set(out_cmds) != {"engine", "host", "consumer"}:
        raise RuntimeError(f"INTEGRATION.md recipe has steps {sorted(out_cmds)}")
    return out_cmds


def _recipe_sources(argv):
    return [a for a in argv if a.endswith((".hip", ".cpp"))]


def _newer(target, sources):
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(s) > t for s in sources)


def _run(cmd):
    print("[openr_amd.build]", " ".join(cmd), flush=True)
    subprocess.run(cmd, check=True)


def build_device(force=False):
    cmd = recipe()["engine"]
    srcs = _recipe_sources(cmd) + [os.path.join(INC, "openr_spf.h"),
                                   os.path.join(CSRC, "host", "Parallel.h")]
    if force or _newer(LIB, srcs):
        _run(cmd)
    return LIB


def build_decision(force=False):
    """libopenr_decision.so (host layer) and the standalone consumer."""
    r = recipe()
    hdrs = sorted(glob.glob(os.path.join(CSRC, "host", "*.h"))) + [os.path.join(INC, "openr_spf.h")]
    # linked dynamically against the engine: a rebuilt libopenr_spf.so with the
    # same header needs no relink
    if force or _newer(DECISION, _recipe_sources(r["host"]) + hdrs):
        _run(r["host"])
    if force or _newer(CONSUMER, _recipe_sources(r["consumer"]) + hdrs + [DECISION]):
        _run(r["consumer"])
    return DECISION


def build_host(force=False):
    import pybind11

    hdrs = sorted(glob.glob(os.path.join(CSRC, "host", "*.h")))
    bind = os.path.join(CSRC, "py", "bindings.cpp")
    if force or _newer(EXT, hdrs + [bind, os.path.join(INC, "openr_spf.h")]):
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
                bind,
                "-o",
                EXT,
                f"-L{HERE}",
                "-lopenr_decision",
                "-lopenr_spf",
                "-Wl,-rpath,$ORIGIN",
            ]
        )
    return EXT


def build(force=False):
    build_device(force)
    build_decision(force)
    build_host(force)


if __name__ == "__main__":
    build(force="--force" in sys.argv)
