"""CPU checks of the drop-in boundary (no GPU, no compute calls):

  * libopenr_spf.so exists, loads, and exports every function that
    include/openr_spf.h declares — and nothing named spf_* that it does not;
  * the ctypes view (openr_amd.abi.EXPORTED_SYMBOLS) lists the same set;
  * the host extension links the engine library (no CPU SPF path in it);
  * the error-string entry point answers without a device.
"""

import os
import re
import subprocess

from openr_amd import abi

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HDR_DIR = os.path.join(ROOT, "include")


def _declared():
    names = set()
    for fn in os.listdir(HDR_DIR):
        if not fn.endswith(".h"):
            continue
        text = open(os.path.join(HDR_DIR, fn)).read()
        text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
        for m in re.finditer(r"\b(spf_[a-z0-9_]+)\s*\(", text):
            names.add(m.group(1))
    return names


def _exported(path):
    out = subprocess.run(
        ["nm", "-D", "--defined-only", path], check=True, capture_output=True, text=True
    ).stdout
    return {l.split()[-1] for l in out.splitlines() if " T " in l and l.split()[-1].startswith("spf_")}


def test_header_matches_exports():
    declared = _declared()
    assert declared, "no spf_* declarations found in include/*.h"
    exported = _exported(abi.LIB_PATH)
    assert declared == exported, (declared - exported, exported - declared)
    assert set(abi.EXPORTED_SYMBOLS) == declared


def test_library_loads_without_gpu():
    lib = abi.load()
    for s in abi.EXPORTED_SYMBOLS:
        assert hasattr(lib, s), s
    assert lib.spf_error_string(0).decode()
    assert lib.spf_error_string(-3).decode()


def test_host_extension_links_engine():
    import glob

    ext = glob.glob(os.path.join(ROOT, "openr_amd", "_openr_spf*.so"))
    assert ext, "host extension not built"
    out = subprocess.run(["ldd", ext[0]], check=True, capture_output=True, text=True).stdout
    assert "libopenr_spf.so" in out
    # the product never links the oracle
    assert "_oracle_ref" not in out
