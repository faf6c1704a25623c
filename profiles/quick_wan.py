"""WAN-100k delta-stepping variants on one GPU (runs on the GPU box).

Builds the config-3 WAN once, then for each variant (a set of OPENR_SPF_DSTEP_*
environment knobs, read by the engine at query creation / launch) runs a
distance-only query over N spread sources (plus the 32 golden sources of
tests/golden/wan100k_rows.json), reports the kernel time per SPF and checks
every row against the first variant (device-side compare) and the golden
rows against their committed sha256.

  python profiles/quick_wan.py [N] [variant ...]   variant = "K=V,K=V" or "base"
"""

import hashlib
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

KNOBS = ("OPENR_SPF_DSTEP_FINE", "OPENR_SPF_DSTEP_NORET", "OPENR_SPF_DSTEP_SHIFT",
         "OPENR_SPF_DSTEP_G", "OPENR_SPF_DSTEP_PACK", "OPENR_SPF_DSTEP_STATS",
         "OPENR_SPF_DSTEP_HASH", "OPENR_SPF_DSTEP_HCAP", "OPENR_SPF_DSTEP_HCHUNK",
         "OPENR_SPF_DSTEP_LDSROW", "OPENR_SPF_DSTEP_LSHIFT", "OPENR_SPF_DSTEP_LG",
         "OPENR_SPF_DSTEP_LPF")


def main():
    import torch

    from openr_amd import abi
    from openr_amd import topologies as TP

    n = int(sys.argv[1]) if len(sys.argv) > 1 else 8192
    variants = sys.argv[2:] or ["base"]
    torch.cuda.set_device(0)
    t = time.time()
    csr = TP.wan(100000, 1000000).csr()
    V = csr.num_nodes
    print(f"wan generated in {time.time() - t:.1f}s", flush=True)
    gold = json.load(open(os.path.join(ROOT, "tests", "golden", "wan100k_rows.json")))["rows"]
    srcs = sorted(set(range(0, V, max(1, V // n))) | {r["src"] for r in gold})
    srcs = np.asarray(srcs, dtype=np.uint32)
    pos = {int(s): i for i, s in enumerate(srcs)}
    g = abi.Graph(csr)
    base = None
    out = []
    for var in variants:
        for k in KNOBS:
            os.environ.pop(k, None)
        if var != "base":
            for kv in var.split(","):
                k, v = kv.split("=")
                os.environ["OPENR_SPF_DSTEP_" + k] = v
        q = g.query(srcs, 0)
        q.run()
        times = []
        for _ in range(2):
            q.run()
            times.append(q.elapsed_ms())
        rows = torch.empty((len(srcs), V), dtype=torch.int32, device="cuda:0")
        q.fetch_rows(0, len(srcs), rows.data_ptr(), V * 4, on_device=True)
        torch.cuda.synchronize()
        bad_gold = 0
        for r in gold:
            row = rows[pos[r["src"]]].cpu().numpy().view(np.uint32)
            bad_gold += hashlib.sha256(row.tobytes()).hexdigest() != r["sha256"]
        if base is None:
            base = rows
            diff = 0
        else:
            diff = int((rows != base).any(dim=1).sum())
            del rows
        ms = min(times)
        rec = {"variant": var, "kernel": q.kernel, "sources": len(srcs), "ms": round(ms, 2),
               "us_per_spf": round(1e3 * ms / len(srcs), 2), "rows_differing": diff,
               "golden_bad": bad_gold}
        print(json.dumps(rec), flush=True)
        out.append(rec)
        q.close()
    g.close()
    return out


if __name__ == "__main__":
    main()
