"""Golden for BASELINE configs[2] (the 100k-node / 1M-link WAN, SURVEY §8(d)
row 3): the (reached, sum of distances, 0, mix) summary of EVERY one of the
100,000 sources, from oracle/csr_spf.h (int CSR, binary-heap Dijkstra in which
only the source or non-overloaded nodes relax, LinkState.cpp:806-880), so the
GPU test can pin every row of the all-sources table, not a sample.

Pinned before it is written:
  * row n0's sum equals the REFERENCE's runSpf checksum from the survey
    container (tests/golden/wan_anchors.json);
  * the 32 rows of tests/golden/wan100k_rows.json (sha256 of the uint32 row)
    recomputed here equal the committed digests, and their summaries equal
    the summaries this script writes for the same sources.

  mix = sum_v splitmix64((d[v] << 24) ^ v) over reached v (mod 2^64)

Run: python -m tests.golden.make_wan_allsources [threads]   (~10 min on 8 cores)
"""

import hashlib
import json
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

OUT = os.path.join(HERE, "wan100k_allsources.npz")


def main():
    from oracle import build as OB

    OB.build()
    from oracle import _oracle_ref as O
    from openr_amd import topologies as TP

    threads = int(sys.argv[1]) if len(sys.argv) > 1 else os.cpu_count()
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 100000
    t0 = time.time()
    csr = TP.wan(100000, 1000000).csr()
    V = csr.num_nodes
    args = (csr.row_ptr, csr.col, csr.metric.astype(np.uint64), csr.link_id, csr.overloaded)
    print(f"wan generated in {time.time() - t0:.1f}s", flush=True)
    # pins: the reference anchor and the 32 committed rows
    anchor = [a for a in json.load(open(os.path.join(HERE, "wan_anchors.json")))["anchors"]
              if a["V"] == 100000 and a["S"] == 1][0]
    gold = json.load(open(os.path.join(HERE, "wan100k_rows.json")))["rows"]
    gs = np.asarray([r["src"] for r in gold], dtype=np.uint32)
    rows = O.csr_spf_rows(*args, gs, True, threads)
    for r, row in zip(gold, rows):
        r32 = np.where(row == np.uint64(2**64 - 1), np.uint64(0xFFFFFFFF), row).astype(np.uint32)
        assert hashlib.sha256(r32.tobytes()).hexdigest() == r["sha256"], r["src"]
    S = np.zeros((n, 4), dtype=np.uint64)
    step = 4096
    for lo in range(0, n, step):
        src = np.arange(lo, min(n, lo + step), dtype=np.uint32)
        S[lo:lo + len(src)] = O.csr_spf_summary(*args, src, None, None, True, False, threads)
        print(f"{lo + len(src)} / {n} sources, {time.time() - t0:.0f}s", flush=True)
    assert int(S[0, 1]) == anchor["sum_dist"], "reference anchor of row n0"
    Sg = O.csr_spf_summary(*args, gs, None, None, True, False, threads)
    for i, s in enumerate(gs):
        if s < n:
            assert (S[s] == Sg[i]).all(), int(s)
    if n == V:
        np.savez_compressed(OUT, summary=S)
        print("wrote", OUT, flush=True)
    print(f"done in {time.time() - t0:.0f}s", flush=True)


if __name__ == "__main__":
    main()
