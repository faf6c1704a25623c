"""Where spf_graph_create / spf_graph_destroy spend their time on the fabric
(the device graph LinkState::patchStructure recreates on every link flap):
OPENR_SPF_CREATE_TIMING=1 prints the create phases; destroy is timed here.

  OPENR_SPF_CREATE_TIMING=1 python profiles/graph_create_probe.py
"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch

    torch.cuda.init()
    from openr_amd import abi
    from openr_amd import topologies as T

    csr = T.fabric(10000).csr()
    for i in range(4):
        t0 = time.perf_counter()
        g = abi.Graph(csr, device=0)
        t1 = time.perf_counter()
        g.close()
        t2 = time.perf_counter()
        print(f"create {1e3 * (t1 - t0):.2f} ms  destroy {1e3 * (t2 - t1):.2f} ms", file=sys.stderr,
              flush=True)


if __name__ == "__main__":
    main()
