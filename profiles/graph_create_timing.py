import time, sys
import torch
torch.cuda.init()
sys.path.insert(0, '.')
from openr_amd import topologies as T, abi
topo = T.wan()
csr = topo.csr()
for i in range(4):
    t0 = time.perf_counter(); g = abi.Graph(csr, device=0); t1 = time.perf_counter()
    g.close(); t2 = time.perf_counter()
    print(f"create {1e3*(t1-t0):.1f} ms close {1e3*(t2-t1):.1f} ms", flush=True)
d, k = abi._graph_desc(csr, 0)
t0 = time.perf_counter(); d, k = abi._graph_desc(csr, 0); print(f"desc {1e3*(time.perf_counter()-t0):.2f} ms")
