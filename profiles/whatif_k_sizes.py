"""K sizes of the what-if repair on the configs[4] areas (host only, scipy):
for the first 600 sampled links of each area, the set K of nodes downstream
of the failed link's tight halves (spf_sssp_kernel whatif_repair_init's
closure over the baseline's tight usable edges from the border node).
Output: profiles/r04m/k_sizes.txt."""
import numpy as np, sys, collections
sys.path.insert(0,'/root/repo')
from openr_amd import topologies as TP
from scipy.sparse import csr_matrix
from scipy.sparse.csgraph import dijkstra
areas = list(TP.whatif_two_area())
for name, topo, links in areas:
    csr = topo.csr(); V=csr.num_nodes
    r,_ = topo.rank(); s = int(r[topo.names.index(TP.WHATIF_BORDER)])
    rp=csr.row_ptr.astype(np.int64); col=csr.col.astype(np.int64); w=csr.metric.astype(np.int64); lid=csr.link_id.astype(np.int64); ov=csr.overloaded
    A=csr_matrix((w,col,rp),shape=(V,V))
    d=dijkstra(A,indices=s).astype(np.int64)
    src_of=np.repeat(np.arange(V),np.diff(rp))
    tight=(d[src_of]+w==d[col])
    usable=np.ones(V,bool); usable[ov.astype(bool)]=False; usable[s]=True
    tight&=usable[src_of]
    ks=[]; kok=[]
    # adjacency of tight edges
    for l in links[:600]:
        es=np.flatnonzero(lid==l)
        seeds=[int(col[e]) for e in es if tight[e]]
        if not seeds: continue
        K=set(seeds); st=list(seeds)
        while st:
            u=st.pop()
            for e in range(rp[u],rp[u+1]):
                if tight[e] and lid[e]!=l and col[e] not in K:
                    K.add(int(col[e])); st.append(int(col[e]))
        ks.append(len(K))
    ks=np.array(ks)
    print(name, V, 'tight queries (of 600):', len(ks), 'K mean', ks.mean() if len(ks) else 0, 'median', np.median(ks) if len(ks) else 0, 'max', ks.max() if len(ks) else 0, 'p90', np.percentile(ks,90) if len(ks) else 0)
