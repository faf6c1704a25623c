set -o pipefail
B="python bench.py --no-wan --no-whatif --no-repair --no-cpu-baseline --steps 5 --warmup 2"
timeout -k 10 200 $B > gpurun_out/m_base.json 2>gpurun_out/m_base.err &&
GLIBC_TUNABLES=glibc.malloc.trim_threshold=1073741824:glibc.malloc.mmap_threshold=33554432 timeout -k 10 200 $B > gpurun_out/m_trim.json 2>gpurun_out/m_trim.err &&
GLIBC_TUNABLES=glibc.malloc.trim_threshold=1073741824:glibc.malloc.mmap_threshold=33554432:glibc.malloc.arena_max=1 timeout -k 10 200 $B > gpurun_out/m_arena1.json 2>gpurun_out/m_arena1.err &&
GLIBC_TUNABLES=glibc.malloc.trim_threshold=1073741824:glibc.malloc.mmap_threshold=33554432:glibc.malloc.tcache_count=4096 timeout -k 10 200 $B > gpurun_out/m_tcache.json 2>gpurun_out/m_tcache.err
