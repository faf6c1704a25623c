// FETCH_SIZE / WRITE_SIZE calibration for the access shapes of the
// next-hop kernel (spf_nh_levels_held_kernel): 4-byte loads per lane (a wave
// reads 256 contiguous bytes of a level row) and 16-byte stores of a
// contiguous 32-byte run per lane; plus the guide's 16-byte-per-lane
// streaming load as the reference shape.  Each kernel touches every byte of
// a 1 GiB buffer exactly once (4x the 256 MiB Infinity Cache), so the
// counters can be compared with a known byte count.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

constexpr size_t kBytes = 1ull << 30;

__global__ void read4(const uint32_t* p, size_t n, uint32_t* sink) {
  uint32_t acc = 0;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n;
       i += (size_t)gridDim.x * blockDim.x) {
    acc ^= p[i];
  }
  if (acc == 0x9E3779B9u) {
    sink[0] = acc; // practically never: keeps the loads
  }
}

__global__ void read16(const uint4* p, size_t n, uint32_t* sink) {
  uint32_t acc = 0;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n;
       i += (size_t)gridDim.x * blockDim.x) {
    const uint4 v = p[i];
    acc ^= v.x ^ v.y ^ v.z ^ v.w;
  }
  if (acc == 0x9E3779B9u) {
    sink[0] = acc;
  }
}

// lane L of a wave writes bytes [32 L, 32 L + 32) of the wave's 2 KB run as
// two 16-byte stores (the held kernel's Wm = 1 store)
__global__ void write32run(ulonglong2* p, size_t n_runs) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n_runs;
       i += (size_t)gridDim.x * blockDim.x) {
    p[2 * i] = make_ulonglong2(i, i + 1);
    p[2 * i + 1] = make_ulonglong2(i + 2, i + 3);
  }
}

#define CK(x)                                                          \
  do {                                                                 \
    hipError_t e_ = (x);                                               \
    if (e_ != hipSuccess) {                                            \
      std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));     \
      return 1;                                                        \
    }                                                                  \
  } while (0)

int main() {
  char* buf = nullptr;
  uint32_t* sink = nullptr;
  CK(hipMalloc(&buf, kBytes));
  CK(hipMalloc(&sink, 64));
  CK(hipMemset(buf, 1, kBytes));
  CK(hipDeviceSynchronize());
  const dim3 grid(4096), block(256);
  for (int rep = 0; rep < 3; ++rep) {
    hipLaunchKernelGGL(read4, grid, block, 0, 0, (const uint32_t*)buf, kBytes / 4, sink);
    hipLaunchKernelGGL(read16, grid, block, 0, 0, (const uint4*)buf, kBytes / 16, sink);
    hipLaunchKernelGGL(write32run, grid, block, 0, 0, (ulonglong2*)buf, kBytes / 32);
  }
  CK(hipGetLastError());
  CK(hipDeviceSynchronize());
  std::printf("bytes per kernel: %zu\n", kBytes);
  CK(hipFree(buf));
  CK(hipFree(sink));
  return 0;
}
