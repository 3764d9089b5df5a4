// PCIe rates of kernel loads and stores on pinned host memory (the host
// path's zero-copy reads and writes) beside SDMA copies.
//   hipcc --offload-arch=gfx950 -O3 -o build/pcie_bw tools/pcie_bw.hip && build/pcie_bw
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

#define CK(x)                                                       \
  do {                                                              \
    hipError_t e_ = (x);                                            \
    if (e_ != hipSuccess) {                                         \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));       \
      exit(1);                                                      \
    }                                                               \
  } while (0)

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

template <int U>
__global__ void copy_kernel(const u32x4 *__restrict__ src, u32x4 *__restrict__ dst, size_t n) {
  const size_t stride = (size_t)gridDim.x * blockDim.x;
  size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  for (; i + (U - 1) * stride < n; i += U * stride) {
    u32x4 v[U];
#pragma unroll
    for (int k = 0; k < U; k++) v[k] = __builtin_nontemporal_load(src + i + k * stride);
#pragma unroll
    for (int k = 0; k < U; k++) __builtin_nontemporal_store(v[k], dst + i + k * stride);
  }
  for (; i < n; i += stride) dst[i] = src[i];
}

int main() {
  const size_t bytes = (size_t)256 << 20, n = bytes / 16;
  void *h1, *h2, *d1, *d2;
  CK(hipHostMalloc(&h1, bytes, hipHostMallocDefault));
  CK(hipHostMalloc(&h2, bytes, hipHostMallocDefault));
  CK(hipMalloc(&d1, bytes));
  CK(hipMalloc(&d2, bytes));
  CK(hipMemset(d1, 1, bytes));
  for (size_t i = 0; i < bytes; i += 4096) ((char *)h1)[i] = 1;
  hipStream_t s1, s2;
  CK(hipStreamCreate(&s1));
  CK(hipStreamCreate(&s2));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  auto timed = [&](const char *what, auto fn) {
    fn();
    CK(hipDeviceSynchronize());
    float best = 1e9;
    for (int r = 0; r < 5; r++) {
      CK(hipEventRecord(e0, 0));
      fn();
      CK(hipEventRecord(e1, 0));
      CK(hipEventSynchronize(e1));
      CK(hipDeviceSynchronize());
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      best = ms < best ? ms : best;
    }
    printf("%-40s %7.2f GB/s\n", what, bytes / (best * 1e-3) / 1e9);
    fflush(stdout);
  };
  const int grids[] = {256, 1024, 4096};
  for (int g : grids) {
    char name[64];
    snprintf(name, sizeof name, "kernel read host  grid %d x256 U4", g);
    timed(name, [&] { copy_kernel<4><<<g, 256, 0, 0>>>((const u32x4 *)h1, (u32x4 *)d2, n); });
    snprintf(name, sizeof name, "kernel write host grid %d x256 U4", g);
    timed(name, [&] { copy_kernel<4><<<g, 256, 0, 0>>>((const u32x4 *)d1, (u32x4 *)h2, n); });
  }
  timed("kernel read host  grid 1024 x256 U8", [&] { copy_kernel<8><<<1024, 256, 0, 0>>>((const u32x4 *)h1, (u32x4 *)d2, n); });
  timed("kernel read+write (2 streams) 1024", [&] {
    copy_kernel<4><<<1024, 256, 0, s1>>>((const u32x4 *)h1, (u32x4 *)d2, n);
    copy_kernel<4><<<1024, 256, 0, s2>>>((const u32x4 *)d1, (u32x4 *)h2, n);
  });
  timed("sdma h2d", [&] { CK(hipMemcpyAsync(d2, h1, bytes, hipMemcpyHostToDevice, 0)); });
  timed("sdma d2h", [&] { CK(hipMemcpyAsync(h2, d1, bytes, hipMemcpyDeviceToHost, 0)); });
  timed("sdma h2d+d2h (2 streams)", [&] {
    CK(hipMemcpyAsync(d2, h1, bytes, hipMemcpyHostToDevice, s1));
    CK(hipMemcpyAsync(h2, d1, bytes, hipMemcpyDeviceToHost, s2));
  });
  return 0;
}
