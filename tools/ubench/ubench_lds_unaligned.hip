// ubench_lds_unaligned.hip -- can a 4-byte aligned address feed ds_read_b64 /
// ds_read_b128 on gfx950 (the decode's window reads two or three consecutive
// stream words at any word), and how fast are they against ds_read2_b32 on
// random per-lane addresses?
//
//   hipcc --offload-arch=gfx950 -O3 tools/ubench/ubench_lds_unaligned.hip -o /tmp/ubench_lds_unaligned
//
// Check: every lane reads words (k, k+1[, k+2, k+3]) at a random word k and
// compares them with the pattern.  Timing: chains of dependent random reads
// (the next address from the data read), 16 waves per CU, per variant.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#define CHECK(x)                                                                        \
  do {                                                                                  \
    hipError_t e_ = (x);                                                                \
    if (e_ != hipSuccess) {                                                             \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      exit(1);                                                                          \
    }                                                                                   \
  } while (0)

constexpr int kWords = 8192;  // 32 KiB of LDS
constexpr int kIters = 4096;

typedef __attribute__((address_space(3))) uint32_t lds_u32;

__device__ __forceinline__ uint32_t pat(uint32_t k) { return k * 2654435761u ^ 0x5bd1e995u; }

template <int V>
__global__ __launch_bounds__(1024) void kern(uint32_t *bad, unsigned long long *cyc, uint32_t *sink) {
  __shared__ uint32_t w[kWords + 8];
  for (uint32_t i = threadIdx.x; i < kWords + 8; i += blockDim.x) w[i] = pat(i);
  __syncthreads();
  uint32_t k = (threadIdx.x * 7919u + blockIdx.x * 104729u) % kWords;
  uint32_t acc = 0, errs = 0;
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < kIters; it++) {
    const uint32_t a = (uint32_t)(uintptr_t)(w + k);  // 4-byte aligned LDS address
    uint32_t x0, x1, x2 = 0, x3 = 0;
    if (V == 0) {  // two dword reads, one instruction
      uint64_t v;
      asm volatile("ds_read2_b32 %0, %1 offset1:1\n s_waitcnt lgkmcnt(0)" : "=v"(v) : "v"(a));
      x0 = (uint32_t)v;
      x1 = (uint32_t)(v >> 32);
    } else if (V == 1) {  // one 8-byte read at a 4-byte aligned address
      uint64_t v;
      asm volatile("ds_read_b64 %0, %1\n s_waitcnt lgkmcnt(0)" : "=v"(v) : "v"(a));
      x0 = (uint32_t)v;
      x1 = (uint32_t)(v >> 32);
    } else if (V == 2) {  // one 16-byte read at a 4-byte aligned address
      typedef unsigned int u4 __attribute__((ext_vector_type(4)));
      u4 v;
      asm volatile("ds_read_b128 %0, %1\n s_waitcnt lgkmcnt(0)" : "=v"(v) : "v"(a));
      x0 = v.x;
      x1 = v.y;
      x2 = v.z;
      x3 = v.w;
    } else {  // V == 3: ds_read2_b32 + ds_read_b32 (the decode's pair window, three words)
      uint64_t v;
      asm volatile("ds_read2_b32 %0, %2 offset1:1\n ds_read_b32 %1, %2 offset:8\n s_waitcnt lgkmcnt(0)"
                   : "=v"(v), "=v"(x2)
                   : "v"(a));
      x0 = (uint32_t)v;
      x1 = (uint32_t)(v >> 32);
    }
    errs += (x0 != pat(k)) + (x1 != pat(k + 1));
    if (V == 2) errs += (x2 != pat(k + 2)) + (x3 != pat(k + 3));
    if (V == 3) errs += (x2 != pat(k + 2));
    acc += x0 ^ x1 ^ x2 ^ x3;
    k = (k + ((x0 ^ x1) & 1023u) + 1u) % kWords;  // the next address depends on the data (a chain)
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  if (errs) atomicAdd(bad, errs);
  if (threadIdx.x == 0) atomicAdd(cyc, t1 - t0);
  if (acc == 0x12345678u) sink[0] = acc;
}

template <int V>
void run(const char *name, int cus) {
  uint32_t *bad, *sink;
  unsigned long long *cyc;
  CHECK(hipMalloc(&bad, 4));
  CHECK(hipMalloc(&cyc, 8));
  CHECK(hipMalloc(&sink, 4));
  CHECK(hipMemset(bad, 0, 4));
  CHECK(hipMemset(cyc, 0, 8));
  hipEvent_t a, b;
  CHECK(hipEventCreate(&a));
  CHECK(hipEventCreate(&b));
  kern<V><<<cus, 1024>>>(bad, cyc, sink);  // warm
  CHECK(hipDeviceSynchronize());
  CHECK(hipMemset(bad, 0, 4));
  CHECK(hipMemset(cyc, 0, 8));
  CHECK(hipEventRecord(a));
  kern<V><<<cus, 1024>>>(bad, cyc, sink);
  CHECK(hipEventRecord(b));
  CHECK(hipDeviceSynchronize());
  float ms;
  CHECK(hipEventElapsedTime(&ms, a, b));
  uint32_t hb;
  unsigned long long hc;
  CHECK(hipMemcpy(&hb, bad, 4, hipMemcpyDeviceToHost));
  CHECK(hipMemcpy(&hc, cyc, 8, hipMemcpyDeviceToHost));
  const double reads = (double)cus * 1024 / 64 * kIters;  // wave-instructions (chains)
  printf("%-28s errors %u  %.3f ms  %.2f ns per wave-read per CU  %.0f cycles per dependent read (wave 0s)\n", name, hb,
         ms, ms * 1e6 / (reads / cus), (double)hc / cus / kIters);
  CHECK(hipFree(bad));
  CHECK(hipFree(cyc));
  CHECK(hipFree(sink));
}

int main() {
  int dev = 0, cus = 0;
  CHECK(hipGetDevice(&dev));
  CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
  run<0>("ds_read2_b32 (2 words)", cus);
  run<1>("ds_read_b64 @4-aligned", cus);
  run<2>("ds_read_b128 @4-aligned", cus);
  run<3>("ds_read2_b32+b32 (3 words)", cus);
  return 0;
}
