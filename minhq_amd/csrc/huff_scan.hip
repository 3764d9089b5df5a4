// huff_scan.hip -- exclusive scans that turn per-literal lengths into offset
// arrays (encode output offsets and decode capacities).  Three passes: block
// sums, one-block scan of the sums, apply.
#include <hip/hip_runtime.h>

#include "huff_common.h"
#include "huff_kernels.h"

namespace mhq {
namespace dev {

int g_cus = 0;

int device_cus() {
  if (g_cus == 0) {
    int d = 0, v = 0;
    if (hipGetDevice(&d) == hipSuccess &&
        hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, d) == hipSuccess && v > 0)
      g_cus = v;
    else
      g_cus = 256;
  }
  return g_cus;
}

}  // namespace dev

namespace {

constexpr int kScanBlock = 256;
constexpr int kScanItems = 8;
constexpr int kScanChunk = kScanBlock * kScanItems;

struct LenVal {  // enc_len -> (bytes, decode capacity)
  const uint32_t *len;
  __device__ inline void operator()(uint64_t i, uint64_t &a, uint64_t &b) const {
    const uint64_t v = len[i];
    a = v;
    b = (v * 8u) / 5u;
  }
};
struct CapVal {  // in_off -> decode capacity floor(8*len/5)
  const uint64_t *off;
  __device__ inline void operator()(uint64_t i, uint64_t &a, uint64_t &b) const {
    const uint64_t v = off[i + 1] - off[i];
    a = (v * 8u) / 5u;
    b = 0;
  }
};

__device__ inline void block_scan2(uint64_t &a, uint64_t &b, uint64_t *sa, uint64_t *sb, uint64_t &ta,
                                   uint64_t &tb) {
  // inclusive scan of (a,b) across the block; returns block totals
  const int tid = threadIdx.x;
  sa[tid] = a;
  sb[tid] = b;
  __syncthreads();
  for (int d = 1; d < kScanBlock; d <<= 1) {
    uint64_t xa = 0, xb = 0;
    if (tid >= d) {
      xa = sa[tid - d];
      xb = sb[tid - d];
    }
    __syncthreads();
    sa[tid] += xa;
    sb[tid] += xb;
    __syncthreads();
  }
  a = sa[tid];
  b = sb[tid];
  ta = sa[kScanBlock - 1];
  tb = sb[kScanBlock - 1];
  __syncthreads();
}

template <class F>
__global__ __launch_bounds__(kScanBlock) void scan_reduce_kernel(F f, uint64_t n, uint64_t *sums) {
  __shared__ uint64_t sa[kScanBlock], sb[kScanBlock];
  const uint64_t base = (uint64_t)blockIdx.x * kScanChunk + (uint64_t)threadIdx.x * kScanItems;
  uint64_t a = 0, b = 0;
  for (int k = 0; k < kScanItems; k++) {
    if (base + k < n) {
      uint64_t x, y;
      f(base + k, x, y);
      a += x;
      b += y;
    }
  }
  uint64_t ta, tb;
  block_scan2(a, b, sa, sb, ta, tb);
  if (threadIdx.x == 0) {
    sums[2 * blockIdx.x] = ta;
    sums[2 * blockIdx.x + 1] = tb;
  }
}

__global__ __launch_bounds__(kScanBlock) void scan_sums_kernel(uint64_t *sums, uint64_t nb) {
  __shared__ uint64_t sa[kScanBlock], sb[kScanBlock];
  uint64_t carry_a = 0, carry_b = 0;
  for (uint64_t base = 0; base < nb; base += kScanBlock) {
    const uint64_t i = base + threadIdx.x;
    uint64_t a = i < nb ? sums[2 * i] : 0, b = i < nb ? sums[2 * i + 1] : 0;
    const uint64_t ea = a, eb = b;
    uint64_t ta, tb;
    block_scan2(a, b, sa, sb, ta, tb);
    if (i < nb) {  // exclusive
      sums[2 * i] = carry_a + a - ea;
      sums[2 * i + 1] = carry_b + b - eb;
    }
    carry_a += ta;
    carry_b += tb;
  }
}

template <class F>
__global__ __launch_bounds__(kScanBlock) void scan_apply_kernel(F f, uint64_t n, const uint64_t *sums,
                                                                 uint64_t base_val, uint64_t *oa,
                                                                 uint64_t *ob) {
  __shared__ uint64_t sa[kScanBlock], sb[kScanBlock];
  const uint64_t base = (uint64_t)blockIdx.x * kScanChunk + (uint64_t)threadIdx.x * kScanItems;
  uint64_t xa[kScanItems], xb[kScanItems];
  uint64_t a = 0, b = 0;
#pragma unroll
  for (int k = 0; k < kScanItems; k++) {
    xa[k] = 0;
    xb[k] = 0;
    if (base + k < n) f(base + k, xa[k], xb[k]);
    a += xa[k];
    b += xb[k];
  }
  const uint64_t la = a, lb = b;
  uint64_t ta, tb;
  block_scan2(a, b, sa, sb, ta, tb);
  uint64_t ra = base_val + sums[2 * blockIdx.x] + a - la;
  uint64_t rb = base_val + sums[2 * blockIdx.x + 1] + b - lb;
#pragma unroll
  for (int k = 0; k < kScanItems; k++) {
    if (base + k <= n) {  // position n receives the grand total
      if (oa) oa[base + k] = ra;
      if (ob) ob[base + k] = rb;
    }
    ra += xa[k];
    rb += xb[k];
  }
}

template <class F>
hipError_t run_scan(F f, uint64_t n, uint64_t base, uint64_t *oa, uint64_t *ob, hipStream_t s) {
  // n+1 outputs; blocks cover indices 0..n inclusive
  const uint64_t nb = (n + 1 + kScanChunk - 1) / kScanChunk;
  uint64_t *sums = nullptr;
  hipError_t e = hipMallocAsync((void **)&sums, nb * 2 * sizeof(uint64_t), s);
  if (e != hipSuccess) return e;
  scan_reduce_kernel<F><<<dim3((unsigned)nb), dim3(kScanBlock), 0, s>>>(f, n, sums);
  scan_sums_kernel<<<dim3(1), dim3(kScanBlock), 0, s>>>(sums, nb);
  scan_apply_kernel<F><<<dim3((unsigned)nb), dim3(kScanBlock), 0, s>>>(f, n, sums, base, oa, ob);
  e = hipGetLastError();
  hipError_t e2 = hipFreeAsync(sums, s);
  return e != hipSuccess ? e : e2;
}

}  // namespace

hipError_t launch_offsets(const uint32_t *enc_len, uint64_t n, uint64_t base, uint64_t *out_off,
                          uint64_t *cap_off, hipStream_t s) {
  return run_scan(LenVal{enc_len}, n, base, out_off, cap_off, s);
}

hipError_t launch_capacity(const uint64_t *in_off, uint64_t n, uint64_t base, uint64_t *cap_off,
                           hipStream_t s) {
  return run_scan(CapVal{in_off}, n, base, cap_off, nullptr, s);
}

}  // namespace mhq
