// huff_scan.hip -- exclusive scans that turn per-literal lengths into offset
// arrays (encode output offsets and decode capacities).
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

using dev::kWave;
using dev::u32x4;

// Two passes over n+1 items (item n is 0, so position n receives the total):
//   1. block sums of (a, b) per chunk of kChunk items;
//   2. each block adds up the sums of the chunks before it (at most a few
//      thousand u64 pairs, read from L2), then scans its chunk and writes.
// A thread owns kItems consecutive items; waves combine with shuffles, the
// kWaves of a block through LDS.
constexpr int kScanBlock = 256;
#ifndef MHQ_SCAN_ITEMS  // items per thread (a multiple of 4)
#define MHQ_SCAN_ITEMS 8
#endif
constexpr int kItems = MHQ_SCAN_ITEMS;
static_assert(kItems % 4 == 0, "whole 16-B loads of lengths");
constexpr int kChunk = kScanBlock * kItems;
constexpr int kWaves = kScanBlock / kWave;

struct LenVal {  // enc_len -> (bytes, decode capacity)
  const uint32_t *len;
  uint64_t n;
  __device__ inline void load(uint64_t i0, uint64_t *a, uint64_t *b) const {
    uint32_t v[kItems];
    if (i0 + kItems <= n) {
      const u32x4 *p = (const u32x4 *)(len + i0);  // i0 is a multiple of kItems: 16-B aligned
#pragma unroll
      for (int q = 0; q < kItems / 4; q++) {
        const u32x4 x = p[q];
        v[4 * q] = x.x; v[4 * q + 1] = x.y; v[4 * q + 2] = x.z; v[4 * q + 3] = x.w;
      }
    } else {
#pragma unroll
      for (int k = 0; k < kItems; k++) v[k] = i0 + k < n ? len[i0 + k] : 0u;
    }
#pragma unroll
    for (int k = 0; k < kItems; k++) {
      a[k] = v[k];
      b[k] = ((uint64_t)v[k] * 8u) / 5u;
    }
  }
};
struct CapVal {  // in_off -> decode capacity floor(8*len/5)
  const uint64_t *off;
  uint64_t n;
  __device__ inline void load(uint64_t i0, uint64_t *a, uint64_t *b) const {
    uint64_t prev = i0 < n ? off[i0] : 0;
#pragma unroll
    for (int k = 0; k < kItems; k++) {
      const uint64_t i = i0 + k;
      const uint64_t next = i < n ? off[i + 1] : prev;
      a[k] = ((next - prev) * 8u) / 5u;
      b[k] = 0;
      prev = next;
    }
  }
};

__device__ inline uint64_t wave_sum(uint64_t x) {
#pragma unroll
  for (int d = 1; d < kWave; d <<= 1) x += __shfl_xor(x, d);
  return x;
}

__device__ inline uint64_t wave_incl_scan(uint64_t x, int lane) {
#pragma unroll
  for (int d = 1; d < kWave; d <<= 1) {
    const uint64_t y = __shfl_up(x, d);
    if (lane >= d) x += y;
  }
  return x;
}

// Block-wide sum of (a, b); every thread gets the result.
__device__ inline void block_sum2(uint64_t &a, uint64_t &b, uint64_t *sh) {
  const int tid = threadIdx.x, lane = tid % kWave, wave = tid / kWave;
  a = wave_sum(a);
  b = wave_sum(b);
  if (lane == 0) {
    sh[2 * wave] = a;
    sh[2 * wave + 1] = b;
  }
  __syncthreads();
  a = 0;
  b = 0;
#pragma unroll
  for (int w = 0; w < kWaves; w++) {
    a += sh[2 * w];
    b += sh[2 * w + 1];
  }
  __syncthreads();
}

template <class F>
__global__ __launch_bounds__(kScanBlock) void scan_reduce_kernel(F f, uint64_t n, uint64_t *sums) {
  __shared__ uint64_t sh[2 * kWaves];
  const uint64_t i0 = (uint64_t)blockIdx.x * kChunk + (uint64_t)threadIdx.x * kItems;
  uint64_t a[kItems], b[kItems];
  f.load(i0, a, b);
  uint64_t ta = 0, tb = 0;
#pragma unroll
  for (int k = 0; k < kItems; k++) {
    ta += a[k];
    tb += b[k];
  }
  block_sum2(ta, tb, sh);
  if (threadIdx.x == 0) {
    sums[2 * blockIdx.x] = ta;
    sums[2 * blockIdx.x + 1] = tb;
  }
}

template <class F>
// `sums` holds (a, b) pairs for consecutive groups of kChunk / g items: the
// reduce pass writes one per chunk (g = 1), encode_len one per block of
// kLenSumBlock literals (g = kChunk / kLenSumBlock).
__global__ __launch_bounds__(kScanBlock) void scan_apply_kernel(F f, uint64_t n, const uint64_t *sums, uint32_t g,
                                                                 uint64_t base, uint64_t *oa, uint64_t *ob) {
  __shared__ uint64_t sh[2 * kWaves];
  const int tid = threadIdx.x, lane = tid % kWave, wave = tid / kWave;
  // this chunk's items first: their loads are in flight during the prefix
  const uint64_t i0 = (uint64_t)blockIdx.x * kChunk + (uint64_t)tid * kItems;
  uint64_t a[kItems], b[kItems];
  f.load(i0, a, b);
  // prefix of the chunks before this one
  typedef unsigned long long u64x2 __attribute__((ext_vector_type(2)));
  const u64x2 *sp = (const u64x2 *)sums;
  // (batches of eight independent loads per thread: one L2 round trip per
  // batch, not per pair)
  uint64_t pa = 0, pb = 0;
  const uint32_t cnt = blockIdx.x * g;
  for (uint32_t j0 = 0; j0 < cnt; j0 += 8u * kScanBlock) {
    u64x2 v[8];
#pragma unroll
    for (int k = 0; k < 8; k++) {
      const uint32_t j = j0 + (uint32_t)k * kScanBlock + tid;
      v[k] = j < cnt ? sp[j] : u64x2{0ull, 0ull};
    }
#pragma unroll
    for (int k = 0; k < 8; k++) {
      pa += v[k].x;
      pb += v[k].y;
    }
  }
  block_sum2(pa, pb, sh);
  uint64_t ta = 0, tb = 0;
#pragma unroll
  for (int k = 0; k < kItems; k++) {
    ta += a[k];
    tb += b[k];
  }
  const uint64_t ia = wave_incl_scan(ta, lane), ib = wave_incl_scan(tb, lane);
  if (lane == kWave - 1) {
    sh[2 * wave] = ia;
    sh[2 * wave + 1] = ib;
  }
  __syncthreads();
  uint64_t ra = base + pa + ia - ta, rb = base + pb + ib - tb;
  for (int w = 0; w < wave; w++) {
    ra += sh[2 * w];
    rb += sh[2 * w + 1];
  }
  uint64_t xa[kItems], xb[kItems];
#pragma unroll
  for (int k = 0; k < kItems; k++) {
    xa[k] = ra;
    xb[k] = rb;
    ra += a[k];
    rb += b[k];
  }
  const uint64_t c0 = (uint64_t)blockIdx.x * kChunk;
  if (c0 + kChunk <= n + 1) {
    // a whole chunk: through LDS, so each wave-wide 16-B store covers 1 KiB
    // of consecutive offsets (stores straight from the owning threads touch
    // 64 lines each)
    __shared__ u64x2 st[kChunk];  // a's chunk in .x, b's in .y
#pragma unroll
    for (int k = 0; k < kItems; k++) st[tid * kItems + k] = u64x2{xa[k], xb[k]};
    __syncthreads();
#pragma unroll
    for (int k = 0; k < kItems / 2; k++) {
      const uint32_t j = 2u * ((uint32_t)tid + (uint32_t)k * kScanBlock);
      const u64x2 v0 = st[j], v1 = st[j + 1];
      if (oa) *(u64x2 *)(oa + c0 + j) = u64x2{v0.x, v1.x};
      if (ob) *(u64x2 *)(ob + c0 + j) = u64x2{v0.y, v1.y};
    }
  } else if (i0 + kItems <= n + 1) {  // a whole run of outputs: 16-B stores (i0 is a multiple of 8)
#pragma unroll
    for (int k = 0; k < kItems; k += 2) {
      if (oa) *(u64x2 *)(oa + i0 + k) = u64x2{xa[k], xa[k + 1]};
      if (ob) *(u64x2 *)(ob + i0 + k) = u64x2{xb[k], xb[k + 1]};
    }
  } else {
#pragma unroll
    for (int k = 0; k < kItems; k++) {
      if (i0 + k <= n) {
        if (oa) oa[i0 + k] = xa[k];
        if (ob) ob[i0 + k] = xb[k];
      }
    }
  }
}

template <class F>
hipError_t run_scan(F f, uint64_t n, uint64_t base, uint64_t *oa, uint64_t *ob, hipStream_t s) {
  // n+1 outputs; blocks cover indices 0..n inclusive
  const uint64_t nb = (n + 1 + kChunk - 1) / kChunk;
  uint64_t *sums = nullptr;
  hipError_t e = hipMallocAsync((void **)&sums, nb * 2 * sizeof(uint64_t), s);
  if (e != hipSuccess) return e;
  scan_reduce_kernel<F><<<dim3((unsigned)nb), dim3(kScanBlock), 0, s>>>(f, n, sums);
  scan_apply_kernel<F><<<dim3((unsigned)nb), dim3(kScanBlock), 0, s>>>(f, n, sums, 1u, base, oa, ob);
  e = hipGetLastError();
  hipError_t e2 = hipFreeAsync(sums, s);
  return e != hipSuccess ? e : e2;
}

}  // namespace

hipError_t launch_offsets(const uint32_t *enc_len, uint64_t n, uint64_t base, uint64_t *out_off,
                          uint64_t *cap_off, hipStream_t s) {
  return run_scan(LenVal{enc_len, n}, n, base, out_off, cap_off, s);
}

hipError_t launch_offsets_sums(const uint32_t *enc_len, uint64_t n, const uint64_t *block_sums, uint64_t base,
                               uint64_t *out_off, uint64_t *cap_off, hipStream_t s) {
  static_assert(kChunk % kLenSumBlock == 0, "whole encode_len blocks per scan chunk");
  const uint64_t nb = (n + 1 + kChunk - 1) / kChunk;
  scan_apply_kernel<LenVal><<<dim3((unsigned)nb), dim3(kScanBlock), 0, s>>>(LenVal{enc_len, n}, n, block_sums,
                                                                          (uint32_t)(kChunk / kLenSumBlock),
                                                                          base, out_off, cap_off);
  return hipGetLastError();
}

hipError_t launch_capacity(const uint64_t *in_off, uint64_t n, uint64_t base, uint64_t *cap_off,
                           hipStream_t s) {
  return run_scan(CapVal{in_off, n}, n, base, cap_off, nullptr, s);
}

}  // namespace mhq
