// huff_scan.hip -- exclusive scans that turn per-literal lengths into offset
// arrays (encode output offsets and decode capacities).
#include <hip/hip_runtime.h>

#include <algorithm>

#include <atomic>

#include "huff_common.h"
#include "huff_kernels.h"

namespace mhq {
namespace dev {

// CU count of the calling thread's current device, looked up once per device
// ordinal (host threads driving different devices call this concurrently).
constexpr int kMaxOrdinals = 64;
std::atomic<int> g_cus[kMaxOrdinals];

int device_cus() {
  int d = 0;
  if (hipGetDevice(&d) != hipSuccess || d < 0) d = 0;
  std::atomic<int> *slot = d < kMaxOrdinals ? &g_cus[d] : nullptr;
  int v = slot ? slot->load(std::memory_order_relaxed) : 0;
  if (v > 0) return v;
  if (hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, d) != hipSuccess || v <= 0) v = 256;
  if (slot) slot->store(v, std::memory_order_relaxed);
  return v;
}

}  // namespace dev

namespace {

using dev::kWave;
using dev::u32x4;

// Three linear passes over n+1 items (item n is 0, so position n receives the
// total):
//   1. block sums of (a, b) per chunk of kChunk items (or encode_len's sums
//      per kLenSumBlock literals, written by the sizing kernel itself);
//   2. those sums scanned in superblocks of kSup, each superblock's total
//      kept aside;
//   3. each chunk adds the superblock totals before it (one pair per kSup
//      sums) to its local prefix, then scans its chunk and writes.
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
#ifndef MHQ_SCAN_NT  // the apply pass's offsets leave as streaming stores (layout call north star 26.1 -> 24.1 us)
#define MHQ_SCAN_NT 1
#endif
#ifndef MHQ_SCAN_DIRECT_U  // the apply pass's direct-sum loads in flight per thread
#define MHQ_SCAN_DIRECT_U 16
#endif
constexpr int kDirectU = MHQ_SCAN_DIRECT_U;

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

struct PairVal {  // two independent u32 lengths -> two offset arrays (b null: one, the other sums 0)
  const uint32_t *a, *b;  // 16-B aligned
  uint64_t n;
  __device__ inline void load(uint64_t i0, uint64_t *x, uint64_t *y) const {
    if (i0 + kItems <= n) {
#pragma unroll
      for (int q = 0; q < kItems / 4; q++) {
        const u32x4 u = ((const u32x4 *)(a + i0))[q];
        const u32x4 v = b ? ((const u32x4 *)(b + i0))[q] : u32x4{0u, 0u, 0u, 0u};
        x[4 * q] = u.x; x[4 * q + 1] = u.y; x[4 * q + 2] = u.z; x[4 * q + 3] = u.w;
        y[4 * q] = v.x; y[4 * q + 1] = v.y; y[4 * q + 2] = v.z; y[4 * q + 3] = v.w;
      }
    } else {
#pragma unroll
      for (int k = 0; k < kItems; k++) {
        x[k] = i0 + k < n ? a[i0 + k] : 0u;
        y[k] = b && i0 + k < n ? b[i0 + k] : 0u;
      }
    }
  }
};

struct ReadCapVal {  // read_strings' framed strings -> output capacities (launch_read_caps_sums)
  const uint64_t *start, *next;
  const uint32_t *hend;
  const uint8_t *kind;
  uint64_t n;
  __device__ inline void load(uint64_t i0, uint64_t *x, uint64_t *y) const {
#pragma unroll
    for (int k = 0; k < kItems; k++) {
      const uint64_t i = i0 + k;
      uint64_t c = 0;
      if (i < n) {
        const uint32_t kd = kind[i] & 3u;
        const uint64_t st = start[i];
        if (kd == 1u)
          c = (uint64_t)(uint32_t)((uint64_t)(uint32_t)(hend[i] - (uint32_t)st) * 8u / 5u);
        else if (kd == 0u)
          c = (uint64_t)(uint32_t)(next[i] - st);
      }
      x[k] = c;
      y[k] = 0;
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

// Second pass, linear in the number of sums: superblock k (kSup consecutive
// (a, b) pairs of `sums`, pairs at or past ns read as zero) is scanned in
// place to exclusive prefixes within the superblock, and its total goes to
// sup[k].  sums must hold room for ns + 1 pairs: pair ns receives the
// superblock-local prefix of everything before it.
constexpr int kSup = kScanBlock;
__global__ __launch_bounds__(kScanBlock) void scan_sums_kernel(uint64_t *sums, uint64_t ns, uint64_t *sup) {
  __shared__ uint64_t sh[2 * kWaves];
  const int tid = threadIdx.x, lane = tid % kWave, wave = tid / kWave;
  const uint64_t j = (uint64_t)blockIdx.x * kSup + tid;
  const uint64_t a = j < ns ? sums[2 * j] : 0, b = j < ns ? sums[2 * j + 1] : 0;
  const uint64_t ia = wave_incl_scan(a, lane), ib = wave_incl_scan(b, lane);
  if (lane == kWave - 1) {
    sh[2 * wave] = ia;
    sh[2 * wave + 1] = ib;
  }
  __syncthreads();
  uint64_t ra = ia - a, rb = ib - b, ta = 0, tb = 0;
#pragma unroll
  for (int w = 0; w < kWaves; w++) {
    if (w < wave) {
      ra += sh[2 * w];
      rb += sh[2 * w + 1];
    }
    ta += sh[2 * w];
    tb += sh[2 * w + 1];
  }
  if (j <= ns) {
    sums[2 * j] = ra;
    sums[2 * j + 1] = rb;
  }
  if (tid == 0) {
    sup[2 * blockIdx.x] = ta;
    sup[2 * blockIdx.x + 1] = tb;
  }
}

// Third pass: chunk c's prefix is the sum of the superblock totals before its
// superblock (at most (n+1) / (kChunk * kSup / g) pairs, a few KB at 2^24
// items) plus the superblock-local prefix of its first pair, c*g, where `g`
// is the number of pairs per chunk: 1 for the reduce pass, kChunk /
// kLenSumBlock for encode_len's per-block sums.
// One chunk of the apply pass (chunk = blockIdx.x, or a chunk of a looping
// block's share).
template <class F>
__device__ __forceinline__ void scan_apply_chunk(const F &f, uint64_t n, const uint64_t *sums, const uint64_t *sup,
                                                 uint32_t g, uint64_t base, uint64_t *oa, uint64_t *ob,
                                                 uint64_t lim_a, uint64_t lim_b, uint64_t chunk) {
  __shared__ uint64_t sh[2 * kWaves];
  const int tid = threadIdx.x, lane = tid % kWave, wave = tid / kWave;
  // this chunk's items first: their loads are in flight during the prefix
  const uint64_t i0 = (uint64_t)chunk * kChunk + (uint64_t)tid * kItems;
  uint64_t a[kItems], b[kItems];
  f.load(i0, a, b);
  const uint64_t first = (uint64_t)chunk * g;  // this chunk's first pair
  uint64_t pa = 0, pb = 0;
  if (!sup) {
    // direct form (few sums, see direct_sums): the raw pairs before this
    // chunk's first, added up here; no second pass
    // (kDirectU loads per thread in flight at once: the pairs are L2 reads,
    // and one round trip per load was most of this kernel's time)
    typedef unsigned long long u64x2 __attribute__((ext_vector_type(2)));
    for (uint64_t j0 = tid; j0 < first; j0 += (uint64_t)kScanBlock * kDirectU) {
      u64x2 v[kDirectU];
#pragma unroll
      for (int u = 0; u < kDirectU; u++) {
        const uint64_t j = j0 + (uint64_t)u * kScanBlock;
        v[u] = j < first ? ((const u64x2 *)sums)[j] : u64x2{0ull, 0ull};
      }
#pragma unroll
      for (int u = 0; u < kDirectU; u++) {
        pa += v[u].x;
        pb += v[u].y;
      }
    }
    block_sum2(pa, pb, sh);
  } else {
    const uint64_t sb = first / kSup;
    for (uint64_t j = tid; j < sb; j += kScanBlock) {
      pa += sup[2 * j];
      pb += sup[2 * j + 1];
    }
    block_sum2(pa, pb, sh);
    pa += sums[2 * first];
    pb += sums[2 * first + 1];
  }
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
    xa[k] = min(ra, lim_a);  // offsets past a buffer's end become the end
    xb[k] = min(rb, lim_b);
    ra += a[k];
    rb += b[k];
  }
  typedef unsigned long long u64x2 __attribute__((ext_vector_type(2)));
  const uint64_t c0 = (uint64_t)chunk * kChunk;
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
#if MHQ_SCAN_NT
      if (oa) __builtin_nontemporal_store(u64x2{v0.x, v1.x}, (u64x2 *)(oa + c0 + j));
      if (ob) __builtin_nontemporal_store(u64x2{v0.y, v1.y}, (u64x2 *)(ob + c0 + j));
#else
      if (oa) *(u64x2 *)(oa + c0 + j) = u64x2{v0.x, v1.x};
      if (ob) *(u64x2 *)(ob + c0 + j) = u64x2{v0.y, v1.y};
#endif
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
__global__ __launch_bounds__(kScanBlock) void scan_apply_kernel(F f, uint64_t n, const uint64_t *sums,
                                                                 const uint64_t *sup, uint32_t g, uint64_t base,
                                                                 uint64_t *oa, uint64_t *ob, uint64_t lim_a = ~0ull,
                                                                 uint64_t lim_b = ~0ull,
                                                                 const uint64_t *gate = nullptr,
                                                                 uint64_t gen = 0) {
  // gated (read_strings): runs only when its producer stored this call's gen
  if (gate && __builtin_nontemporal_load(gate) != gen) return;
  scan_apply_chunk(f, n, sums, sup, g, base, oa, ob, lim_a, lim_b, blockIdx.x);
}

// The apply pass as a small grid looping over the chunks: for a gated pass
// that usually does nothing (read_strings' fallback layout), a few hundred
// workgroups that read the gate and end cost less than one per chunk.
template <class F>
__global__ __launch_bounds__(kScanBlock) void scan_apply_loop_kernel(F f, uint64_t n, const uint64_t *sums,
                                                                      const uint64_t *sup, uint32_t g, uint64_t base,
                                                                      uint64_t *oa, uint64_t *ob, uint64_t lim_a,
                                                                      uint64_t lim_b, const uint64_t *gate,
                                                                      uint64_t gen) {
  if (gate && __builtin_nontemporal_load(gate) != gen) return;
  const uint64_t nb = (n + 1 + kChunk - 1) / kChunk;
  for (uint64_t c = blockIdx.x; c < nb; c += gridDim.x) {
    scan_apply_chunk(f, n, sums, sup, g, base, oa, ob, lim_a, lim_b, c);
    __syncthreads();  // the chunk's LDS is read to the end before the next one's writes
  }
}

// Superblocks over ns pairs (pair ns included).
inline uint64_t sup_count(uint64_t ns) { return (ns + 1 + kSup - 1) / kSup; }

// The apply pass adds up the raw sums before its chunk itself (no second
// pass, one launch fewer) while that reads at most ~32 MB of L2 in all:
// nb blocks x ns pairs x 16 B / 2 (at 2^20 literals: the layout call's 513
// chunks over 4,096 encode_len sums; a scan's own 513 reduce sums).
#ifndef MHQ_SCAN_DIRECT_LOG2  // the direct form while nb x ns <= 2^this
#define MHQ_SCAN_DIRECT_LOG2 22
#endif
inline bool direct_sums(uint64_t nb, uint64_t ns) {
#ifdef MHQ_SCAN_NODIRECT  // timing builds: always the three passes
  return false;
#endif
  return nb * ns <= (1ull << MHQ_SCAN_DIRECT_LOG2);
}

inline size_t run_scan_bytes(uint64_t n) {
  const uint64_t nb = (n + 1 + kChunk - 1) / kChunk;
  return (size_t)(nb + 1 + sup_count(nb)) * 2 * sizeof(uint64_t);
}

// `scratch`: run_scan_bytes(n) bytes, or null for a hipMallocAsync of them on s.
template <class F>
hipError_t run_scan(F f, uint64_t n, uint64_t base, uint64_t *oa, uint64_t *ob, hipStream_t s,
                    void *scratch = nullptr, uint64_t lim_a = ~0ull, uint64_t lim_b = ~0ull) {
  // n+1 outputs; blocks cover indices 0..n inclusive
  const uint64_t nb = (n + 1 + kChunk - 1) / kChunk;
  const uint64_t nsup = sup_count(nb);
  uint64_t *sums = (uint64_t *)scratch;
  hipError_t e = hipSuccess;
  if (!sums && (e = hipMallocAsync((void **)&sums, run_scan_bytes(n), s)) != hipSuccess) return e;
  uint64_t *sup = sums + 2 * (nb + 1);
  scan_reduce_kernel<F><<<dim3((unsigned)nb), dim3(kScanBlock), 0, s>>>(f, n, sums);
  const bool direct = direct_sums(nb, nb);
  if (!direct) scan_sums_kernel<<<dim3((unsigned)nsup), dim3(kScanBlock), 0, s>>>(sums, nb, sup);
  scan_apply_kernel<F><<<dim3((unsigned)nb), dim3(kScanBlock), 0, s>>>(f, n, sums, direct ? nullptr : sup, 1u, base,
                                                                        oa, ob, lim_a, lim_b);
  e = hipGetLastError();
  if (scratch) return e;
  hipError_t e2 = hipFreeAsync(sums, s);
  return e != hipSuccess ? e : e2;
}

}  // namespace

size_t offsets_sums_scratch_bytes(uint64_t n) {
  const uint64_t ns = (n + kLenSumBlock - 1) / kLenSumBlock;
  return (size_t)(ns + 1 + sup_count(ns)) * 2 * sizeof(uint64_t);
}

size_t offsets_scratch_bytes(uint64_t n) { return run_scan_bytes(n); }

hipError_t launch_offsets(const uint32_t *enc_len, uint64_t n, uint64_t base, uint64_t *out_off,
                          uint64_t *cap_off, hipStream_t s, void *scratch) {
  return run_scan(LenVal{enc_len, n}, n, base, out_off, cap_off, s, scratch);
}

hipError_t launch_offsets_sums(const uint32_t *enc_len, uint64_t n, uint64_t *block_sums, uint64_t base,
                               uint64_t *out_off, uint64_t *cap_off, hipStream_t s) {
  static_assert(kChunk % kLenSumBlock == 0, "whole encode_len blocks per scan chunk");
  static_assert(kSup % (kChunk / kLenSumBlock) == 0, "no scan chunk straddles two superblocks");
  const uint64_t nb = (n + 1 + kChunk - 1) / kChunk;
  const uint64_t ns = (n + kLenSumBlock - 1) / kLenSumBlock;
  const uint64_t nsup = sup_count(ns);
  uint64_t *sup = block_sums + 2 * (ns + 1);
  const bool direct = direct_sums(nb, ns);
  if (!direct) scan_sums_kernel<<<dim3((unsigned)nsup), dim3(kScanBlock), 0, s>>>(block_sums, ns, sup);
  scan_apply_kernel<LenVal><<<dim3((unsigned)nb), dim3(kScanBlock), 0, s>>>(
      LenVal{enc_len, n}, n, block_sums, direct ? nullptr : sup, (uint32_t)(kChunk / kLenSumBlock), base, out_off,
      cap_off);
  return hipGetLastError();
}

size_t offsets_pair_scratch_bytes(uint64_t n) { return run_scan_bytes(n); }

hipError_t launch_offsets_pair_sums(const uint32_t *a, const uint32_t *b, uint64_t n, uint64_t *block_sums,
                                    uint64_t lim_a, uint64_t lim_b, uint64_t *oa, uint64_t *ob, hipStream_t s,
                                    const uint64_t *gate, uint64_t gen) {
  const uint64_t nb = (n + 1 + kChunk - 1) / kChunk;
  const uint64_t ns = (n + kLenSumBlock - 1) / kLenSumBlock;
  const uint64_t nsup = sup_count(ns);
  uint64_t *sup = block_sums + 2 * (ns + 1);
  const bool direct = direct_sums(nb, ns);
  if (!direct) scan_sums_kernel<<<dim3((unsigned)nsup), dim3(kScanBlock), 0, s>>>(block_sums, ns, sup);
  scan_apply_kernel<PairVal><<<dim3((unsigned)nb), dim3(kScanBlock), 0, s>>>(
      PairVal{a, b, n}, n, block_sums, direct ? nullptr : sup, (uint32_t)(kChunk / kLenSumBlock), 0, oa, ob, lim_a,
      lim_b, gate, gen);
  return hipGetLastError();
}

hipError_t launch_read_caps_sums(const uint64_t *start, const uint32_t *hend, const uint64_t *next,
                                 const uint8_t *kind, uint64_t n, uint64_t *block_sums, uint64_t lim,
                                 uint64_t *out_off, hipStream_t s, const uint64_t *gate, uint64_t gen) {
  const uint64_t nb = (n + 1 + kChunk - 1) / kChunk;
  const uint64_t ns = (n + kLenSumBlock - 1) / kLenSumBlock;
  const uint64_t nsup = sup_count(ns);
  uint64_t *sup = block_sums + 2 * (ns + 1);
  const bool direct = direct_sums(nb, ns);
  if (!direct) scan_sums_kernel<<<dim3((unsigned)nsup), dim3(kScanBlock), 0, s>>>(block_sums, ns, sup);
  // (gated, usually a no-op: a looping grid of at most 256 workgroups)
  scan_apply_loop_kernel<ReadCapVal><<<dim3((unsigned)std::min<uint64_t>(nb, 256)), dim3(kScanBlock), 0, s>>>(
      ReadCapVal{start, next, hend, kind, n}, n, block_sums, direct ? nullptr : sup, (uint32_t)(kChunk / kLenSumBlock),
      0, out_off, nullptr, lim, lim, gate, gen);
  return hipGetLastError();
}

hipError_t launch_offsets_pair(const uint32_t *a, const uint32_t *b, uint64_t n, uint64_t lim_a, uint64_t lim_b,
                               uint64_t *oa, uint64_t *ob, void *scratch, hipStream_t s) {
  return run_scan(PairVal{a, b, n}, n, 0, oa, ob, s, scratch, lim_a, lim_b);
}

hipError_t launch_capacity(const uint64_t *in_off, uint64_t n, uint64_t base, uint64_t *cap_off,
                           hipStream_t s) {
  return run_scan(CapVal{in_off, n}, n, base, cap_off, nullptr, s);
}

}  // namespace mhq
