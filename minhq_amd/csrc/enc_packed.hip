// enc_packed.hip -- the encode side of a batch in ONE launch: sizes
// (hc/io.go:157-172: the temp-buffer encode's length, ceil(code bits / 8)),
// their placement (the exclusive scans of enc_len and of the decode
// capacities floor(8 enc_len / 5)) and the encoded bytes (HuffmanCompressor
// Write + Pad, hc/huffman.go:23-37, io/bitio.go:72-149), where
// encode_len + the offsets scan + encode are three launches that read the
// plaintext twice.
//
// Structure: workgroup b owns literals [512 b, 512 b + 512), one per thread
// (the thread form of huff_encode.hip, for batches of short literals).
//   * its plaintext is staged once in LDS, sorted by length, sized
//     (encode_one without output) and block-scanned into range-relative
//     offsets;
//   * the range's totals are published (agent-scope atomic stores, tagged
//     with the call), and a decoupled look-back adds up the predecessors'
//     totals -- each window of 512 predecessors is read in one round trip and
//     stops at the nearest published inclusive prefix -- then the range
//     publishes its own inclusive prefix;
//   * enc_len, out_off and cap_off are written, and the staged plaintext is
//     encoded into the zeroed output staging at the range's real alignment
//     and stored with aligned 16-B stores.
// A range whose plaintext or output exceeds the staging slices (a long
// literal among short ones) is sized and encoded by one thread per literal
// straight from global memory.  The look-back slots live in a buffer kept
// per caller stream for look-backs only (mhq_api.cpp), so a slot holds this
// call's tag or an earlier call's, never another entry point's data; a
// workgroup only waits for lower-numbered ones, which the dispatcher started
// first, so the grid need not be resident at once.
#include <hip/hip_runtime.h>

#include "huff_encode_dev.h"

namespace mhq {
namespace {

using namespace dev;

struct alignas(16) PackSmem {
  uint2 code[256];                  // (code right-justified, length)
  uint32_t in_w[kInCap / 4 + 4];    // plaintext, natural byte order
  uint32_t out_w[kOutCap / 4 + 4];  // output staging (global alignment, zero-filled)
  uint32_t rec[kT + 1];             // literal boundaries: input byte index from the 16-B aligned start
  uint32_t rel[kT];                 // by literal: enc_len, then its range-relative output offset
  uint16_t order[kT];               // literals by ascending plaintext length
  uint32_t hist[kBuckets];
  uint32_t wsum[2][kT / kWave];     // per-wave totals of enc_len and capacity
  uint32_t lb_stop[2];              // look-back: nearest inclusive prefix in the window (enc, cap)
  unsigned long long lb_sum[2];     // look-back: the window's sums (enc, cap)
};

struct PackArgs {
  const uint8_t *in;
  const uint64_t *in_off;
  uint64_t in_bias, n, base;
  uint32_t *enc_len;
  uint64_t *out_off, *cap_off;  // cap_off may be null
  uint8_t *out;
  uint64_t out_cap;
  uint64_t *slots;  // 2 per workgroup: enc and capacity, pack_slot()
  uint32_t tag;     // the call's look-back tag: 30 bits, never 0
};

// A look-back slot: [63:34] the call's tag, [33:32] 1 aggregate / 2
// inclusive prefix, [31:0] the value (the caller keeps batches under 2^29
// plaintext bytes, so every sum of encoded bytes or capacities is < 2^32).
__device__ __forceinline__ uint64_t pack_slot(uint32_t tag, uint32_t flag, uint32_t v) {
  return (uint64_t)tag << 34 | (uint64_t)flag << 32 | v;
}

// Sum of v over the workgroup, added to *dst (LDS, zeroed before the call).
__device__ __forceinline__ void wg_add(unsigned long long *dst, uint64_t v) {
#pragma unroll
  for (int d = 1; d < kWave; d <<= 1) v += __shfl_xor((unsigned long long)v, d);
  if (threadIdx.x % kWave == 0 && v) atomicAdd(dst, (unsigned long long)v);
}

// Totals (enc, cap) of workgroups [0, b): windows of kT predecessors, each
// read in one round trip (spinning on slots not yet published), summed down
// to the nearest inclusive prefix of each quantity.
__device__ void look_back(const PackArgs &a, PackSmem &sm, uint32_t b, uint64_t &se, uint64_t &sc) {
  const uint32_t tid = threadIdx.x;
  se = sc = 0;
  bool de = false, dc = false;  // (uniform)
  for (int64_t hi = (int64_t)b - 1; hi >= 0 && !(de && dc); hi -= kT) {
    const int64_t g = hi - (int64_t)tid;
    uint64_t ve = 0, vc = 0;
    if (g >= 0) {
      for (;;) {
        ve = __hip_atomic_load((unsigned long long *)a.slots + 2 * g, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        vc = __hip_atomic_load((unsigned long long *)a.slots + 2 * g + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if ((uint32_t)(ve >> 34) == a.tag && (uint32_t)(vc >> 34) == a.tag) break;
        __builtin_amdgcn_s_sleep(1);
      }
    }
    if (tid == 0) {
      sm.lb_stop[0] = sm.lb_stop[1] = kT;
      sm.lb_sum[0] = sm.lb_sum[1] = 0;
    }
    __syncthreads();
    if (g >= 0 && ((ve >> 32) & 3u) == 2u) atomicMin(&sm.lb_stop[0], tid);
    if (g >= 0 && ((vc >> 32) & 3u) == 2u) atomicMin(&sm.lb_stop[1], tid);
    __syncthreads();
    const uint32_t stop_e = sm.lb_stop[0], stop_c = sm.lb_stop[1];
    // the aggregates before the nearest inclusive prefix, and that prefix
    wg_add(&sm.lb_sum[0], (!de && g >= 0 && tid <= stop_e) ? (uint32_t)ve : 0u);
    wg_add(&sm.lb_sum[1], (!dc && g >= 0 && tid <= stop_c) ? (uint32_t)vc : 0u);
    __syncthreads();
    se += de ? 0u : sm.lb_sum[0];
    sc += dc ? 0u : sm.lb_sum[1];
    de = de || stop_e < (uint32_t)kT;
    dc = dc || stop_c < (uint32_t)kT;
    __syncthreads();  // the window's LDS words are read before the next window resets them
  }
}

// Code bits of global bytes [src, src + nbytes) (a range too large to stage).
__device__ uint64_t size_literal_global(const uint8_t *src, uint64_t nbytes, const uint2 *code) {
  uint64_t bits = 0;
  for (uint64_t i = 0; i < nbytes; i++) bits += code[src[i]].y;
  return bits;
}

__global__ __launch_bounds__(kT) __attribute__((amdgpu_waves_per_eu((kT / 64 * MHQ_ENC_BLOCKS + 3) / 4))) void encode_packed_kernel(
    PackArgs a, const uint32_t *__restrict__ g_code, const uint8_t *__restrict__ g_len) {
  __shared__ PackSmem sm;
  const uint32_t tid = threadIdx.x, lane = tid % kWave, wave = tid / kWave, b = blockIdx.x;
  const uint64_t n = a.n, L0 = (uint64_t)b * kT;  // (the grid is ceil(n / kT): L0 < n)
  const uint32_t cnt = (uint32_t)min((uint64_t)kT, n - L0);
  const uint64_t ib = uniform64(vload(a.in_off, L0)), ie = uniform64(vload(a.in_off, L0 + cnt));
  const uint64_t e_t = a.in_off[L0 + min(tid, cnt - 1u) + 1u];  // this thread's literal's end
  for (uint32_t i = tid; i < 256u; i += kT) sm.code[i] = make_uint2(g_code[i], g_len[i]);
  const uint8_t *ia = a.in + (ib - a.in_bias);
  const uint32_t idelta = (uint32_t)((uintptr_t)ia & 15u);
  const bool staged = (ie - ib) + idelta <= (uint64_t)kInCap;  // (uniform)
  if (staged) {
    const u32x4 *src = (const u32x4 *)(ia - idelta);
    // (nothing for an empty range: its aligned chunk may lie past the buffer)
    const uint32_t chunks = ie > ib ? (uint32_t)(((ie - ib) + idelta + 15u) >> 4) : 0u;
    for (uint32_t c = tid; c < chunks; c += kT)
      *(u32x4 *)(sm.in_w + 4u * c) = __builtin_nontemporal_load(src + c);  // aligned, holds a valid byte
    if (tid == 0) sm.rec[0] = idelta;
    if (tid < cnt) sm.rec[tid + 1] = (uint32_t)(e_t - ib) + idelta;
  }
  if (tid < kBuckets) sm.hist[tid] = 0;
  __syncthreads();
  // sizing: staged, in length order (the 64 literals of a wave alike)
  uint32_t lit = tid;
  if (staged) {
    uint32_t bk = 0, rk = 0;
    if (tid < cnt) {
      const uint32_t bytes = sm.rec[tid + 1] - sm.rec[tid];
      bk = bytes < 48u ? bytes : min(48u + ((bytes - 48u) >> 3), (uint32_t)kBuckets - 1u);
      rk = atomicAdd(&sm.hist[bk], 1u);
    }
    __syncthreads();
    if (wave == 0) {
      const uint32_t h = sm.hist[lane];
      sm.hist[lane] = wave_incl_scan(h) - h;
    }
    __syncthreads();
    if (tid < cnt) sm.order[sm.hist[bk] + rk] = (uint16_t)tid;
    __syncthreads();
    lit = tid < cnt ? sm.order[tid] : tid;
  }
  if (tid < cnt) {
    uint64_t bits;
    if (staged) {
      bits = encode_one<false>(sm, sm.rec[lit], sm.rec[lit + 1], 0u);
    } else {
      const uint64_t s0 = a.in_off[L0 + tid];
      bits = size_literal_global(a.in + (s0 - a.in_bias), e_t - s0, sm.code);
    }
    sm.rel[lit] = (uint32_t)((bits + 7u) >> 3);
  }
  __syncthreads();
  // the range's layout: exclusive scans of enc_len and capacity, in literal order
  const uint32_t v = tid < cnt ? sm.rel[tid] : 0u;
  const uint32_t c = (uint32_t)((uint64_t)v * 8u / 5u);
  const uint32_t ve = wave_incl_scan(v), vc = wave_incl_scan(c);
  if (lane == kWave - 1) {
    sm.wsum[0][wave] = ve;
    sm.wsum[1][wave] = vc;
  }
  __syncthreads();
  uint32_t be = 0, bc = 0, T = 0, C = 0;
#pragma unroll
  for (int w = 0; w < kT / kWave; w++) {
    be += w < (int)wave ? sm.wsum[0][w] : 0u;
    bc += w < (int)wave ? sm.wsum[1][w] : 0u;
    T += sm.wsum[0][w];
    C += sm.wsum[1][w];
  }
  const uint32_t rel_e = be + ve - v, rel_c = bc + vc - c;
  // publish the range's totals, add up the predecessors', publish the prefix
  if (tid == 0) {
    __hip_atomic_store((unsigned long long *)a.slots + 2 * b, pack_slot(a.tag, 1u, T), __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store((unsigned long long *)a.slots + 2 * b + 1, pack_slot(a.tag, 1u, C), __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
  }
  uint64_t base_e, base_c;
  look_back(a, sm, b, base_e, base_c);
  if (tid == 0) {
    __hip_atomic_store((unsigned long long *)a.slots + 2 * b, pack_slot(a.tag, 2u, (uint32_t)(base_e + T)),
                       __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store((unsigned long long *)a.slots + 2 * b + 1, pack_slot(a.tag, 2u, (uint32_t)(base_c + C)),
                       __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  if (tid < cnt) {
    __builtin_nontemporal_store(v, a.enc_len + L0 + tid);
    a.out_off[L0 + tid] = a.base + base_e + rel_e;
    if (a.cap_off) a.cap_off[L0 + tid] = a.base + base_c + rel_c;
    sm.rel[tid] = rel_e;
  }
  if (tid == 0 && L0 + cnt == n) {
    a.out_off[n] = a.base + base_e + T;
    if (a.cap_off) a.cap_off[n] = a.base + base_c + C;
  }
  // encode: the literals whose regions end inside out_cap
  const uint64_t fit_end = a.out_cap > base_e ? a.out_cap - base_e : 0u;  // range-relative bytes inside out
  uint8_t *oa = a.out + base_e;
  const uint32_t odelta = (uint32_t)((uintptr_t)oa & 15u);
  if (staged && T + odelta <= (uint32_t)kOutCap) {  // (uniform)
    for (uint32_t q = tid; q < (T + odelta + 15u) >> 4; q += kT) *(u32x4 *)(sm.out_w + 4u * q) = u32x4{0u, 0u, 0u, 0u};
    __syncthreads();  // zeroed; sm.rel holds the offsets
    if (tid < cnt) {
      const uint32_t r = sm.rel[lit], len = (lit + 1u < cnt ? sm.rel[lit + 1] : T) - r;
      if (len && r + len <= fit_end) encode_one<true>(sm, sm.rec[lit], sm.rec[lit + 1], odelta + r);
    }
    __syncthreads();
    store_out(oa - odelta, (const uint8_t *)sm.out_w, odelta, odelta + (uint32_t)min((uint64_t)T, fit_end), tid, kT);
  } else if (tid < cnt && v && rel_e + v <= fit_end) {
    const uint64_t s0 = a.in_off[L0 + tid];
    encode_literal_global<true>(a.in + (s0 - a.in_bias), e_t - s0, oa + rel_e, sm.code, nullptr);
  }
}

__global__ void set_base_kernel(uint64_t *out_off, uint64_t *cap_off, uint64_t base) {
  out_off[0] = base;
  if (cap_off) cap_off[0] = base;
}

}  // namespace

size_t encode_packed_slot_bytes(uint64_t n) { return 16u * ((n + kT - 1) / kT); }

hipError_t launch_encode_packed(const DevTables &t, const uint8_t *in, const uint64_t *in_off, uint64_t in_bias,
                                uint64_t n, uint64_t base, uint32_t *enc_len, uint64_t *out_off, uint64_t *cap_off,
                                uint8_t *out, uint64_t out_cap, uint64_t *slots, uint64_t gen, hipStream_t s) {
  if (n == 0) {
    set_base_kernel<<<1, 1, 0, s>>>(out_off, cap_off, base);
    return hipGetLastError();
  }
  const unsigned grid = (unsigned)((n + kT - 1) / kT);
  PackArgs a{in, in_off, in_bias, n, base, enc_len, out_off, cap_off, out, out_cap, slots,
             (uint32_t)(gen % 0x3fffffffull) + 1u};
  encode_packed_kernel<<<dim3(grid), dim3(kT), 0, s>>>(a, t.code, t.len);
  return hipGetLastError();
}

}  // namespace mhq
