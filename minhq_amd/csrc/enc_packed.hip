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
//     totals -- kLbW windows of 64 predecessors are read per round trip, and
//     it stops at the nearest published inclusive prefix -- then the range
//     publishes its own inclusive prefix;
//   * enc_len, out_off and cap_off are written, and the staged plaintext is
//     encoded into the zeroed output staging at the range's real alignment
//     and stored with aligned 16-B stores.
// A range whose plaintext exceeds the staging (longer literals among short
// ones) is sized, then (after its look-back) encoded, in two halves staged one
// after the other; a staged range whose codes exceed the output staging
// (printable text) is encoded in two halves too.  A half that still
// overflows is sized or encoded by one thread per literal straight from
// global memory.
// The look-back slots live in a buffer kept
// per caller stream for look-backs only (mhq_api.cpp), so a slot holds this
// call's tag or an earlier call's, never another entry point's data; a
// workgroup only waits for lower-numbered ones, which the dispatcher started
// first, so the grid need not be resident at once.  First is per XCD,
// though: the dispatcher starts a launch's workgroups in order on each XCD,
// not across the chip, so with concurrent launches (several streams) a
// workgroup can be resident and polling while a predecessor waits for a
// slot on another XCD that other polling workgroups hold.  A predecessor
// still unpublished after MHQ_PK_HELP_POLLS polls is therefore sized by the
// polling workgroup itself from global memory: the look-back
// never depends on a workgroup being scheduled.
#include <hip/hip_runtime.h>

#include <cstdlib>

#include "huff_encode_dev.h"

namespace mhq {
namespace {

using namespace dev;

#ifdef MHQ_DIAG_PKTL  // diagnostic build: per-workgroup phase stamps (s_memrealtime, 100 MHz)
// by range: [0] start, [1] staged, [2] sorted, [3] sized, [4] scanned +
// published, [5] wave 0's encode done, [6] look-back done, [7] base barrier
// passed, [8] end
constexpr int kPkSlots = 16;
constexpr int kPkWgs = 8192;
__device__ unsigned long long g_pktl[kPkWgs * kPkSlots];
#define PKTL(r, slot, cond)                                                                        \
  do {                                                                                             \
    if ((cond) && (r) < (uint64_t)kPkWgs) g_pktl[(r) * kPkSlots + (slot)] = wall_clock64();         \
  } while (0)
#else
#define PKTL(r, slot, cond) \
  do {                      \
  } while (0)
#endif

#ifndef MHQ_PK_STG  // 1: the staging's loads all issued before its LDS stores (r05ay: config 2 -2 %)
#define MHQ_PK_STG 1
#endif
#ifndef MHQ_PK_GW  // 1: unstaged ranges read their literals as aligned dwords (size_literal_global, encode_literal_global)
#define MHQ_PK_GW 1
#endif
#ifndef MHQ_PK_SLEEP  // the look-back's back-off between polls (s_sleep units of 64 clocks)
#define MHQ_PK_SLEEP 2
#endif
#ifndef MHQ_PK_NT_OFF  // 1: out_off / cap_off as streaming stores (r05bk: -2 to -4 %)
#define MHQ_PK_NT_OFF 1
#endif
#ifndef MHQ_PK_SORT  // 1: a range's literals sized and encoded in length order (the waves' lanes alike)
#define MHQ_PK_SORT 1
#endif
// Shapes of the kernel, by the batch's mean literal (launch_encode_packed):
// four resident workgroups per CU with 20,224-B plaintext and 15,360-B output
// staging (r05ax: config 2 -10 %, north star -7 %), ranges of kT literals
// while such a range fits the staging and of kShortR = 448 above that, to the
// packed route's 40-B bound (r05bh: -4 to -5 % against three workgroups with
// 24 / 20 KB and 512-literal ranges; a range that overflowed the staging then
// took the per-literal global path: a 40-B mean in 512-literal ranges at four
// ran 4.8x slower, r05bb; such ranges now go in staged halves, r06z).  The three-workgroup shape remains for means past
// 42.9 B (none on the packed route) and MHQ_PK_SHORT_R=0 builds.
#ifndef MHQ_PK_FOUR_RANGE_BYTES  // the four-workgroup shape up to this mean range of kT literals (bytes)
#define MHQ_PK_FOUR_RANGE_BYTES 19200
#endif
#ifndef MHQ_PK_LBW  // look-back windows of 64 predecessors read per round trip (r06: 3, 4 costs more with the stuck exit)
#define MHQ_PK_LBW 3
#endif
constexpr int kLbW = MHQ_PK_LBW;

template <int kB>
struct PkShape {
  static constexpr int kIn = kB >= 4 ? 20224 : kInCap;    // plaintext staging (bytes)
  static constexpr int kOut = kB >= 4 ? 15360 : kOutCap;  // output staging (bytes)
};

template <int kB>
struct alignas(16) PackSmem {
  static constexpr int kPkIn = PkShape<kB>::kIn, kPkOut = PkShape<kB>::kOut;
  uint2 code[256];                  // (code right-justified, length)
  uint32_t in_w[kPkIn / 4 + 4];     // plaintext, natural byte order
  union alignas(16) {
    uint32_t out_w[kPkOut / 4 + 4];  // output staging (global alignment, zero-filled)
    struct {                         // the length sort, done before the staging is zeroed
      uint16_t order[kT];            // literals by ascending plaintext length
      uint32_t hist[kBuckets];
    };
  };
  uint16_t rec[kT + 1];             // literal boundaries: input byte index from the 16-B aligned start
  uint32_t rel[kT];                 // by literal: enc_len, then its range-relative output offset
  uint32_t wsum[2][kT / kWave];     // per-wave totals of enc_len and capacity
  uint64_t base[2];                 // the range's place: enc and capacity bytes before it
  uint64_t stuck;                   // a predecessor range look_back found unpublished too long, or ~0
  static_assert(kPkIn + 16 < 65536, "rec holds 16-bit input indices");
  static_assert(sizeof(uint16_t) * kT + sizeof(uint32_t) * kBuckets <= sizeof(uint32_t) * (kPkOut / 4 + 4),
                "sort in staging");
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
  uint32_t R;       // literals per range: kT, or kShortR (launch_encode_packed)
  uint64_t in_bytes;  // the caller's in_off[n] - in_off[0], verified by every workgroup
  uint32_t help_polls;  // polls of a predecessor's slot before the polling wave sizes its range itself
};

// A look-back slot: [63:34] the call's tag, [33:32] 1 aggregate / 2
// inclusive prefix, [31:0] the value (the caller keeps batches under 2^29
// plaintext bytes, so every sum of encoded bytes or capacities is < 2^32).
__device__ __forceinline__ uint64_t pack_slot(uint32_t tag, uint32_t flag, uint32_t v) {
  return (uint64_t)tag << 34 | (uint64_t)flag << 32 | v;
}

// Sum of v over the 64 lanes of a wave (every lane gets it).
__device__ __forceinline__ uint64_t wave_sum64(uint64_t v) {
#pragma unroll
  for (int d = 1; d < kWave; d <<= 1) v += __shfl_xor((unsigned long long)v, d);
  return v;
}

// Sum of a u32 over the 64 lanes of a full wave, in DPP moves (no LDS round
// trips, unlike the shuffles of wave_sum64).
__device__ __forceinline__ uint32_t wave_sum32(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_readlane((int)wave_incl_scan(v), kWave - 1);
}

// Totals (enc, cap) of workgroups [0, b), by ONE wave: lane l reads the
// slots of workgroups b - 1 - l - 64 k (k < kLbW windows at once, spinning
// until they carry the call's tag), a ballot per window finds the nearest
// inclusive prefix of each quantity, and the aggregates before it are added
// up with it; with none in the windows, their aggregates are added and the
// next kLbW windows are read.  (One wave per workgroup polls, no workgroup
// barrier; in a generation of ranges started together the nearest inclusive
// prefix can lie several windows back.)
// Returns false, with `stuck` one of them, when a predecessor's slots stay
// unpublished past a.help_polls polls (see the top).
__device__ bool look_back(const PackArgs &a, uint32_t b, uint32_t lane, uint64_t &se, uint64_t &sc,
                          uint64_t &stuck) {
  se = sc = 0;
  bool de = false, dc = false;  // (uniform over the wave)
  unsigned long long *sl = (unsigned long long *)a.slots;
  for (int64_t hi = (int64_t)b - 1; hi >= 0 && !(de && dc); hi -= (int64_t)kWave * kLbW) {
    uint64_t ve[kLbW], vc[kLbW];
#pragma unroll
    for (int k = 0; k < kLbW; k++) {
      const int64_t g = hi - (int64_t)kWave * k - (int64_t)lane;
      ve[k] = vc[k] = 0;
      if (g >= 0) {
        ve[k] = __hip_atomic_load(sl + 2 * g, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        vc[k] = __hip_atomic_load(sl + 2 * g + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
    }
#pragma unroll
    for (int k = 0; k < kLbW; k++) {
      const int64_t g = hi - (int64_t)kWave * k - (int64_t)lane;
      // polled as a wave (the poll count is scalar)
      uint32_t polls = 0;
      for (uint64_t m; (m = __ballot(g >= 0 && ((uint32_t)(ve[k] >> 34) != a.tag ||
                                                 (uint32_t)(vc[k] >> 34) != a.tag))) != 0;) {
        if (++polls > a.help_polls) {
          stuck = (uint64_t)(hi - (int64_t)kWave * k - (int64_t)__builtin_ctzll(m));
          return false;
        }
        if (MHQ_PK_SLEEP) __builtin_amdgcn_s_sleep(MHQ_PK_SLEEP);
        if (g >= 0 && ((uint32_t)(ve[k] >> 34) != a.tag || (uint32_t)(vc[k] >> 34) != a.tag)) {
          ve[k] = __hip_atomic_load(sl + 2 * g, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          vc[k] = __hip_atomic_load(sl + 2 * g + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
      }
    }
#pragma unroll
    for (int k = 0; k < kLbW; k++) {
      if (de && dc) break;
      const int64_t g = hi - (int64_t)kWave * k - (int64_t)lane;
      const uint64_t me = __ballot(g >= 0 && ((ve[k] >> 32) & 3u) == 2u);
      const uint64_t mc = __ballot(g >= 0 && ((vc[k] >> 32) & 3u) == 2u);
      const uint32_t stop_e = me ? (uint32_t)__builtin_ctzll(me) : (uint32_t)kWave;
      const uint32_t stop_c = mc ? (uint32_t)__builtin_ctzll(mc) : (uint32_t)kWave;
      // the aggregates before the nearest inclusive prefix, and that prefix
      // (u32 sums in DPP moves: every sum of a batch's totals is < 2^32, see
      // pack_slot; the 64-bit shuffle sums cost 72 LDS round trips a look-back:
      // north star -0.5 us, profiles/r06/r06y_packed_lookback_dpp.txt)
      const uint64_t xe = wave_sum32((!de && g >= 0 && lane <= stop_e) ? (uint32_t)ve[k] : 0u);
      const uint64_t xc = wave_sum32((!dc && g >= 0 && lane <= stop_c) ? (uint32_t)vc[k] : 0u);
      se += xe;
      sc += xc;
      de = de || stop_e < (uint32_t)kWave;
      dc = dc || stop_c < (uint32_t)kWave;
    }
  }
  return true;
}

// Global bytes [lo, hi) from o_al (16-B aligned) <- staging bytes
// [lo - shift, hi - shift): whole 16-B chunks as aligned stores of dwords
// realigned from the staging (v_alignbyte), the bytes of the partial end
// chunks one per thread (neighbours untouched).  lo >= shift.
__device__ __forceinline__ void store_out_shifted(uint8_t *o_al, const uint32_t *stage, uint32_t lo, uint32_t hi,
                                                  uint32_t shift, uint32_t tid, uint32_t nthreads) {
  if (hi <= lo) return;
  const uint32_t f0 = (lo + 15u) >> 4, f1 = hi >> 4;  // whole chunks [f0, f1)
  const uint32_t r = shift & 3u;
  for (uint32_t c = f0 + tid; c < f1; c += nthreads) {
    const uint32_t x = 16u * c - shift;  // the chunk's first staging byte
    const uint32_t w = x >> 2;
    uint32_t d[5];
#pragma unroll
    for (int k = 0; k < 5; k++) d[k] = stage[w + (uint32_t)k];
    u32x4 v;
    v.x = __builtin_amdgcn_alignbyte(d[1], d[0], (x & 3u));
    v.y = __builtin_amdgcn_alignbyte(d[2], d[1], (x & 3u));
    v.z = __builtin_amdgcn_alignbyte(d[3], d[2], (x & 3u));
    v.w = __builtin_amdgcn_alignbyte(d[4], d[3], (x & 3u));
    __builtin_nontemporal_store(v, (u32x4 *)(o_al + 16u * c));
  }
  (void)r;
  const uint32_t head_end = min(hi, f0 << 4), tail_start = max(head_end, f1 << 4);
  const uint32_t y = tid < 16u ? lo + tid : tail_start + tid - 16u;
  if (tid < 32u && y < (tid < 16u ? head_end : hi))
    o_al[y] = (uint8_t)(stage[(y - shift) >> 2] >> (8u * ((y - shift) & 3u)));
}

// Code bits of global bytes [src, src + nbytes) (a range too large to stage).
__device__ uint64_t size_literal_global(const uint8_t *src, uint64_t nbytes, const uint2 *code) {
  uint64_t bits = 0;
  const uint8_t *p = src, *e = src + nbytes;
#if MHQ_PK_GW
  // whole aligned dwords between a byte-wise head and tail
  for (; p < e && ((uintptr_t)p & 3u); p++) bits += code[*p].y;
  for (; p + 4 <= e; p += 4) {
    const uint32_t w = *(const uint32_t *)p;
    bits += code[w & 0xffu].y + code[(w >> 8) & 0xffu].y + code[(w >> 16) & 0xffu].y + code[w >> 24].y;
  }
#endif
  for (; p < e; p++) bits += code[*p].y;
  return bits;
}

// Stages the plaintext of literals [lo, hi) of the range at L0 (the pieces of
// a range over the staging): in_w from the 16-B aligned start, rec[lo..hi]
// their boundaries.  False, staging nothing, when the piece does not fit.
// (uniform)
template <int kPkIn, class SM>
__device__ __forceinline__ bool stage_piece(SM &sm, const PackArgs &a, uint64_t L0, uint32_t lo, uint32_t hi,
                                            uint32_t tid) {
  const uint64_t pb = uniform64(vload(a.in_off, L0 + lo)), pe = uniform64(vload(a.in_off, L0 + hi));
  const uint8_t *pa = a.in + (pb - a.in_bias);
  const uint32_t pd = (uint32_t)((uintptr_t)pa & 15u);
  if ((pe - pb) + pd > (uint64_t)kPkIn) return false;
  const u32x4 *src = (const u32x4 *)(pa - pd);
  const uint32_t chunks = pe > pb ? (uint32_t)(((pe - pb) + pd + 15u) >> 4) : 0u;
  constexpr int kSC = (kPkIn / 16 + kT - 1) / kT;
  u32x4 v4[kSC];
#pragma unroll
  for (int k = 0; k < kSC; k++) {
    const uint32_t c = tid + (uint32_t)kT * k;
    if (c < chunks) v4[k] = __builtin_nontemporal_load(src + c);  // aligned, holds a valid byte
  }
#pragma unroll
  for (int k = 0; k < kSC; k++) {
    const uint32_t c = tid + (uint32_t)kT * k;
    if (c < chunks) *(u32x4 *)(sm.in_w + 4u * c) = v4[k];
  }
  if (tid == 0) sm.rec[lo] = (uint16_t)pd;
  if (tid >= lo && tid < hi) sm.rec[tid + 1] = (uint16_t)((uint32_t)(a.in_off[L0 + tid + 1] - pb) + pd);
  return true;
}

template <int kB>
__global__ __launch_bounds__(kT) __attribute__((amdgpu_waves_per_eu((kT / 64 * kB + 3) / 4))) void encode_packed_kernel(
    PackArgs a, const uint32_t *__restrict__ g_code, const uint8_t *__restrict__ g_len) {
  __shared__ PackSmem<kB> sm;
  constexpr int kPkIn = PackSmem<kB>::kPkIn, kPkOut = PackSmem<kB>::kPkOut;
  const uint32_t tid = threadIdx.x, lane = tid % kWave, wave = tid / kWave, b = blockIdx.x;
  PKTL(b, 0, tid == 0);
  const uint64_t n = a.n, L0 = (uint64_t)b * a.R;  // (the grid is ceil(n / R): L0 < n)
  const uint32_t cnt = (uint32_t)min((uint64_t)a.R, n - L0);
  // The caller's in_bytes chose this path and bounds every look-back sum
  // (< 2^32): a batch whose offsets say otherwise is not encoded; out_off[n]
  // = UINT64_MAX tells the caller (include/mhq_huff.h).
  if (uniform64(vload(a.in_off, n)) - uniform64(vload(a.in_off, 0)) != a.in_bytes) {
    if (b == 0 && tid == 0) a.out_off[n] = ~0ull;
    return;
  }
  const uint64_t ib = uniform64(vload(a.in_off, L0)), ie = uniform64(vload(a.in_off, L0 + cnt));
  const uint64_t e_t = a.in_off[L0 + min(tid, cnt - 1u) + 1u];  // this thread's literal's end
  for (uint32_t i = tid; i < 256u; i += kT) sm.code[i] = make_uint2(g_code[i], g_len[i]);
  const uint8_t *ia = a.in + (ib - a.in_bias);
  const uint32_t idelta = (uint32_t)((uintptr_t)ia & 15u);
  const bool staged = (ie - ib) + idelta <= (uint64_t)kPkIn;  // (uniform)
  if (staged) {
    const u32x4 *src = (const u32x4 *)(ia - idelta);
    // (nothing for an empty range: its aligned chunk may lie past the buffer)
    const uint32_t chunks = ie > ib ? (uint32_t)(((ie - ib) + idelta + 15u) >> 4) : 0u;
#if MHQ_PK_STG
    // every load issued before the first LDS store (one HBM round trip)
    constexpr int kSC = (kPkIn / 16 + kT - 1) / kT;
    u32x4 v4[kSC];
#pragma unroll
    for (int k = 0; k < kSC; k++) {
      const uint32_t c = tid + (uint32_t)kT * k;
      if (c < chunks) v4[k] = __builtin_nontemporal_load(src + c);  // aligned, holds a valid byte
    }
#pragma unroll
    for (int k = 0; k < kSC; k++) {
      const uint32_t c = tid + (uint32_t)kT * k;
      if (c < chunks) *(u32x4 *)(sm.in_w + 4u * c) = v4[k];
    }
#else
    for (uint32_t c = tid; c < chunks; c += kT)
      *(u32x4 *)(sm.in_w + 4u * c) = __builtin_nontemporal_load(src + c);  // aligned, holds a valid byte
#endif
    if (tid == 0) sm.rec[0] = (uint16_t)idelta;
    if (tid < cnt) sm.rec[tid + 1] = (uint16_t)((uint32_t)(e_t - ib) + idelta);
  }
  if (tid < kBuckets) sm.hist[tid] = 0;
  __syncthreads();
  PKTL(b, 1, tid == 0);
  // sizing: staged, in length order (the 64 literals of a wave alike)
  uint32_t lit = tid;
  if (staged && MHQ_PK_SORT) {
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
  PKTL(b, 2, tid == 0);
  if (staged) {
    if (tid < cnt) sm.rel[lit] = (encode_one<false>(sm, sm.rec[lit], sm.rec[lit + 1], 0u) + 7u) >> 3;
  } else {
    // a range over the staging (long literals among short ones): its two
    // halves are staged one after the other; a half that still overflows is
    // sized a literal a thread from global memory
    for (uint32_t q = 0; q < 2u; q++) {
      const uint32_t lo = q ? cnt / 2u : 0u, hi = q ? cnt : cnt / 2u;
      const bool pf = stage_piece<kPkIn>(sm, a, L0, lo, hi, tid);
      __syncthreads();
      if (tid >= lo && tid < hi) {
        uint64_t bits;
        if (pf) {
          bits = encode_one<false>(sm, sm.rec[tid], sm.rec[tid + 1], 0u);
        } else {
          const uint64_t s0 = a.in_off[L0 + tid];
          bits = size_literal_global(a.in + (s0 - a.in_bias), e_t - s0, sm.code);
        }
        sm.rel[tid] = (uint32_t)((bits + 7u) >> 3);
      }
      __syncthreads();  // (the next half's staging overwrites in_w and rec)
    }
  }
  __syncthreads();
  PKTL(b, 3, tid == 0);
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
  // publish the range's totals at once, so that the ranges after it can
  // add them up while this one encodes
  if (tid == 0) {
    __hip_atomic_store((unsigned long long *)a.slots + 2 * b, pack_slot(a.tag, 1u, T), __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store((unsigned long long *)a.slots + 2 * b + 1, pack_slot(a.tag, 1u, C), __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
  }
  PKTL(b, 4, tid == 0);
  // encode into the staging at the range-relative offsets (the range's
  // place in the output is not known yet: the store below realigns)
  const bool staged_out = staged && T <= (uint32_t)kPkOut;  // (uniform)
  if (staged_out) {
    if (tid < cnt) sm.rel[tid] = rel_e;  // (every thread read its enc_len into v above)
    for (uint32_t q = tid; q < (T + 15u) >> 4; q += kT) *(u32x4 *)(sm.out_w + 4u * q) = u32x4{0u, 0u, 0u, 0u};
    __syncthreads();  // zeroed; sm.rel holds the offsets
    if (tid < cnt) {
      const uint32_t r = sm.rel[lit], len = (lit + 1u < cnt ? sm.rel[lit + 1] : T) - r;
      if (len) encode_one<true>(sm, sm.rec[lit], sm.rec[lit + 1], r);
    }
  }
  // the predecessors' totals (one wave), then this range's inclusive prefix
  for (;;) {
    if (wave == 0) {
      PKTL(b, 5, lane == 0);
      uint64_t se, sc, stuck = 0;
      const bool done = look_back(a, b, lane, se, sc, stuck);
      PKTL(b, 6, lane == 0);
      if (lane == 0) {
        sm.stuck = done ? ~0ull : stuck;
        if (done) {
          sm.base[0] = se;
          sm.base[1] = sc;
          __hip_atomic_store((unsigned long long *)a.slots + 2 * b, pack_slot(a.tag, 2u, (uint32_t)(se + T)),
                             __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          __hip_atomic_store((unsigned long long *)a.slots + 2 * b + 1, pack_slot(a.tag, 2u, (uint32_t)(sc + C)),
                             __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
      }
    }
    __syncthreads();  // the base; the staging complete
    const uint64_t g = uniform64(sm.stuck);
    if (g == ~0ull) break;
    // range g stayed unpublished (see the top): this workgroup sizes it, a
    // literal a thread, publishes its aggregate on its behalf -- the value
    // its own workgroup publishes too -- and looks back again
    const uint64_t Lg = g * a.R;
    const uint32_t cg = (uint32_t)min((uint64_t)a.R, n - Lg);
    uint32_t hv = 0;
    if (tid < cg) {  // (a plain byte loop: a rare path, kept small)
      uint32_t bits = 0;
      const uint8_t *q = a.in + (a.in_off[Lg + tid] - a.in_bias), *qe = a.in + (a.in_off[Lg + tid + 1] - a.in_bias);
      for (; q < qe; q++) bits += sm.code[*q].y;
      hv = (bits + 7u) >> 3;
    }
    const uint64_t hw = wave_sum64((uint64_t)hv | (uint64_t)((uint64_t)hv * 8u / 5u) << 32);
    if (lane == 0) {
      sm.wsum[0][wave] = (uint32_t)hw;
      sm.wsum[1][wave] = (uint32_t)(hw >> 32);
    }
    __syncthreads();
    if (tid == 0) {
      uint32_t te = 0, tc = 0;
#pragma unroll
      for (int w = 0; w < kT / kWave; w++) {
        te += sm.wsum[0][w];
        tc += sm.wsum[1][w];
      }
      __hip_atomic_store((unsigned long long *)a.slots + 2 * g, pack_slot(a.tag, 1u, te), __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store((unsigned long long *)a.slots + 2 * g + 1, pack_slot(a.tag, 1u, tc), __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_AGENT);
      __threadfence();
    }
    __syncthreads();
  }
  PKTL(b, 7, tid == 0);
  const uint64_t base_e = sm.base[0], base_c = sm.base[1];
  if (tid < cnt) {
    __builtin_nontemporal_store(v, a.enc_len + L0 + tid);
#if MHQ_PK_NT_OFF
    __builtin_nontemporal_store(a.base + base_e + rel_e, a.out_off + L0 + tid);
    if (a.cap_off) __builtin_nontemporal_store(a.base + base_c + rel_c, a.cap_off + L0 + tid);
#else
    a.out_off[L0 + tid] = a.base + base_e + rel_e;
    if (a.cap_off) a.cap_off[L0 + tid] = a.base + base_c + rel_c;
#endif
  }
  if (tid == 0 && L0 + cnt == n) {
    a.out_off[n] = a.base + base_e + T;
    if (a.cap_off) a.cap_off[n] = a.base + base_c + C;
  }
  // the codes: out + base_e on (never past out_cap, which the caller sized
  // for the worst case: mhq_huff_encode_packed_dev)
  const uint64_t room = a.out_cap > base_e ? a.out_cap - base_e : 0u;
  uint8_t *oa = a.out + base_e;
  const uint32_t odelta = (uint32_t)((uintptr_t)oa & 15u);
  if (staged_out) {
    store_out_shifted(oa - odelta, sm.out_w, odelta, odelta + (uint32_t)min((uint64_t)T, room), odelta, tid, kT);
  } else {
    // in two halves, each encoded into the output staging and stored at its
    // place (rel_e of its first literal): a staged range whose codes overflow
    // the output staging (printable text: ~1 code byte a byte), or a range
    // over the plaintext staging, whose halves are staged again here; a half
    // whose plaintext or codes overflow is encoded a literal a thread from
    // global memory
    if (tid < cnt) sm.rel[tid] = rel_e;
    for (uint32_t q = 0; q < 2u; q++) {
      const uint32_t lo = q ? cnt / 2u : 0u, hi = q ? cnt : cnt / 2u;
      __syncthreads();  // sm.rel complete; the previous half stored
      const uint32_t r0 = __builtin_amdgcn_readfirstlane(lo < cnt ? sm.rel[lo] : T);
      const uint32_t r1 = __builtin_amdgcn_readfirstlane(hi < cnt ? sm.rel[hi] : T);
      const uint32_t tq = r1 - r0;
      const bool pf = tq <= (uint32_t)kPkOut && (staged || stage_piece<kPkIn>(sm, a, L0, lo, hi, tid));
      if (pf)
        for (uint32_t c = tid; c < (tq + 15u) >> 4; c += kT) *(u32x4 *)(sm.out_w + 4u * c) = u32x4{0u, 0u, 0u, 0u};
      __syncthreads();
      if (tid >= lo && tid < hi && v) {
        if (pf) {
          encode_one<true>(sm, sm.rec[tid], sm.rec[tid + 1], rel_e - r0);
        } else if (rel_e + v <= room) {
          const uint64_t s0 = a.in_off[L0 + tid], e0 = a.in_off[L0 + tid + 1];
          encode_literal_global<true>(a.in + (s0 - a.in_bias), e0 - s0, oa + rel_e, sm.code, nullptr);
        }
      }
      __syncthreads();
      if (pf) {
        uint8_t *og = oa + r0;
        const uint32_t od = (uint32_t)((uintptr_t)og & 15u);
        const uint64_t rq = room > r0 ? room - r0 : 0u;
        store_out_shifted(og - od, sm.out_w, od, od + (uint32_t)min((uint64_t)tq, rq), od, tid, kT);
      }
    }
  }
  PKTL(b, 8, tid == 0);
}

__global__ void set_base_kernel(uint64_t *out_off, uint64_t *cap_off, uint64_t base) {
  out_off[0] = base;
  if (cap_off) cap_off[0] = base;
}

}  // namespace

#ifdef MHQ_DIAG_PKTL
extern "C" int mhq_diag_pktimeline(unsigned long long *out, int n) {
  const int m = n < kPkWgs * kPkSlots ? n : kPkWgs * kPkSlots;
  hipDeviceSynchronize();
  const int rc = hipMemcpyFromSymbol(out, HIP_SYMBOL(g_pktl), m * sizeof(unsigned long long)) == hipSuccess ? kPkSlots : -1;
  static unsigned long long zeros[kPkWgs * kPkSlots];
  hipMemcpyToSymbol(HIP_SYMBOL(g_pktl), zeros, sizeof(zeros));
  return rc;
}
#endif

#ifndef MHQ_PK_SHORT_R  // the four-workgroup shape's shorter ranges for means past MHQ_PK_FOUR_RANGE_BYTES / kT (0: none)
#define MHQ_PK_SHORT_R 448
#endif
constexpr uint32_t kShortR = MHQ_PK_SHORT_R ? MHQ_PK_SHORT_R : kT;
static_assert(kShortR <= (uint32_t)kT && kShortR % kWave == 0, "range size");

// (for either range size)
size_t encode_packed_slot_bytes(uint64_t n) { return 16u * ((n + kShortR - 1) / kShortR); }

#ifndef MHQ_PK_HELP_POLLS  // ~100 us of polls (a generation of ranges publishes within ~20 us)
#define MHQ_PK_HELP_POLLS 400
#endif
// The look-backs' patience (the packed encode's, read_fallback_kernel's):
// MHQ_PK_HELP_POLLS, or the environment's, read once (tests force the help
// with 0).
uint32_t lookback_help_polls() {
  static const uint32_t t = [] {
    const char *e = getenv("MHQ_PK_HELP_POLLS");
    return e ? (uint32_t)strtoul(e, nullptr, 10) : (uint32_t)MHQ_PK_HELP_POLLS;
  }();
  return t;
}

hipError_t launch_encode_packed(const DevTables &t, const uint8_t *in, const uint64_t *in_off, uint64_t in_bias,
                                uint64_t n, uint64_t base, uint32_t *enc_len, uint64_t *out_off, uint64_t *cap_off,
                                uint8_t *out, uint64_t out_cap, uint64_t *slots, uint32_t tag, hipStream_t s,
                                uint64_t in_bytes) {
  if (n == 0) {
    set_base_kernel<<<1, 1, 0, s>>>(out_off, cap_off, base);
    return hipGetLastError();
  }
  // four workgroups per CU while a mean range fits MHQ_PK_FOUR_RANGE_BYTES:
  // ranges of kT literals, or of kShortR for a larger mean; three otherwise
  const uint64_t fit = (uint64_t)MHQ_PK_FOUR_RANGE_BYTES * n;
  const bool four = in_bytes * (uint64_t)kShortR <= fit;
  const uint32_t R = four && in_bytes * (uint64_t)kT > fit ? kShortR : (uint32_t)kT;
  const unsigned grid = (unsigned)((n + R - 1) / R);
  PackArgs a{in,   in_off, in_bias, n, base, enc_len, out_off, cap_off, out, out_cap, slots, (uint32_t)tag, R,
             in_bytes, lookback_help_polls()};
  if (four)
    encode_packed_kernel<4><<<dim3(grid), dim3(kT), 0, s>>>(a, t.code, t.len);
  else
    encode_packed_kernel<3><<<dim3(grid), dim3(kT), 0, s>>>(a, t.code, t.len);
  return hipGetLastError();
}

}  // namespace mhq
