// huff_encode.hip -- gfx950 batch encode of RFC 7541 Huffman literals.
//
// Semantics: HuffmanCompressor.Write + Pad (hc/huffman.go:23-37) over
// bitWriter (io/bitio.go:72-149): codes MSB-first, the last octet padded with
// 1 bits; encode_len is ceil(sum of code lengths / 8), the size the Auto
// choice compares with the raw length (hc/io.go:172).
//
// Structure: one workgroup of kT threads owns a block tile of kT consecutive
// literals and encodes it with one thread per literal (the same skeleton as
// huff_decode.hip):
//   * the tile's plaintext is staged in LDS (aligned 16-B loads) and read back
//     a word (4 bytes) at a time; the 256-entry code table sits in LDS too;
//   * a counting sort by plaintext length gives thread t the literal of rank
//     t, so the 64 literals of a wave have similar lengths;
//   * each thread appends codes to a 64-bit bit buffer and ORs complete
//     big-endian words into a zeroed LDS staging copy of the tile's output
//     region (words shared with the neighbouring literals need no ordering:
//     each literal ORs only its own bits); the region then leaves with
//     aligned 16-B stores, after the next tile's loads have been issued;
//   * while a tile is encoded, the block's next tile's offsets and plaintext
//     are in flight into registers;
//   * a tile whose plaintext exceeds the staging slice is processed as several
//     sub-tiles; a single literal larger than the slice is encoded by one
//     thread straight from global memory.
#include <hip/hip_runtime.h>

#include "huff_encode_dev.h"

namespace mhq {
namespace {

using namespace dev;

template <bool kEmit>
__global__ __launch_bounds__(kT) __attribute__((amdgpu_waves_per_eu((kT / 64 * MHQ_ENC_BLOCKS + 3) / 4))) void encode_kernel(
    const uint8_t *__restrict__ in, const uint64_t *__restrict__ in_off, uint64_t in_bias, uint64_t n,
    uint8_t *__restrict__ out, const uint64_t *__restrict__ out_off, uint64_t out_bias,
    uint32_t *__restrict__ enc_len, const uint32_t *__restrict__ g_code, const uint8_t *__restrict__ g_len,
    uint64_t per_block, uint32_t n_persist, uint32_t long_elsewhere) {
  __shared__ Smem<kEmit> sm;
  const uint32_t tid = threadIdx.x;
  const uint32_t lane = tid % kWave;
  const uint32_t wave = tid / kWave;
  // long_elsewhere: a batch outside the thread form's band (thread_form) is
  // the cooperative kernel's, launched beside this one: end at once
  if (long_elsewhere && !thread_form(in_off[n] - in_off[0], n)) return;
  // Two grids in one launch (the grid holds max(ceil(n / kT), n_persist)
  // workgroups): short literals (a mean under kShortMean bytes, so kT of them
  // fill about one staging slice) take one range of kT literals per
  // workgroup, and the dispatcher refills a CU as its workgroups end; longer
  // ones take n_persist persistent ranges of per_block literals (greedy
  // sub-tiles stay full) in the first workgroups, the others ending at once.
  // The short form's offsets are loaded beside the batch's bounds (its bytes
  // only once the form is known: a workgroup that ends at once loads nothing).
  // (A grid capped below ceil(n / kT) -- huge batches, so that the launch of
  // the form the batch does not take stays small -- makes the short form's
  // workgroups take ranges blockIdx.x + k * gridDim.x in turn.)
  const uint64_t bnd0 = in_off[0], bndn = in_off[n];
  uint64_t L0 = (uint64_t)blockIdx.x * kT;
  uint64_t L1 = min(L0 + (uint64_t)kT, n);
  const uint64_t Ls = min(L0, n);
  uint64_t i_cur = uniform64(vload(in_off, Ls)), o_cur = kEmit ? uniform64(vload(out_off, Ls)) : 0u;
  uint64_t i_end = uniform64(vload(in_off, max(L1, Ls)));
  const bool persist = (bndn - bnd0) > (uint64_t)MHQ_ENC_PERSIST_MEAN * n;
  if (persist) {
    if (blockIdx.x >= n_persist) return;
    L0 = (uint64_t)blockIdx.x * per_block;
    if (L0 >= n) return;
    L1 = min(L0 + per_block, n);
    i_cur = uniform64(vload(in_off, L0));
    o_cur = kEmit ? uniform64(vload(out_off, L0)) : 0u;
    i_end = uniform64(vload(in_off, L1));
  } else if (L0 >= n) {
    return;
  }
  Next nx;
  issue_next<kEmit>(nx, in, in_bias, in_off, out_off, L0, L1, i_cur, i_end, tid);
  uint64_t cur = L0;
  for (uint32_t i = tid; i < 256u; i += kT) sm.code[i] = make_uint2(g_code[i], g_len[i]);
  uint8_t *pd_o = nullptr;  // the previous sub-tile's output, still in LDS
  uint32_t pd_lo = 0, pd_hi = 0;
  bool pending = false;

  for (;;) {
  if (cur >= L1) {
    // the short form's next range (a capped grid), its first sub-tile's loads issued now
    if (persist || L1 >= n) break;
    L0 += (uint64_t)gridDim.x * kT;
    if (L0 >= n) break;
    L1 = min(L0 + (uint64_t)kT, n);
    __syncthreads();  // in_w free
    i_cur = uniform64(vload(in_off, L0));
    o_cur = kEmit ? uniform64(vload(out_off, L0)) : 0u;
    i_end = uniform64(vload(in_off, L1));
    issue_next<kEmit>(nx, in, in_bias, in_off, out_off, L0, L1, i_cur, i_end, tid);
    cur = L0;
  }
    // consume the prefetch (the previous sub-tile ended with a barrier: in_w is free)
    const uint32_t cnt = (uint32_t)min((uint64_t)kT, L1 - cur);
    const uint32_t ie = (uint32_t)(nx.ie64 - i_cur), oe = kEmit ? (uint32_t)(nx.oe64 - o_cur) : 0u;
    const uint8_t *ia = in + (i_cur - in_bias);
    uint8_t *oa = kEmit ? out + (o_cur - out_bias) : nullptr;
    const uint32_t idelta = (uint32_t)((uintptr_t)ia & 15u);
    const uint32_t odelta = kEmit ? (uint32_t)((uintptr_t)oa & 15u) : 0u;
    {
      const uint32_t chunks = prefetch_chunks(in, in_bias, i_cur, i_end);
#pragma unroll
      for (int k = 0; k < kPF; k++) {
        const uint32_t c = tid + (uint32_t)kT * k;
        if (c < chunks) *(u32x4 *)(sm.in_w + 4u * c) = nx.v[k];
      }
    }
    const bool fits = tid < cnt && ie + idelta <= (uint32_t)kInCap && (!kEmit || oe + odelta <= (uint32_t)kOutCap);
    uint32_t m = (uint32_t)__syncthreads_count(fits);
    const bool oversized = m == 0;  // literal `cur` alone is larger than a slice
    m = oversized ? 1u : m;
    if (tid == m - 1u) {
      sm.nbase[0] = nx.ie64;
      sm.nbase[1] = kEmit ? nx.oe64 : 0u;
    }
    if (tid == 0) sm.rec[0] = idelta | odelta << 16;
    if (fits) sm.rec[tid + 1] = (ie + idelta) | (oe + odelta) << 16;
    if (tid < kBuckets) sm.hist[tid] = 0;
    __syncthreads();
    const uint64_t i_nxt = sm.nbase[0], o_nxt = sm.nbase[1];
    issue_next<kEmit>(nx, in, in_bias, in_off, out_off, cur + m, L1, i_nxt, i_end, tid);
    if (kEmit && pending) store_out(pd_o, (const uint8_t *)sm.out_w, pd_lo, pd_hi, tid, kT);
    pending = false;
    if (oversized) {
      // (an empty output region: the caller skips this literal)
      if (tid == 0 && (!kEmit || o_nxt != o_cur))
        encode_literal_global<kEmit>(ia, i_nxt - i_cur, oa, sm.code, enc_len + cur);
    } else {
      const uint32_t out_bytes = kEmit ? sm.rec[m] >> 16 : 0u;
      if (kEmit) {
        __syncthreads();  // out_w has been read by the flush
        for (uint32_t c = tid; c < (out_bytes + 15u) >> 4; c += kT) *(u32x4 *)(sm.out_w + 4u * c) = u32x4{0u, 0u, 0u, 0u};
      }
      // counting sort by plaintext length
      uint32_t bk = 0, rk = 0;
      if (tid < m) {
        const uint32_t bytes = (sm.rec[tid + 1] & 0xffffu) - (sm.rec[tid] & 0xffffu);
        bk = bytes < 48u ? bytes : min(48u + ((bytes - 48u) >> 3), (uint32_t)kBuckets - 1u);
        rk = atomicAdd(&sm.hist[bk], 1u);
      }
      __syncthreads();
      if (wave == 0) {
        const uint32_t h = sm.hist[lane];
        sm.hist[lane] = wave_incl_scan(h) - h;
      }
      __syncthreads();
      if (tid < m) sm.order[sm.hist[bk] + rk] = (uint16_t)tid;
      __syncthreads();
      if (tid < m) {
        const uint32_t lit = sm.order[tid];
        const uint32_t r0 = sm.rec[lit], r1 = sm.rec[lit + 1];
        // an empty output region: the caller skips this literal (mhq_huff.h)
        const uint32_t bits = (!kEmit || (r1 >> 16) != (r0 >> 16))
                                  ? encode_one<kEmit>(sm, r0 & 0xffffu, r1 & 0xffffu, r0 >> 16)
                                  : 0u;
        if (!kEmit) enc_len[cur + lit] = (bits + 7u) >> 3;
      }
      __syncthreads();  // in_w free, out_w complete
      if (kEmit) {
        pd_o = oa - odelta;
        pd_lo = odelta;
        pd_hi = out_bytes;
        pending = true;
      }
    }
    cur += m;
    i_cur = i_nxt;
    o_cur = o_nxt;
  }
  if (kEmit && pending) store_out(pd_o, (const uint8_t *)sm.out_w, pd_lo, pd_hi, tid, kT);
}

// ---- encode_len: sum of code lengths per literal --------------------------
// Sizes for the Auto choice and the output layout (hc/io.go:157-172: the
// length of the temp-buffer encode, ceil(sum of code lengths / 8)).
//
// A wave takes 64 consecutive literals and walks their whole byte range
// [A, B) in rounds of 1 KiB: lane l loads aligned 16-B chunk l of the round
// (one coalesced load per lane, each byte loaded once), looks up its 16 code
// lengths (LDS, one per dword) and forms their running sums; a wave scan of
// the lane totals turns them into P(x) = code bits of the range's bytes
// before x, for every byte x of the round, written to the wave's LDS row.
// A literal [a, b) has P(b) - P(a) bits: each lane picks up P at its two
// ends in the rounds that hold them (u32 arithmetic mod 2^32, exact for any
// literal of < 2^32 bits).  Every lane does the same work whatever the
// length mix, and long literals are spread over the wave.
constexpr int kLenT = kLenSumBlock;  // 4 waves of 64 literals
#ifndef MHQ_LEN_RB  // encode_len: rounds whose loads are issued together
#define MHQ_LEN_RB 4
#endif
constexpr int kLenRB = MHQ_LEN_RB;
constexpr uint32_t kRound = kWave * 16;  // bytes per round

// Slot of P(x) in a wave's row: lane l's 16 values (4 chunks of 4) go to
// chunk slots j ^ (l % 4), so the 8 lanes of a ds_write_b128 group spread over
// the banks (64-B lane stride: linear, lanes l and l+2 collide 4-way).
// Position kRound (one past the round) stays where it is.
__device__ __forceinline__ uint32_t prow(uint32_t x) {
  return x < kRound ? x ^ ((x >> 2) & 0xcu) : x;
}

__device__ __forceinline__ uint32_t chunk_bits(const u32x4 &x, const uint8_t *lens, uint32_t q[16]) {
  const uint32_t w[4] = {x.x, x.y, x.z, x.w};
  uint32_t t = 0;
#pragma unroll
  for (int k = 0; k < 16; k++) {
    q[k] = t;
    t += lens[(w[k >> 2] >> (8 * (k & 3))) & 0xffu];
  }
  return t;
}

// A wave sizes kLenLPL x 64 consecutive literals (lane l: literals l, l + 64,
// ...), a workgroup of kLenT / kLenLPL threads the kLenT literals of one
// block sum.  More literals per lane pay a wave's two dependent HBM trips
// (offsets, then the bytes they locate) less often, but cost registers: the
// occupancy matters more (layout call).
constexpr int kLenLPL = MHQ_LEN_LPL;
constexpr int kLenThreads = kLenT / kLenLPL;
static_assert(kLenThreads % kWave == 0 && kLenThreads <= 256, "encode_len workgroup shape");

__global__ __launch_bounds__(kLenThreads) void encode_len_kernel(const uint8_t *__restrict__ in,
                                                                 const uint64_t *__restrict__ in_off,
                                                                 uint64_t in_bias, uint64_t n,
                                                                 uint32_t *__restrict__ enc_len,
                                                                 const uint8_t *__restrict__ g_len,
                                                                 uint64_t *__restrict__ block_sums) {
  // code lengths one byte each: byte values b and b+1..b+3 share a dword
  // (a broadcast), and only b and b+128 share a bank (ds_read_u8 banks by
  // dword): text lookups are nearly conflict-free, where a u32 table put
  // 0x21 / 0x41 / 0x61 on one bank
  constexpr int kW = kLenThreads / kWave;
  __shared__ uint8_t lens[256];
  // P over one round as chunk prefixes (u32, + the position after the round)
  // and in-chunk prefixes (u8 or u16, at most 15 x 30 bits): one or two 16-B
  // stores per lane and round
  __shared__ uint32_t ppre[kW][kWave + 4];
  __shared__ __attribute__((aligned(16))) uint16_t pq[kW][kRound];
  __shared__ uint64_t part[2 * kW];
  const uint32_t lane = threadIdx.x % kWave, wave = threadIdx.x / kWave;
  const uint64_t s = (uint64_t)blockIdx.x * kLenT + (uint64_t)wave * (kWave * kLenLPL);  // the wave's first literal
  for (uint32_t x = threadIdx.x; x < 256u; x += kLenThreads) lens[x] = g_len[x];
  uint64_t a[kLenLPL];
#pragma unroll
  for (int k = 0; k < kLenLPL; k++) a[k] = in_off[min(s + (uint64_t)(kWave * k) + lane, n) + vzero()] - in_bias;
  const uint64_t bw = in_off[min(s + (uint64_t)(kWave * kLenLPL), n) + vzero()] - in_bias;  // the range's end
  __syncthreads();
  uint32_t el[kLenLPL] = {};
  if (s < n) {
    // literal s + 64k + l ends where the next one starts
    uint64_t b[kLenLPL];
#pragma unroll
    for (int k = 0; k < kLenLPL; k++) {
      const uint64_t nx = (uint64_t)__shfl_down((unsigned long long)a[k], 1);  // every lane active
      const uint64_t wrap = k + 1 < kLenLPL ? uniform64(a[k + 1 < kLenLPL ? k + 1 : k]) : bw;
      b[k] = lane < kWave - 1 ? nx : wrap;
    }
    const uint64_t aw = uniform64(a[0]);  // lane 0: literal s
    const uint8_t *base8 = in + aw - ((uintptr_t)(in + aw) & 15u);  // pointer arithmetic: global loads, not flat
    const uintptr_t base = (uintptr_t)base8;
    const u32x4 *src = (const u32x4 *)base8;
    // aligned chunks holding a byte of [aw, bw): none for an empty range
    const uint64_t nchunk = bw > aw ? ((uintptr_t)(in + bw) - base + 15u) >> 4 : 0u;
    const uint32_t nround = (uint32_t)((nchunk + kWave - 1) / kWave);
    uint32_t pa[kLenLPL], pb[kLenLPL], Pa[kLenLPL] = {}, Pb[kLenLPL] = {};
#pragma unroll
    for (int k = 0; k < kLenLPL; k++) {
      pa[k] = (uint32_t)((uintptr_t)(in + a[k]) - base);
      pb[k] = (uint32_t)((uintptr_t)(in + b[k]) - base);
    }
    uint32_t *pre_row = ppre[wave];
    uint16_t *q_row = pq[wave];
    uint32_t carry = 0;
    for (uint32_t r0 = 0; r0 < nround; r0 += kLenRB) {
      u32x4 v[kLenRB];
#pragma unroll
      for (int k = 0; k < kLenRB; k++) {
        const uint64_t c = (uint64_t)(r0 + k) * kWave + lane;
        v[k] = u32x4{0u, 0u, 0u, 0u};
        if (c < nchunk) v[k] = __builtin_nontemporal_load(src + c);  // aligned, holds a valid byte
      }
#pragma unroll
      for (int k = 0; k < kLenRB; k++) {
        if (r0 + k >= nround) break;  // wave-uniform
        uint32_t q[16];
        const uint32_t tot = chunk_bits(v[k], lens, q);
        const uint32_t pre = carry + wave_incl_scan(tot) - tot;
        // When every in-chunk prefix of the round fits a byte (chunks under
        // 16 bits per byte: all text), q is stored as bytes, lane l's 16 at
        // 16 l (one 16-B store; a store group's 8 lanes on 128 consecutive
        // bytes); otherwise as u16, lane l's 32 bytes at 32 l (two stores, a
        // group's lanes on 256 consecutive bytes).  No bank conflict either way.
        const bool bytes = __ballot(q[15] > 255u) == 0;  // (uniform)
        if (bytes) {
          uint32_t d[4];
#pragma unroll
          for (int j = 0; j < 4; j++) d[j] = q[4 * j] | q[4 * j + 1] << 8 | q[4 * j + 2] << 16 | q[4 * j + 3] << 24;
          *(u32x4 *)((uint8_t *)q_row + 16u * lane) = u32x4{d[0], d[1], d[2], d[3]};
        } else {
          *(u32x4 *)(q_row + 16u * lane) =
              u32x4{q[0] | q[1] << 16, q[2] | q[3] << 16, q[4] | q[5] << 16, q[6] | q[7] << 16};
          *(u32x4 *)(q_row + 16u * lane + 8u) =
              u32x4{q[8] | q[9] << 16, q[10] | q[11] << 16, q[12] | q[13] << 16, q[14] | q[15] << 16};
        }
        pre_row[lane] = pre;
        if (lane == kWave - 1) pre_row[kWave] = pre + tot;  // the position after the round
        wave_sync();
        const uint32_t lo = (r0 + k) * kRound;  // positions [lo, lo + kRound]
        const uint8_t *q8 = (const uint8_t *)q_row;
        auto P = [&](uint32_t x, uint32_t &dst) {
          if (x < kRound) dst = pre_row[x >> 4] + (bytes ? (uint32_t)q8[x] : (uint32_t)q_row[x]);
          if (x == kRound) dst = pre_row[kWave];
        };
#pragma unroll
        for (int j = 0; j < kLenLPL; j++) {
          P(pa[j] - lo, Pa[j]);
          P(pb[j] - lo, Pb[j]);
        }
        carry = __builtin_amdgcn_readlane(pre + tot, kWave - 1);
        wave_sync();
      }
    }
#pragma unroll
    for (int k = 0; k < kLenLPL; k++) {
      el[k] = (Pb[k] - Pa[k] + 7u) >> 3;
      const uint64_t i = s + (uint64_t)(kWave * k) + lane;
#if MHQ_ENC_NTST
      if (i < n) __builtin_nontemporal_store(el[k], enc_len + i);
#else
      if (i < n) enc_len[i] = el[k];
#endif
    }
  }
  if (!block_sums) return;  // uniform over the grid
  // the block's (sum of enc_len, sum of decode capacities) for the offsets scan
  uint64_t sa = 0, sb = 0;
#pragma unroll
  for (int k = 0; k < kLenLPL; k++) {
    sa += el[k];
    sb += ((uint64_t)el[k] * 8u) / 5u;
  }
#pragma unroll
  for (int d = 1; d < kWave; d <<= 1) {
    sa += __shfl_xor(sa, d);
    sb += __shfl_xor(sb, d);
  }
  if (lane == 0) {
    part[2 * wave] = sa;
    part[2 * wave + 1] = sb;
  }
  __syncthreads();
  if (threadIdx.x < 2) {
    uint64_t v = 0;
#pragma unroll
    for (int w = 0; w < kW; w++) v += part[2 * w + threadIdx.x];
    block_sums[2 * blockIdx.x + threadIdx.x] = v;
  }
}

// ---- wave-cooperative encode ----------------------------------------------
// A wave takes K groups of 64 consecutive literals (64 K literals) and walks
// their whole byte range in rounds of 1 KiB, lane l on aligned 16-B chunk l of
// the round (one coalesced load per lane, every byte loaded once), as
// encode_len does.  No lane owns a literal; where a code goes follows from the
// output layout itself:
//   * a literal's first code starts at bit 8 * out_off[i] (relative to the
//     wave's 16-B aligned output base, plus kPB): the lane holding the literal
//     writes that position into the round's qtab at the literal's first byte
//     (zero = no literal starts at that byte);
//   * every other code starts where the previous byte's code ended.  So the
//     position of a chunk's first byte is a segmented scan over the lanes:
//     each lane's chunk sums up to (starts in it?, end position) -- its last
//     start's position plus the code lengths after it, or the sum of all its
//     lengths -- and the wave combines them (a start resets the sum) in one
//     DPP scan, carried from round to round;
//   * each lane then places its 16 codes through a two-word window and ORs
//     complete words into the wave's LDS output ring.
// The ring holds the complement of the output (the table's codes are stored
// complemented, bits a code does not cover stay 0), so the padding after a
// literal's last code -- bitWriter.Pad(0xff), io/bitio.go:135-149 -- needs no
// work: every bit no code wrote comes out as 1 when the ring is stored
// inverted.  After each round the complete 16-B chunks of the ring leave as
// aligned stores (bytes of the chunks at the wave's two ends that belong to a
// neighbour's region are left alone).
// Bytes that belong to no literal of the wave cost nothing extra: positions
// start kPB bits before the region, so the bytes before the first literal (in
// the first chunk) are placed there, before the first literal's start resets
// the position; the range's end is one more start (at the region's end), so
// the bytes after it land past the region; chunks past the range read as '0'
// (5-bit codes) and land past it too.  Nothing outside [region start, region
// end) is ever stored.
// Waves whose layout the ring cannot express (a literal with an empty output
// region -- the caller skips it -- or offsets out of order, or more than
// 2^27 bytes, or a round whose output would overflow the ring: regions much
// longer than their codes) encode one literal per lane from global memory.
#ifndef MHQ_ENC_COOP  // 1: the wave-cooperative encode; 0: one thread per literal (encode_kernel)
#define MHQ_ENC_COOP 1
#endif
#ifndef MHQ_ENC_X  // timing experiments only (wrong output): 1 no table lookups, 2 no ring ORs in pass 2, 4 no qtab reads
#define MHQ_ENC_X 0
#endif
#ifndef MHQ_ENC_K  // literal groups of 64 per wave (0: by batch size)
#define MHQ_ENC_K 0
#endif
constexpr int kCT = 256;          // threads per workgroup: 4 waves
constexpr int kCW = kCT / kWave;
constexpr uint32_t kRingW = 1024;  // output ring words per wave (4 KiB)
constexpr uint32_t kPB = 512;      // bit positions start 64 bytes before the wave's output base
constexpr uint32_t kZeroBytes = 0x30303030u;  // '0' x 4: 5-bit codes for chunks past the range

struct alignas(16) CoopSmem {
  uint2 code[256];                 // (complemented code, left-aligned; length)
  uint32_t ring[kCW][kRingW];      // complemented output words (MSB-first values), zero where unwritten
  uint32_t qtab[kCW][kRound];      // (prow) output bit position of a literal starting at a byte; 0: none
};

// Segmented inclusive scan of x = value | flag << 31 over the wave (lane order):
// combine(earlier e, later x) = flag(x) ? x : e + x.  DPP moves as in
// wave_incl_scan; every lane must be active.
__device__ __forceinline__ uint32_t seg_incl_scan(uint32_t x) {
#define MHQ_SEG_STEP(ctrl, rmask, bc)                                                     \
  {                                                                                       \
    const uint32_t t = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, ctrl, rmask, 0xf, bc); \
    x = (int32_t)x < 0 ? x : t + x;                                                       \
  }
  MHQ_SEG_STEP(0x111, 0xf, true)   // row_shr:1
  MHQ_SEG_STEP(0x112, 0xf, true)   // row_shr:2
  MHQ_SEG_STEP(0x114, 0xf, true)   // row_shr:4
  MHQ_SEG_STEP(0x118, 0xf, true)   // row_shr:8
  MHQ_SEG_STEP(0x142, 0xa, false)  // row_bcast:15
  MHQ_SEG_STEP(0x143, 0xc, false)  // row_bcast:31
#undef MHQ_SEG_STEP
  return x;
}

// Lane l gets v of lane l + 1, lane 63 gets `last` (DPP wave_shl:1 with every
// lane active: a shuffle under `lane < 63 ? ... : ...` may run with lane 63
// masked off, and a read from an inactive lane returns 0).
__device__ __forceinline__ uint64_t from_next_lane(uint64_t v, uint64_t last) {
  const uint32_t lo = (uint32_t)__builtin_amdgcn_update_dpp((int)(uint32_t)last, (int)(uint32_t)v, 0x130, 0xf, 0xf, false);
  const uint32_t hi =
      (uint32_t)__builtin_amdgcn_update_dpp((int)(uint32_t)(last >> 32), (int)(uint32_t)(v >> 32), 0x130, 0xf, 0xf, false);
  return (uint64_t)lo | ((uint64_t)hi << 32);
}

// One literal by one lane straight from global memory (the fallback waves),
// from the complemented, left-aligned table.
__device__ void encode_literal_coop_global(const uint8_t *src, uint64_t nbytes, uint8_t *dst, const uint2 *code) {
  BitOutGlobal bo{dst, 0, 0};
  for (uint64_t i = 0; i < nbytes; i++) {
    const uint2 c = code[src[i]];
    bo.put(~(c.x >> (32u - c.y)) & ((1u << c.y) - 1u), c.y);
  }
  bo.finish();
}

#ifdef MHQ_DIAG_ETL  // diagnostic build: per-wave timeline of the coop encode (s_memrealtime, 100 MHz)
constexpr int kEtlSlots = 64;  // [0] start, [1] table ready, [2] offsets used, [3] first loads issued, [4 + r] round r done, [63] end
constexpr int kEtlWaves = 16384;
__device__ unsigned long long g_etl[kEtlWaves * kEtlSlots];
#define ETL(slot)                                                                                    \
  do {                                                                                               \
    const uint32_t _w = blockIdx.x * kCW + threadIdx.x / kWave;                                      \
    const int _s = (slot);                                                                           \
    if (threadIdx.x % kWave == 0 && _w < kEtlWaves && _s < kEtlSlots) g_etl[_w * kEtlSlots + _s] = wall_clock64(); \
  } while (0)
#else
#define ETL(slot) \
  do {            \
  } while (0)
#endif

template <int K>
__global__ __launch_bounds__(kCT) void encode_coop_kernel(const uint8_t *__restrict__ in,
                                                          const uint64_t *__restrict__ in_off, uint64_t in_bias,
                                                          uint64_t n, uint8_t *__restrict__ out,
                                                          const uint64_t *__restrict__ out_off, uint64_t out_bias,
                                                          const uint32_t *__restrict__ g_code,
                                                          const uint8_t *__restrict__ g_len,
                                                          uint32_t short_elsewhere) {
  __shared__ CoopSmem sm;
  const uint32_t tid = threadIdx.x, lane = tid % kWave, wave = tid / kWave;
  // short_elsewhere: a batch in the thread form's band (thread_form) is
  // encode_kernel's, launched beside this one: end at once
  if (short_elsewhere && thread_form(in_off[n] - in_off[0], n)) return;
  ETL(0);
  // the code table; the waves are independent after the barrier
  {
    const uint32_t L = g_len[tid];
    const uint32_t c = ~g_code[tid] & ((1u << L) - 1u);
    sm.code[tid] = make_uint2(c << (32u - L), L);  // left-aligned (every length is 5..30)
  }
  uint32_t *ring = sm.ring[wave];
  uint32_t *qtab = sm.qtab[wave];
  __syncthreads();
  ETL(1);
  // Persistent: wave w takes the ranges of K groups of 64 literals
  // [s, s + 64 K), s = 64 K (w + j * waves in the grid), j = 0, 1, ...: one
  // generation of waves (the launch holds at most what stays resident), so a
  // launch that ends at once (short_elsewhere) costs only that generation.
  const uint64_t stride = (uint64_t)gridDim.x * kCW * (uint64_t)(kWave * K);
  for (uint64_t s = ((uint64_t)blockIdx.x * kCW + wave) * (uint64_t)(kWave * K); s < n; s += stride) {
  uint64_t a[K], o[K];
#pragma unroll
  for (int k = 0; k < K; k++) {
    const uint64_t i = min(s + (uint64_t)(kWave * k) + lane, n) + vzero();
    a[k] = in_off[i] - in_bias;
    o[k] = out_off[i] - out_bias;
  }
  const uint64_t ae = in_off[min(s + (uint64_t)(kWave * K), n) + vzero()] - in_bias;
  const uint64_t oend = out_off[min(s + (uint64_t)(kWave * K), n) + vzero()] - out_bias;
#pragma unroll
  for (int k = 0; k < 4; k++) {  // (a range that fell back, or ended past its region, leaves words behind)
    ((u32x4 *)ring)[lane + kWave * k] = u32x4{0u, 0u, 0u, 0u};
    ((u32x4 *)qtab)[lane + kWave * k] = u32x4{0u, 0u, 0u, 0u};
  }
  wave_sync();
  const uint64_t A = uniform64(a[0]), OA = uniform64(o[0]);
  // layouts the ring cannot express: a literal whose output region is empty
  // (the caller skips it, mhq_huff.h), offsets out of order, or a range over
  // 2^27 bytes (positions are u32 bit counts)
  bool odd = ae < A || oend < OA || (ae - A) >= (1u << 27) || (oend - OA) >= (1u << 27);
  bool nonempty[K];
  uint64_t b[K], oe[K];
#pragma unroll
  for (int k = 0; k < K; k++) {
    const uint64_t na = k + 1 < K ? uniform64(a[k + 1 < K ? k + 1 : k]) : ae;
    const uint64_t no = k + 1 < K ? uniform64(o[k + 1 < K ? k + 1 : k]) : oend;
    b[k] = from_next_lane(a[k], na);
    oe[k] = from_next_lane(o[k], no);
    const bool valid = s + (uint64_t)(kWave * k) + lane < n;
    nonempty[k] = valid && b[k] > a[k];
    odd = odd || (valid && ((nonempty[k] && oe[k] == o[k]) || oe[k] < o[k] || b[k] < a[k]));
  }
  bool fallback = __ballot(odd) != 0;
  if (!fallback && ae > A) {
    const uint8_t *ia = in + A;
    const uint8_t *ibase = ia - ((uintptr_t)ia & 15u);
    uint8_t *oa = out + OA;
    uint8_t *obase = oa - ((uintptr_t)oa & 15u);
    const uint32_t odelta = (uint32_t)((uintptr_t)oa & 15u);
    const uint32_t out_hi = odelta + (uint32_t)(oend - OA);  // the region's end, bytes from obase
    const uint32_t b_rel = (uint32_t)((in + ae) - ibase);    // the range's end from ibase
    // per literal: its first byte from ibase (~0: empty, never a start) and
    // the bit position of its first code; per group, the span of its first bytes
    uint32_t a_rel[K], q_lit[K], g_lo[K], g_hi[K];
#pragma unroll
    for (int k = 0; k < K; k++) {
      a_rel[k] = nonempty[k] ? (uint32_t)((in + a[k]) - ibase) : ~0u;
      q_lit[k] = kPB + 8u * (uint32_t)((out + o[k]) - obase);
      g_lo[k] = (uint32_t)((in + uniform64(a[k])) - ibase);
      const uint64_t a63 = (uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)a[k], kWave - 1) |
                           ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(a[k] >> 32), kWave - 1) << 32);
      g_hi[k] = (uint32_t)((in + a63) - ibase);
    }
    const uint32_t nchunk = (b_rel + 15u) >> 4;
    const uint32_t nround = (nchunk + kWave - 1) / kWave;
    ETL(2);
    const u32x4 *src = (const u32x4 *)ibase;
    // chunk c of the ring = bytes [16 c - 64, 16 c - 48) from obase; chunks
    // 0-3 only ever hold the bytes before the first literal
    const uint32_t end_chunk = (out_hi + 64u + 15u) >> 4;
    // round 0, lane 0 starts 480 bits before the first literal (its <= 15
    // bytes before A take <= 450 bits)
    uint32_t carry = 0x80000000u | (kPB - 480u + 8u * odelta);
    uint32_t flushed = 4;  // ring chunks stored (or never to be stored) so far

    // Stores ring chunks [c0, c1) inverted: whole chunks inside the region as
    // 16-B stores, the bytes of a chunk at either end that lie inside
    // [odelta, out_hi) one by one; each chunk is then zeroed.
    auto flush = [&](uint32_t c0, uint32_t c1) {
      for (uint32_t c = c0 + lane; c < c1; c += kWave) {
        u32x4 *p = (u32x4 *)(ring + ((4u * c) & (kRingW - 1u)));  // words 4c .. 4c+3
        const u32x4 h = *p;
        const u32x4 w = u32x4{~__builtin_bswap32(h.x), ~__builtin_bswap32(h.y), ~__builtin_bswap32(h.z),
                              ~__builtin_bswap32(h.w)};
        const uint32_t lo = 16u * c - 64u, hi = lo + 16u;
        if (lo >= odelta && hi <= out_hi) {
#if MHQ_ENC_NTST
          __builtin_nontemporal_store(w, (u32x4 *)(obase + lo));
#else
          *(u32x4 *)(obase + lo) = w;
#endif
        } else {
          const uint32_t ww[4] = {w.x, w.y, w.z, w.w};
          for (uint32_t x = max(lo, odelta); x < min(hi, out_hi); x++)
            obase[x] = (uint8_t)(ww[(x - lo) >> 2] >> (8u * (x & 3u)));
        }
        *p = u32x4{0u, 0u, 0u, 0u};
      }
    };

    // loads run three rounds ahead; chunk indices are clamped to the last
    // chunk (every lane loads: no predicated register copies; an aligned
    // chunk holding a valid byte never crosses a page)
    u32x4 vb0 = __builtin_nontemporal_load(src + min((uint32_t)lane, nchunk - 1u));
    u32x4 vb1 = __builtin_nontemporal_load(src + min((uint32_t)lane + kWave, nchunk - 1u));
    u32x4 vb2 = __builtin_nontemporal_load(src + min((uint32_t)lane + 2u * kWave, nchunk - 1u));
    ETL(3);
    // One round: consumes vb (loaded three rounds earlier) and reloads it for
    // three rounds later.  The round loop is unrolled by three so that each
    // buffer keeps its registers: a rotation (vb0 = vb1, ...) moves registers
    // whose loads are still in flight, and the compiler waits for every
    // outstanding load and store before such a move.  Returns false when the
    // round's output would overflow the ring.
    auto round = [&](const uint32_t r, u32x4 &vb) -> bool {
      const uint32_t lo = r * kRound;
      // the round's literal starts; the range's end acts as one more start,
      // at the region's end
#pragma unroll
      for (int k = 0; k < K; k++) {
        if (g_hi[k] >= lo && g_lo[k] < lo + kRound) {  // (wave-uniform: a group's starts lie in [g_lo, g_hi])
          const uint32_t x = a_rel[k] - lo;
          if (x < kRound) qtab[prow(x)] = q_lit[k];
        }
      }
      if (lane == 0 && b_rel - lo < kRound) qtab[prow(b_rel - lo)] = kPB + 8u * out_hi;
      const uint32_t c = lo / 16u + lane;  // this lane's chunk
      const u32x4 v = c < nchunk ? vb : u32x4{kZeroBytes, kZeroBytes, kZeroBytes, kZeroBytes};
      vb = __builtin_nontemporal_load(src + min(c + 3u * kWave, nchunk - 1u));
      wave_sync();
      uint32_t q16[16];
#pragma unroll
      for (int j = 0; j < 4; j++) {
        u32x4 *qp = (u32x4 *)(qtab + prow(16u * lane + 4u * j));
#if MHQ_ENC_X & 4
        const u32x4 t = lane == 0 && j == 0 ? *qp : u32x4{0u, 0u, 0u, 0u};
#else
        const u32x4 t = *qp;
        *qp = u32x4{0u, 0u, 0u, 0u};  // (read back before the zeroing: same lane, LDS in order)
#endif
        q16[4 * j] = t.x;
        q16[4 * j + 1] = t.y;
        q16[4 * j + 2] = t.z;
        q16[4 * j + 3] = t.w;
      }
      // code table lookups (complemented left-aligned code, length)
      uint32_t cd[16], ln[16];
      {
        const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
        for (int k = 0; k < 16; k++) {
#if MHQ_ENC_X & 1
          cd[k] = w[k >> 2] << (8 * (k & 3));
          ln[k] = 8u;
#else
          const uint2 t = sm.code[(w[k >> 2] >> (8 * (k & 3))) & 0xffu];
          cd[k] = t.x;
          ln[k] = t.y;
#endif
        }
      }
      // pass 1: the chunk's summary for the segmented scan
      uint32_t acc = 0;
      bool any = false;
#pragma unroll
      for (int k = 0; k < 16; k++) {
        acc = q16[k] != 0u ? q16[k] : acc;
        any = any || q16[k] != 0u;
        acc += ln[k];
      }
      const uint32_t summ = (acc & 0x7fffffffu) | (any ? 0x80000000u : 0u);
      const uint32_t incl = seg_incl_scan(summ);
      uint32_t excl = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)incl, 0x138, 0xf, 0xf, false);  // wave_shr:1
      excl = lane == 0 ? 0u : excl;
      // the position of the chunk's first byte: the carry, then lanes 0..l-1
      const uint32_t start = ((int32_t)excl < 0 ? excl : carry + excl) & 0x7fffffffu;
      const uint32_t last = __builtin_amdgcn_readlane((int32_t)incl, kWave - 1);
      carry = ((int32_t)last < 0 ? last : carry + last) | 0x80000000u;
      // the ring holds chunks [flushed, the carry's chunk]: one word short of
      // the ring at most (a literal region much longer than its code)
      if (((carry & 0x7fffffffu) >> 5) - 4u * flushed >= kRingW - 4u) return false;
      // pass 2: the lane's codes in order through a two-word window (hi, lo)
      // whose top word starts at bit wlo - 32; a code starting at pos lands
      // in hi from bit pos % 32 on (alignbit shifts by pos % 32 only) and
      // spills into lo.  Before a code that starts past the top word, that
      // word is complete: it goes out (OR: the first and last words are
      // shared with the neighbouring lanes) and the window moves on a word.
      {
        uint32_t pos = start, wlo = (start & ~31u) + 32u, hi = 0u, lw = 0u;
#pragma unroll
        for (int k = 0; k < 16; k++) {
          pos = q16[k] != 0u ? q16[k] : pos;  // a literal starts here
          if (pos >= wlo) {
            if (!(MHQ_ENC_X & 2)) atomicOr(ring + (((wlo - 32u) >> 5) & (kRingW - 1u)), hi);
            hi = lw;
            lw = 0u;
            wlo += 32u;
            while (pos >= wlo) {  // a gap of a word or more (a region longer than its code)
              atomicOr(ring + (((wlo - 32u) >> 5) & (kRingW - 1u)), hi);
              hi = lw;
              lw = 0u;
              wlo += 32u;
            }
          }
          hi |= __builtin_amdgcn_alignbit(0u, cd[k], pos);
          lw |= __builtin_amdgcn_alignbit(cd[k], 0u, pos);
          pos += ln[k];
        }
        if (MHQ_ENC_X & 2) {
          if ((hi ^ lw) == 0x12345u) ring[lane] = hi;  // (keeps the values live)
        } else {
          if (hi) atomicOr(ring + (((wlo - 32u) >> 5) & (kRingW - 1u)), hi);
          if (lw) atomicOr(ring + ((wlo >> 5) & (kRingW - 1u)), lw);
        }
      }
      wave_sync();
      if (r == 0 && lane < 4) ((u32x4 *)ring)[lane] = u32x4{0u, 0u, 0u, 0u};  // chunks 0-3: bytes before A
      // every bit before the carry's position is final
      const uint32_t done = min((carry & 0x7fffffffu) >> 7, end_chunk);
      flush(flushed, done);
      flushed = max(flushed, done);
      wave_sync();
      ETL(4 + (int)min(r, 58u));
      return true;
    };
    for (uint32_t r = 0; r < nround && !fallback; r += 3) {
      fallback = !round(r, vb0);
      if (!fallback && r + 1 < nround) fallback = !round(r + 1, vb1);
      if (!fallback && r + 2 < nround) fallback = !round(r + 2, vb2);
    }
    if (!fallback) flush(flushed, end_chunk);
  }
  if (fallback) {  // (offsets read again: nothing of the above stays live through the rounds)
    for (int k = 0; k < K; k++) {
      const uint64_t i = s + (uint64_t)(kWave * k) + lane;
      if (i < n) {
        const uint64_t fa = in_off[i] - in_bias, fb = in_off[i + 1] - in_bias;
        const uint64_t fo = out_off[i] - out_bias, foe = out_off[i + 1] - out_bias;
        if (fb > fa && foe != fo) encode_literal_coop_global(in + fa, fb - fa, out + fo, sm.code);
      }
    }
  }
  wave_sync();
  }
  ETL(63);
}

}  // namespace

#ifdef MHQ_DIAG_ETL
extern "C" int mhq_diag_etimeline(unsigned long long *out, int n) {
  const int m = n < kEtlWaves * kEtlSlots ? n : kEtlWaves * kEtlSlots;
  hipDeviceSynchronize();
  const int rc = hipMemcpyFromSymbol(out, HIP_SYMBOL(g_etl), m * sizeof(unsigned long long)) == hipSuccess ? kEtlSlots : -1;
  static unsigned long long zeros[kEtlWaves * kEtlSlots];
  hipMemcpyToSymbol(HIP_SYMBOL(g_etl), zeros, sizeof(zeros));
  return rc;
}
#endif

hipError_t launch_encode_len(const DevTables &t, const uint8_t *in, const uint64_t *in_off, uint64_t in_bias,
                             uint64_t n, uint32_t *enc_len, hipStream_t s, uint64_t *block_sums) {
  if (n == 0) return hipSuccess;
  // (one workgroup per group of kLenT literals at full occupancy; a
  // persistent grid prefetching the next group was slower)
  encode_len_kernel<<<dim3((unsigned)((n + kLenT - 1) / kLenT)), dim3(kLenThreads), 0, s>>>(in, in_off, in_bias, n,
                                                                                            enc_len, t.len, block_sums);
  return hipGetLastError();
}

hipError_t launch_encode(const DevTables &t, const uint8_t *in, const uint64_t *in_off, uint64_t in_bias,
                         uint64_t n, uint8_t *out, const uint64_t *out_off, uint64_t out_bias, hipStream_t s) {
  if (n == 0) return hipSuccess;
  // Two forms, picked on the device by the batch's mean literal (the host
  // does not know the byte count of a device batch, thread_form): from
  // kTinyMean to kShortMean bytes the thread-per-literal kernel (config 2:
  // 37 us against 47.6 for the cooperative one), outside that band the
  // wave-cooperative kernel (config 3 1.4x, config 4 1.4x, config 5 2.5x
  // faster).  Both are launched; the one the mean does not pick reads the
  // batch's two bounds and ends.  MHQ_ENC_FORM=thread|coop in the
  // environment forces a form, as MHQ_ENC_K (K groups per coop wave) forces
  // the cooperative one: tests and tuning.
  static const int k_env = [] {
    const char *e = getenv("MHQ_ENC_K");
    return e ? atoi(e) : 0;
  }();
  static const int form = [] {  // 0 by the mean, 1 thread, 2 coop
    const char *e = getenv("MHQ_ENC_FORM");
    if (e && !strcmp(e, "thread")) return 1;
    if ((e && !strcmp(e, "coop")) || k_env) return 2;
    return MHQ_ENC_COOP ? 0 : 1;
  }();
  if (form != 2) {
    // persistent form: MHQ_ENC_BLOCKS resident workgroups per CU (never more than the tiles)
    const unsigned persist = dev::tile_grid((n + kT - 1) / kT, 1, MHQ_ENC_BLOCKS * MHQ_PER_CU);
    const uint64_t tiles = (n + kT - 1) / kT;
    // short form: one range of kT literals per workgroup, at most kShortGen
    // resident generations of workgroups (past that they loop over ranges), so
    // that for a batch the cooperative kernel takes this launch stays small
    const uint64_t cap = (uint64_t)persist * MHQ_ENC_SHORT_GENS;
    const uint64_t want = tiles < cap ? tiles : cap;
    const unsigned grid = (unsigned)(want > persist ? want : persist);
    encode_kernel<true><<<dim3(grid), dim3(kT), 0, s>>>(in, in_off, in_bias, n, out, out_off, out_bias, nullptr,
                                                         t.code, t.len, (n + persist - 1) / persist, persist,
                                                         form == 0 ? 1u : 0u);
    if (form == 1) return hipGetLastError();
  }
  // K groups of 64 literals per wave: as many as keep about two waves per
  // SIMD slot (16 per CU) busy
  int K = MHQ_ENC_K ? MHQ_ENC_K : k_env;
  // (a forced K is rounded down to an instantiated one: 1, 2, 4 or 8)
  K = K <= 0 ? 0 : K >= 8 ? 8 : K >= 4 ? 4 : K >= 2 ? 2 : 1;
  if (K == 0) {
    const uint64_t slots = (uint64_t)dev::device_cus() * 16u * 2u;
    K = 1;
    while (K < 4 && (n + (uint64_t)kWave * 2 * K - 1) / ((uint64_t)kWave * 2 * K) >= slots) K *= 2;
    // (K = 8 builds at 131 VGPRs, three waves per SIMD: the resident grid
    // below assumes four; larger batches loop over more ranges instead)
  }
  const uint64_t per_wg = (uint64_t)kCT * K;
  // at most one resident generation: 4 workgroups of 34 KiB LDS per CU
  const uint64_t resident = (uint64_t)dev::device_cus() * 4u;
  const dim3 cgrid((unsigned)std::min<uint64_t>((n + per_wg - 1) / per_wg, resident));
  const uint32_t se = form == 0 ? 1u : 0u;
  switch (K) {
    case 1: encode_coop_kernel<1><<<cgrid, dim3(kCT), 0, s>>>(in, in_off, in_bias, n, out, out_off, out_bias, t.code, t.len, se); break;
    case 2: encode_coop_kernel<2><<<cgrid, dim3(kCT), 0, s>>>(in, in_off, in_bias, n, out, out_off, out_bias, t.code, t.len, se); break;
    case 4: encode_coop_kernel<4><<<cgrid, dim3(kCT), 0, s>>>(in, in_off, in_bias, n, out, out_off, out_bias, t.code, t.len, se); break;
    default: encode_coop_kernel<8><<<cgrid, dim3(kCT), 0, s>>>(in, in_off, in_bias, n, out, out_off, out_bias, t.code, t.len, se); break;
  }
  return hipGetLastError();
}

}  // namespace mhq
