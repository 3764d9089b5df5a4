// str_frame.hip -- batch string-literal framing around the Huffman kernels.
//
// Reader.ReadString / Writer.WriteStringRaw (hc/io.go:73-97, 153-197) with
// the prefix integers of Reader.ReadInt / Writer.WriteInt (hc/io.go:25-55,
// 110-137), over batches of independent string literals.
// A string literal starts with an octet whose low prefix+1 bits are the H bit
// and the length prefix (the caller's opcode fills the bits above: 7/5/3-bit
// prefixes after 1/3/5-bit opcodes, hc/qpackdecoder.go:127,163,340), so every
// payload is a byte-aligned slice and the Huffman payloads batch straight
// into the decode/encode kernels.  The per-string parse and copy kernels here
// are integer/byte work with one thread per string.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <cstdlib>

#include "huff_common.h"
#include "huff_kernels.h"

namespace mhq {
namespace {

using namespace dev;

constexpr int kT = 256;

inline unsigned blocks(uint64_t n) { return (unsigned)((n + kT - 1) / kT); }

// Per-string parse state between the read kernels.
struct ReadScratch {
  uint64_t *start;  // payload start (byte index into blk); start[n] = blk_len (the decode's in_off)
  uint32_t *hend;   // low word of the Huffman payload end: start + take for a Huffman string, start
                    // otherwise (the decode's in_end)
  uint8_t *kind;    // 0 raw, 1 Huffman, 2 header error (hc/io.go:74-81 return ("", nil)); | kDeclared
};

// Reader.ReadBit + Reader.ReadInt(prefix) at byte pos, bit 7-prefix being the
// H bit, reading no byte at or past limit (hc/io.go:25-55, 73-81).
// Each block also writes the capacity sums of its strings, per kLenSumBlock,
// to block_sums: the offsets scan's first pass.
#ifndef MHQ_PARSE_PER  // strings per parse thread: i = block * kT * kParsePer + k * kT + tid (1, 4, 8: 1-4 % slower)
#define MHQ_PARSE_PER 2
#endif
constexpr int kParsePer = MHQ_PARSE_PER;

// Output regions (see launch_read_strings): string i's region starts at
// floor(8 * start_i / 5), its payload start scaled by the Huffman bound.  When
// the strings lie in block order (every payload ends at or before the next
// string's pos) these regions are disjoint, ordered and each holds
// floor(8 * take_i / 5) bytes, so no scan is needed; the kernel writes them
// to out_off and, if some string is out of order, stores `gen` to *order_bad
// (the scan's apply pass then lays the regions out back to back instead).
__device__ __forceinline__ uint64_t scaled(uint64_t x) { return x / 5u * 8u + (x % 5u) * 8u / 5u; }

__global__ __launch_bounds__(kT) void read_parse_kernel(const uint8_t *__restrict__ blk, uint64_t blk_len,
                                                        const uint64_t *__restrict__ pos,
                                                        const uint64_t *__restrict__ limit,
                                                        const uint8_t *__restrict__ prefix, uint64_t n,
                                                        ReadScratch sc, uint64_t *__restrict__ next,
                                                        uint64_t *__restrict__ block_sums,
                                                        uint64_t *__restrict__ out_off, uint64_t *order_bad,
                                                        uint64_t *finish_needed, uint64_t gen) {
  static_assert(kT == kLenSumBlock, "block sums per kLenSumBlock strings: one per k");
  // Every load of the thread's strings is issued before the first one is
  // used (the per-string chain pos -> header octet is two dependent loads).
  const uint64_t i0 = (uint64_t)blockIdx.x * (kT * kParsePer) + threadIdx.x;
  uint64_t p0[kParsePer], lim[kParsePer], pn[kParsePer];
  uint32_t pf[kParsePer], b0[kParsePer];
#pragma unroll
  for (int k = 0; k < kParsePer; k++) {
    const uint64_t i = i0 + (uint64_t)k * kT;
    const uint64_t j = i < n ? i : n - 1;  // (clamped: loads stay inside the arrays)
    p0[k] = pos[j];
    lim[k] = min(limit[j], blk_len);  // a limit past the block is the block's end: no byte past blk_len is read
    pf[k] = prefix[j];
    pn[k] = i + 1 < n ? pos[i + 1] : blk_len;  // the next string's pos (order test)
  }
#pragma unroll
  for (int k = 0; k < kParsePer; k++) b0[k] = p0[k] < lim[k] ? blk[p0[k]] : 0u;
  uint32_t caps[kParsePer];
  bool bad = false, raw = false;
#pragma unroll
  for (int k = 0; k < kParsePer; k++) {
    const uint64_t i = i0 + (uint64_t)k * kT;
    caps[k] = 0;
    if (i >= n) continue;
    uint8_t kind = 2;
    uint64_t start = p0[k], take = 0, v = 0;
    if (pf[k] >= 1 && pf[k] <= 7 && p0[k] < lim[k]) {
      const uint32_t h = (b0[k] >> pf[k]) & 1u;
      const uint64_t mask = (1ull << pf[k]) - 1u;
      v = b0[k] & mask;
      uint64_t q = p0[k] + 1;
      bool ok = true;
      if (v == mask) {
        for (uint32_t sh = 0; sh < 64; sh += 7) {
          if (q >= lim[k]) {  // EOF inside the integer
            ok = false;
            break;
          }
          const uint64_t b = blk[q++];
          if (sh == 63 && (b > 1 || (b == 1 && (v >> 63) == 1))) {  // ErrIntegerOverflow (hc/io.go:46)
            ok = false;
            break;
          }
          v += (b & 0x7f) << sh;
          if ((b & 0x80) == 0) break;
        }
      }
      if (ok) {
        kind = (uint8_t)h;
        start = q;
        const uint64_t avail = lim[k] - q;
        take = v < avail ? v : avail;
      }
    }
    // the decode reads literal i from blk + start: a header-error string's
    // pos may lie anywhere (even past the block), so its (empty) payload is
    // placed at min(pos, blk_len) -- every start stays inside [0, blk_len]
    start = start < blk_len ? start : blk_len;
    sc.start[i] = start;
    sc.hend[i] = (uint32_t)(kind == 1 ? start + take : start);
    if (i == n - 1) sc.start[n] = blk_len;
    sc.kind[i] = kind | (kind != 2 && v != 0 ? kDeclared : 0);
    caps[k] = kind == 1 ? (uint32_t)(take * 8 / 5) : (uint32_t)take;
    raw |= kind == 0;
    next[i] = kind == 2 ? p0[k] : start + take;
    // the region at the scaled payload start; in block order the next one
    // starts at or after scaled(start + take) (its payload starts after its
    // pos, which is at or after this payload's end)
    out_off[i] = scaled(start);
    if (i == n - 1) out_off[n] = scaled(blk_len);
    bad |= start + take > min(pn[k], blk_len);
  }
  if (bad) *order_bad = gen;  // (rare: every writer stores the same value)
  if (raw) *finish_needed = gen;  // raw payloads to copy: the decode finishes its ranges
  // (sum of cap, sum of cap) per kLenSumBlock strings: group k of this block
  __shared__ uint64_t part[kParsePer][kT / 64];
  const uint32_t lane = threadIdx.x % 64, wave = threadIdx.x / 64;
#pragma unroll
  for (int k = 0; k < kParsePer; k++) {
    uint64_t a = caps[k];
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) a += __shfl_xor(a, d);
    if (lane == 0) part[k][wave] = a;
  }
  __syncthreads();
  if (threadIdx.x < kParsePer) {
    const uint64_t g = (uint64_t)blockIdx.x * kParsePer + threadIdx.x;
    if (g * kT < n) {
      uint64_t v = 0;
#pragma unroll
      for (int w = 0; w < kT / 64; w++) v += part[threadIdx.x][w];
      block_sums[2 * g] = v;
      block_sums[2 * g + 1] = v;
    }
  }
}



// ---- write side ----------------------------------------------------------

__device__ __forceinline__ uint32_t int_bytes(uint64_t v, uint32_t pf) {  // Writer.WriteInt octets after the first
  const uint64_t ones = (1ull << pf) - 1u;
  if (v < ones) return 0;
  v -= ones;
  uint32_t k = 1;
  while (v >= 0x80) {
    v >>= 7;
    k++;
  }
  return k;
}

// Huffman iff Always, or Auto and strictly shorter (hc/io.go:172); the frame
// is the H/prefix octet, the integer's continuation octets and the payload.
__global__ void write_size_kernel(const uint64_t *__restrict__ in_off, const uint32_t *__restrict__ enc_len,
                                  const uint8_t *__restrict__ prefix, uint32_t choice, uint64_t n,
                                  uint32_t *__restrict__ frame, uint8_t *__restrict__ huff) {
  const uint64_t i = (uint64_t)blockIdx.x * kT + threadIdx.x;
  if (i >= n) return;
  const uint64_t raw = in_off[i + 1] - in_off[i];
  const uint32_t enc = enc_len[i];
  const bool h = choice == MHQ_HUFF_ALWAYS || (choice == MHQ_HUFF_AUTO && (uint64_t)enc < raw);
  const uint64_t L = h ? enc : raw;
  frame[i] = (uint32_t)(1u + int_bytes(L, prefix[i]) + L);
  huff[i] = h;
}

__global__ void write_frame_kernel(const uint8_t *__restrict__ in, const uint64_t *__restrict__ in_off,
                                   const uint8_t *__restrict__ enc, const uint64_t *__restrict__ enc_off,
                                   const uint8_t *__restrict__ prefix, const uint8_t *__restrict__ lead,
                                   const uint8_t *__restrict__ huff, uint64_t n, const uint64_t *__restrict__ out_off,
                                   uint64_t out_cap, uint8_t *__restrict__ out, uint8_t *__restrict__ status) {
  const uint64_t i = (uint64_t)blockIdx.x * kT + threadIdx.x;
  if (i >= n) return;
  if (out_off[i + 1] > out_cap) {
    status[i] = MHQ_STR_NOSPACE;
    return;
  }
  const uint32_t pf = prefix[i];
  const bool h = huff[i];
  const uint8_t *src = h ? enc + enc_off[i] : in + in_off[i];
  const uint64_t L = h ? enc_off[i + 1] - enc_off[i] : in_off[i + 1] - in_off[i];
  uint8_t *dst = out + out_off[i];
  const uint64_t ones = (1ull << pf) - 1u;
  // the opcode bits, the H bit, the prefix (hc/io.go:181-185, 110-137)
  uint32_t b0 = ((uint32_t)lead[i] << (pf + 1)) | ((uint32_t)h << pf);
  uint64_t k = 0;
  if (L < ones) {
    dst[k++] = (uint8_t)(b0 | (uint32_t)L);
  } else {
    dst[k++] = (uint8_t)(b0 | (uint32_t)ones);
    uint64_t p = L - ones;
    for (bool done = false; !done;) {
      uint32_t b = (uint32_t)(p & 0x7f);
      p >>= 7;
      if (p > 0) b |= 0x80;
      else done = true;
      dst[k++] = (uint8_t)b;
    }
  }
  copy_bytes(dst + k, src, L);
  status[i] = MHQ_STR_OK;
}

// The Huffman payloads the frames will hold: enc_len[i] for a Huffman string
// whose frame fits the output, 0 otherwise (those are not encoded at all), so
// the packed encodings total at most out_cap bytes.
__global__ void write_mask_kernel(const uint32_t *__restrict__ enc_len, const uint8_t *__restrict__ huff,
                                  const uint64_t *__restrict__ out_off, uint64_t out_cap, uint64_t n,
                                  uint32_t *__restrict__ mlen) {
  const uint64_t i = (uint64_t)blockIdx.x * kT + threadIdx.x;
  if (i >= n) return;
  mlen[i] = huff[i] && out_off[i + 1] <= out_cap ? enc_len[i] : 0u;
}

// ---- prefix integers -----------------------------------

// Reader.ReadInt(prefix) at byte pos, the integer's prefix in the low prefix
// bits of that octet, reading no byte at or past limit (hc/io.go:25-55).  The
// caller's opcode owns the bits above the prefix.  MHQ_INT_EOF where ReadBits
// would meet the end of the block, MHQ_INT_OVERFLOW where ReadInt returns
// ErrIntegerOverflow (hc/io.go:46); with `index` set, a value above the
// largest int is ErrIntegerOverflow too (ReadIndex, hc/io.go:59-67).
__global__ void read_ints_kernel(const uint8_t *__restrict__ blk, const uint64_t *__restrict__ pos,
                                 const uint64_t *__restrict__ limit, const uint8_t *__restrict__ prefix, uint64_t n,
                                 uint32_t index, uint64_t *__restrict__ value, uint64_t *__restrict__ next,
                                 uint8_t *__restrict__ status) {
  const uint64_t i = (uint64_t)blockIdx.x * kT + threadIdx.x;
  if (i >= n) return;
  const uint64_t p0 = pos[i], lim = limit[i];
  const uint32_t pf = prefix[i];
  uint8_t st = MHQ_INT_OK;
  uint64_t v = 0, q = p0;
  if (pf < 1 || pf > 8) {
    st = MHQ_INT_BADARG;
  } else if (p0 >= lim) {
    st = MHQ_INT_EOF;
  } else {
    const uint64_t mask = (1ull << pf) - 1u;
    v = blk[q++] & mask;
    if (v == mask) {
      for (uint32_t s = 0; s < 64; s += 7) {
        if (q >= lim) {
          st = MHQ_INT_EOF;
          break;
        }
        const uint64_t b = blk[q++];
        if (s == 63 && (b > 1 || (b == 1 && (v >> 63) == 1))) {
          st = MHQ_INT_OVERFLOW;
          break;
        }
        v += (b & 0x7f) << s;
        if ((b & 0x80) == 0) break;
      }
    }
    if (st == MHQ_INT_OK && index && (v >> 63)) st = MHQ_INT_OVERFLOW;
  }
  value[i] = st == MHQ_INT_OK ? v : 0u;
  next[i] = st == MHQ_INT_OK ? q : p0;
  status[i] = st;
}

__global__ void write_ints_size_kernel(const uint64_t *__restrict__ value, const uint8_t *__restrict__ prefix,
                                       uint64_t n, uint32_t *__restrict__ size) {
  const uint64_t i = (uint64_t)blockIdx.x * kT + threadIdx.x;
  if (i >= n) return;
  const uint32_t pf = prefix[i];
  size[i] = pf >= 1 && pf <= 8 ? 1u + int_bytes(value[i], pf) : 0u;
}

// Writer.WriteInt(v, prefix) after the opcode bits lead[i] (hc/io.go:110-137).
__global__ void write_ints_kernel(const uint64_t *__restrict__ value, const uint8_t *__restrict__ prefix,
                                  const uint8_t *__restrict__ lead, uint64_t n, const uint64_t *__restrict__ out_off,
                                  uint64_t out_cap, uint8_t *__restrict__ out, uint8_t *__restrict__ status) {
  const uint64_t i = (uint64_t)blockIdx.x * kT + threadIdx.x;
  if (i >= n) return;
  const uint32_t pf = prefix[i];
  if (pf < 1 || pf > 8) {
    status[i] = MHQ_INT_BADARG;
    return;
  }
  if (out_off[i + 1] > out_cap) {
    status[i] = MHQ_INT_NOSPACE;
    return;
  }
  uint8_t *dst = out + out_off[i];
  const uint64_t ones = (1ull << pf) - 1u;
  const uint32_t b0 = pf == 8 ? 0u : ((uint32_t)lead[i] << pf);
  uint64_t v = value[i];
  if (v < ones) {
    dst[0] = (uint8_t)(b0 | (uint32_t)v);
  } else {
    dst[0] = (uint8_t)(b0 | (uint32_t)ones);
    v -= ones;
    uint64_t k = 1;
    for (bool done = false; !done;) {
      uint32_t b = (uint32_t)(v & 0x7f);
      v >>= 7;
      if (v > 0) b |= 0x80;
      else done = true;
      dst[k++] = (uint8_t)b;
    }
  }
  status[i] = MHQ_INT_OK;
}

// ---- HTTP/3 (draft) frame varints ---------------------

// ReadVarint at byte pos (frame.go:72-79): the top two bits of the first
// octet give the length (1, 2, 4 or 8 octets), the rest is the value, MSB
// first.  MHQ_VARINT_EOF where ReadBits meets the end of the block.
__device__ __forceinline__ uint8_t read_varint_at(const uint8_t *__restrict__ blk, uint64_t p0, uint64_t lim,
                                                  uint64_t &v, uint64_t &q) {
  v = 0;
  q = p0;
  if (p0 >= lim) return MHQ_VARINT_EOF;
  const uint32_t b0 = blk[p0];
  const uint32_t nb = 1u << (b0 >> 6);
  if (p0 + nb > lim) return MHQ_VARINT_EOF;
  uint64_t x = b0 & 0x3fu;
  for (uint32_t k = 1; k < nb; k++) x = (x << 8) | blk[p0 + k];
  v = x;
  q = p0 + nb;
  return MHQ_VARINT_OK;
}

__global__ void read_varints_kernel(const uint8_t *__restrict__ blk, const uint64_t *__restrict__ pos,
                                    const uint64_t *__restrict__ limit, uint64_t n, uint64_t *__restrict__ value,
                                    uint64_t *__restrict__ next, uint8_t *__restrict__ status) {
  const uint64_t i = (uint64_t)blockIdx.x * kT + threadIdx.x;
  if (i >= n) return;
  uint64_t v, q;
  status[i] = read_varint_at(blk, pos[i], limit[i], v, q);
  value[i] = v;
  next[i] = q;
}

// ReadFrame's header (frame.go:81-92): the payload length as a varint, then
// the type octet; the payload is the next `len` octets.
__global__ void read_frames_kernel(const uint8_t *__restrict__ blk, const uint64_t *__restrict__ pos,
                                   const uint64_t *__restrict__ limit, uint64_t n, uint8_t *__restrict__ type,
                                   uint64_t *__restrict__ payload_len, uint64_t *__restrict__ payload_pos,
                                   uint8_t *__restrict__ status) {
  const uint64_t i = (uint64_t)blockIdx.x * kT + threadIdx.x;
  if (i >= n) return;
  const uint64_t lim = limit[i];
  uint64_t v, q;
  uint8_t st = read_varint_at(blk, pos[i], lim, v, q);
  uint8_t t = 0;
  if (st == MHQ_VARINT_OK) {
    if (q >= lim) {
      st = MHQ_VARINT_EOF;
      v = 0;
    } else {
      t = blk[q++];
    }
  }
  type[i] = t;
  payload_len[i] = st == MHQ_VARINT_OK ? v : 0u;
  payload_pos[i] = st == MHQ_VARINT_OK ? q : pos[i];
  status[i] = st;
}

// WriteVarint (frame.go:128-152): the shortest of 1, 2, 4, 8 octets;
// values >= 2^62 are ErrTooLarge (no octets).
__global__ void write_varints_size_kernel(const uint64_t *__restrict__ value, uint64_t n, uint32_t *__restrict__ size) {
  const uint64_t i = (uint64_t)blockIdx.x * kT + threadIdx.x;
  if (i >= n) return;
  const uint64_t v = value[i];
  size[i] = v >= (1ull << 62) ? 0u : v >= (1ull << 30) ? 8u : v >= (1ull << 14) ? 4u : v >= (1ull << 6) ? 2u : 1u;
}

__global__ void write_varints_kernel(const uint64_t *__restrict__ value, uint64_t n,
                                     const uint64_t *__restrict__ out_off, uint64_t out_cap,
                                     uint8_t *__restrict__ out, uint8_t *__restrict__ status) {
  const uint64_t i = (uint64_t)blockIdx.x * kT + threadIdx.x;
  if (i >= n) return;
  const uint64_t v = value[i];
  if (v >= (1ull << 62)) {
    status[i] = MHQ_VARINT_TOO_LARGE;
    return;
  }
  if (out_off[i + 1] > out_cap) {
    status[i] = MHQ_VARINT_NOSPACE;
    return;
  }
  const uint32_t nb = (uint32_t)(out_off[i + 1] - out_off[i]);
  const uint64_t code = nb == 8 ? 3u : nb == 4 ? 2u : nb == 2 ? 1u : 0u;
  const uint64_t x = v | (code << (8u * nb - 2u));
  uint8_t *dst = out + out_off[i];
  for (uint32_t k = 0; k < nb; k++) dst[k] = (uint8_t)(x >> (8u * (nb - 1u - k)));
  status[i] = MHQ_VARINT_OK;
}

template <class T>
hipError_t scratch(T **p, uint64_t count, hipStream_t s) {
  return hipMallocAsync((void **)p, (count ? count : 1) * sizeof(T), s);
}

}  // namespace

namespace {

// read_strings' scratch, 16-B aligned pieces of one allocation.
struct ReadLayout {
  size_t start, hend, kind, flags, sums, coop, total;
  ReadLayout(uint64_t n, uint64_t blk_len) {
    size_t o = 0;
    auto take_ = [&](size_t bytes) {
      const size_t at = o;
      o += (bytes + 15) & ~(size_t)15;
      return at;
    };
    start = take_(8 * (n + 1));
    hend = take_(4 * n);
    kind = take_(n);
    flags = take_(24);  // order_bad, finish_needed, fallback (the fused pass)
    sums = take_(offsets_sums_scratch_bytes(n));
    coop = take_(8 * 2 * kReadFallbackMaxWgs);  // the fused read's fallback: workgroup sums, raw flags
    total = o;
  }
};

}  // namespace

// Test hook (MHQ_DEBUG_POISON_SCRATCH set in the environment): stale scratch
// contents that could once be mistaken for this call's flags.  The fallback
// word gets gen with its high half inverted (its low word equals gen's low
// word: the round-4 fused pass compared only that), and every look-back slot
// a capacity sum under the round-4 tag of gen (gen's low 24 bits).  The
// whole-word compare and the cleared, never-zero tags make both harmless
// (tests/test_strings.py::test_read_poisoned_scratch).
__global__ void read_poison_kernel(uint64_t *fallback, uint64_t *wg_agg, uint64_t gen) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i == 0) *fallback = gen ^ 0xffffffff00000000ull;
  if (i < kReadFallbackMaxWgs) wg_agg[i] = ((gen & 0xffffffull) << 40) | (12345u + 7u * i);
}

#ifndef MHQ_RS_FUSED  // read_strings: 1 the one-pass kernel, the multi-pass pipeline as its fallback
#define MHQ_RS_FUSED 1
#endif
constexpr bool kFused = MHQ_RS_FUSED;

size_t read_strings_scratch_bytes(uint64_t n, uint64_t blk_len) { return ReadLayout(n, blk_len).total; }

// parse (+ block sums, + the output regions at the scaled payload starts) ->
// only if some string lies out of block order: one scan of the capacities
// into out_off (regions back to back), clamped to the output -> decode of the
// Huffman payloads where they lie in the block (launch_decode with in_end),
// which also finishes every string (StrFinish: the Huffman outcome, raw
// payloads, cut regions).  The scan's apply pass is always launched but returns at once
// unless parse stored this call's generation number to order_bad (a number
// no earlier call used: no reset, and stale scratch contents can only cause
// the always-correct scan).
std::atomic<int> debug_poison_scratch{0};  // mhq_debug_poison_scratch (test hook)

hipError_t launch_read_strings(const DevTables &t, const uint8_t *blk, uint64_t blk_len, const uint64_t *pos,
                               const uint64_t *limit, const uint8_t *prefix, uint64_t n, uint8_t *out,
                               uint64_t out_cap, uint64_t *out_off, uint32_t *out_len, uint8_t *status,
                               uint64_t *next, hipStream_t s, void *scratch) {
  if (n == 0) {
    return hipMemsetAsync(out_off, 0, sizeof(uint64_t), s);
  }
  const ReadLayout L(n, blk_len);
  uint8_t *base = (uint8_t *)scratch;
  hipError_t e = hipSuccess;
  if (!base && (e = hipMallocAsync((void **)&base, L.total, s)) != hipSuccess) return e;
  ReadScratch sc{(uint64_t *)(base + L.start), (uint32_t *)(base + L.hend), base + L.kind};
  uint64_t *order_bad = (uint64_t *)(base + L.flags), *finish_needed = order_bad + 1, *fallback = order_bad + 2;
  // (one generation number per call: the flags are set by storing it, never
  // cleared, so a stale scratch cannot gate this call's passes)
  static std::atomic<uint64_t> g_gen{0};
  const uint64_t gen = 0x6d68712000000000ull + g_gen.fetch_add(1, std::memory_order_relaxed) + 1;
#define TRY(x)                   \
  do {                           \
    e = (x);                     \
    if (e != hipSuccess) goto done; \
  } while (0)
  // MHQ_RS_FUSED: one pass (launch_read_fused), then its fallback, one
  // launch that returns at once unless the pass stored gen to *fallback
  if (kFused) {
    uint64_t *coop = (uint64_t *)(base + L.coop);
    if (debug_poison_scratch.load(std::memory_order_relaxed)) {
      read_poison_kernel<<<(kReadFallbackMaxWgs + 255) / 256, 256, 0, s>>>(fallback, coop, gen);
      TRY(hipGetLastError());
    }
    TRY(launch_read_fused(t, blk, blk_len, pos, limit, prefix, n, out, out_off, out_len, status, next, sc.start,
                          sc.hend, sc.kind, fallback, coop, gen, s));
    TRY(launch_read_fallback(t, blk, blk_len, pos, limit, prefix, n, out, out_cap, out_off, out_len, status, next,
                             sc.start, sc.hend, sc.kind, fallback, coop, coop + kReadFallbackMaxWgs, gen, s));
    goto done;
  }
  read_parse_kernel<<<(unsigned)((n + kT * kParsePer - 1) / (kT * kParsePer)), kT, 0, s>>>(
      blk, blk_len, pos, limit, prefix, n, sc, next, (uint64_t *)(base + L.sums), out_off, order_bad, finish_needed,
      gen);
  TRY(hipGetLastError());
  // strings out of block order: capacities back to back instead
  TRY(launch_read_caps_sums(sc.start, sc.hend, next, sc.kind, n, (uint64_t *)(base + L.sums), out_cap, out_off, s,
                            order_bad, gen));
  {
    // the decode also finishes each string (StrFinish): the Huffman outcome
    // at every length it writes, then raw payloads, raw EOFs and cut regions
    // per workgroup range when the parse flagged a raw string or the output
    // is cut
    StrFinish fin;
    fin.kind = sc.kind;
    fin.start = sc.start;
    fin.next = next;
    fin.hend = sc.hend;
    fin.blk = blk;
    fin.out_cap = out_cap;
    fin.finish_needed = finish_needed;
    fin.gen = gen;
    TRY(launch_decode(t, blk, sc.start, 0, n, out, out_off, 0, out_len, status, s, sc.hend, &fin));
  }
done:
  if (!scratch) {
    const hipError_t e2 = hipFreeAsync(base, s);
    if (e == hipSuccess) e = e2;
  }
  return e;
}

namespace {

struct WriteLayout {  // write_strings' scratch, 16-B aligned pieces of one allocation
  size_t enc_len, frame, mlen, huff, enc_off, sums, enc, total;
  WriteLayout(uint64_t n, uint64_t out_cap) {
    size_t o = 0;
    auto take_ = [&](size_t bytes) {
      const size_t at = o;
      o += (bytes + 15) & ~(size_t)15;
      return at;
    };
    enc_len = take_(4 * n);
    frame = take_(4 * n);
    mlen = take_(4 * n);
    huff = take_(n);
    enc_off = take_(8 * (n + 1));
    sums = take_(offsets_scratch_bytes(n));
    enc = take_(out_cap + 16);
    total = o;
  }
};

}  // namespace

size_t write_strings_scratch_bytes(uint64_t n, uint64_t out_cap) { return WriteLayout(n, out_cap).total; }

// encode_len -> choice and frame sizes -> frame offsets -> the Huffman
// payloads that will be written, packed (at most out_cap bytes: no size has
// to come back to the host, so no synchronisation) -> encode of just those ->
// frames.
hipError_t launch_write_strings(const DevTables &t, const uint8_t *in, const uint64_t *in_off, uint64_t n,
                                const uint8_t *prefix, const uint8_t *lead, uint32_t choice, uint8_t *out,
                                uint64_t out_cap, uint64_t *out_off, uint8_t *status, hipStream_t s,
                                void *scratch) {
  if (n == 0) {
    return hipMemsetAsync(out_off, 0, sizeof(uint64_t), s);
  }
  // without an output only the offsets are wanted: no room for encodings
  const WriteLayout L(n, out ? out_cap : 0);
  uint8_t *base = (uint8_t *)scratch;
  hipError_t e = hipSuccess;
  if (!base && (e = hipMallocAsync((void **)&base, L.total, s)) != hipSuccess) return e;
  uint32_t *enc_len = (uint32_t *)(base + L.enc_len), *frame = (uint32_t *)(base + L.frame);
  uint32_t *mlen = (uint32_t *)(base + L.mlen);
  uint8_t *huff = base + L.huff, *enc = base + L.enc;
  uint64_t *enc_off = (uint64_t *)(base + L.enc_off);
  void *sums = base + L.sums;
  TRY(launch_encode_len(t, in, in_off, 0, n, enc_len, s));
  write_size_kernel<<<blocks(n), kT, 0, s>>>(in_off, enc_len, prefix, choice, n, frame, huff);
  TRY(hipGetLastError());
  TRY(launch_offsets(frame, n, 0, out_off, nullptr, s, sums));
  if (out) {
    write_mask_kernel<<<blocks(n), kT, 0, s>>>(enc_len, huff, out_off, out_cap, n, mlen);
    TRY(hipGetLastError());
    TRY(launch_offsets(mlen, n, 0, enc_off, nullptr, s, sums));
    TRY(launch_encode(t, in, in_off, 0, n, enc, enc_off, 0, s));
    write_frame_kernel<<<blocks(n), kT, 0, s>>>(in, in_off, enc, enc_off, prefix, lead, huff, n, out_off, out_cap,
                                                  out, status);
    TRY(hipGetLastError());
  }
done:
#undef TRY
  if (!scratch) {
    const hipError_t e2 = hipFreeAsync(base, s);
    if (e == hipSuccess) e = e2;
  }
  return e;
}

hipError_t launch_read_ints(const uint8_t *blk, const uint64_t *pos, const uint64_t *limit, const uint8_t *prefix,
                            uint64_t n, int index, uint64_t *value, uint64_t *next, uint8_t *status, hipStream_t s) {
  if (n == 0) return hipSuccess;
  read_ints_kernel<<<blocks(n), kT, 0, s>>>(blk, pos, limit, prefix, n, index ? 1u : 0u, value, next, status);
  return hipGetLastError();
}

hipError_t launch_write_ints(const uint64_t *value, const uint8_t *prefix, const uint8_t *lead, uint64_t n,
                             uint8_t *out, uint64_t out_cap, uint64_t *out_off, uint8_t *status, hipStream_t s) {
  if (n == 0) return hipMemsetAsync(out_off, 0, sizeof(uint64_t), s);
  uint32_t *size = nullptr;
  hipError_t e = scratch(&size, n, s);
  if (e != hipSuccess) return e;
  write_ints_size_kernel<<<blocks(n), kT, 0, s>>>(value, prefix, n, size);
  e = hipGetLastError();
  if (e == hipSuccess) e = launch_offsets(size, n, 0, out_off, nullptr, s);
  if (e == hipSuccess && out) {
    write_ints_kernel<<<blocks(n), kT, 0, s>>>(value, prefix, lead, n, out_off, out_cap, out, status);
    e = hipGetLastError();
  }
  (void)hipFreeAsync(size, s);
  return e;
}

hipError_t launch_read_varints(const uint8_t *blk, const uint64_t *pos, const uint64_t *limit, uint64_t n,
                               uint64_t *value, uint64_t *next, uint8_t *status, hipStream_t s) {
  if (n == 0) return hipSuccess;
  read_varints_kernel<<<blocks(n), kT, 0, s>>>(blk, pos, limit, n, value, next, status);
  return hipGetLastError();
}

hipError_t launch_read_frames(const uint8_t *blk, const uint64_t *pos, const uint64_t *limit, uint64_t n,
                              uint8_t *type, uint64_t *payload_len, uint64_t *payload_pos, uint8_t *status,
                              hipStream_t s) {
  if (n == 0) return hipSuccess;
  read_frames_kernel<<<blocks(n), kT, 0, s>>>(blk, pos, limit, n, type, payload_len, payload_pos, status);
  return hipGetLastError();
}

hipError_t launch_write_varints(const uint64_t *value, uint64_t n, uint8_t *out, uint64_t out_cap,
                                uint64_t *out_off, uint8_t *status, hipStream_t s) {
  if (n == 0) return hipMemsetAsync(out_off, 0, sizeof(uint64_t), s);
  uint32_t *size = nullptr;
  hipError_t e = scratch(&size, n, s);
  if (e != hipSuccess) return e;
  write_varints_size_kernel<<<blocks(n), kT, 0, s>>>(value, n, size);
  e = hipGetLastError();
  if (e == hipSuccess) e = launch_offsets(size, n, 0, out_off, nullptr, s);
  if (e == hipSuccess && out) {
    write_varints_kernel<<<blocks(n), kT, 0, s>>>(value, n, out_off, out_cap, out, status);
    e = hipGetLastError();
  }
  (void)hipFreeAsync(size, s);
  return e;
}

}  // namespace mhq
