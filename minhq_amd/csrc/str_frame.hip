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

#include "huff_kernels.h"

namespace mhq {
namespace {

constexpr int kT = 256;

inline unsigned blocks(uint64_t n) { return (unsigned)((n + kT - 1) / kT); }

// Per-string parse state between the read kernels.
struct ReadScratch {
  uint64_t *start;  // payload start (byte index into blk)
  uint64_t *take;   // payload bytes inside the block (the LimitedReader, truncated at limit)
  uint64_t *declared;
  uint32_t *cap;    // output capacity: floor(8*take/5) (Huffman) or take (raw)
  uint32_t *hsz;    // Huffman payload bytes (0 for raw strings)
  uint8_t *kind;    // 0 raw, 1 Huffman, 2 header error (hc/io.go:74-81 return ("", nil))
};

// Reader.ReadBit + Reader.ReadInt(prefix) at byte pos, bit 7-prefix being the
// H bit, reading no byte at or past limit (hc/io.go:25-55, 73-81).
__global__ void read_parse_kernel(const uint8_t *__restrict__ blk, uint64_t blk_len, const uint64_t *__restrict__ pos,
                                  const uint64_t *__restrict__ limit, const uint8_t *__restrict__ prefix, uint64_t n,
                                  ReadScratch sc, uint64_t *__restrict__ next) {
  const uint64_t i = (uint64_t)blockIdx.x * kT + threadIdx.x;
  if (i >= n) return;
  // a limit past the block is the block's end: no byte past blk_len is read
  const uint64_t p0 = pos[i], lim = min(limit[i], blk_len);
  const uint32_t pf = prefix[i];
  uint8_t kind = 2;
  uint64_t start = p0, take = 0, v = 0;
  if (pf >= 1 && pf <= 7 && p0 < lim) {
    const uint32_t b0 = blk[p0];
    const uint32_t h = (b0 >> pf) & 1u;
    const uint64_t mask = (1ull << pf) - 1u;
    v = b0 & mask;
    uint64_t q = p0 + 1;
    bool ok = true;
    if (v == mask) {
      for (uint32_t s = 0; s < 64; s += 7) {
        if (q >= lim) {  // EOF inside the integer
          ok = false;
          break;
        }
        const uint64_t b = blk[q++];
        if (s == 63 && (b > 1 || (b == 1 && (v >> 63) == 1))) {  // ErrIntegerOverflow (hc/io.go:46)
          ok = false;
          break;
        }
        v += (b & 0x7f) << s;
        if ((b & 0x80) == 0) break;
      }
    }
    if (ok) {
      kind = (uint8_t)h;
      start = q;
      const uint64_t avail = lim - q;
      take = v < avail ? v : avail;
    }
  }
  sc.start[i] = start;
  sc.take[i] = take;
  sc.declared[i] = kind == 2 ? 0 : v;
  sc.kind[i] = kind;
  sc.cap[i] = kind == 1 ? (uint32_t)(take * 8 / 5) : (uint32_t)take;
  sc.hsz[i] = kind == 1 ? (uint32_t)take : 0u;
  next[i] = kind == 2 ? p0 : start + take;
}

// Offsets past a buffer's end become the end, so regions beyond it are empty.
__global__ void clamp_offsets_kernel(uint64_t *__restrict__ off, uint64_t n1, uint64_t limit) {
  const uint64_t i = (uint64_t)blockIdx.x * kT + threadIdx.x;
  if (i < n1 && off[i] > limit) off[i] = limit;
}

// Huffman payloads into the packed decode input (hin[hin_off[i]..]).
__global__ void gather_huff_kernel(const uint8_t *__restrict__ blk, ReadScratch sc, uint64_t n,
                                   const uint64_t *__restrict__ hin_off, uint8_t *__restrict__ hin) {
  const uint64_t i = (uint64_t)blockIdx.x * kT + threadIdx.x;
  if (i >= n || sc.kind[i] != 1) return;
  const uint64_t len = hin_off[i + 1] - hin_off[i];  // clamped: 0 when past the scratch
  const uint8_t *src = blk + sc.start[i];
  uint8_t *dst = hin + hin_off[i];
  for (uint64_t k = 0; k < len; k++) dst[k] = src[k];
}

// Raw payloads into the output (after the decode, which zero-fills the
// regions it stages), then the per-string outcome of hc/io.go:92-96.
__global__ void read_finish_kernel(const uint8_t *__restrict__ blk, ReadScratch sc, uint64_t n,
                                   const uint64_t *__restrict__ out_off, const uint64_t *__restrict__ hin_off,
                                   uint8_t *__restrict__ out, uint32_t *__restrict__ out_len,
                                   uint8_t *__restrict__ status) {
  const uint64_t i = (uint64_t)blockIdx.x * kT + threadIdx.x;
  if (i >= n) return;
  const uint8_t kind = sc.kind[i];
  const uint64_t room = out_off[i + 1] - out_off[i];
  uint8_t st = MHQ_STR_OK;
  uint32_t len = 0;
  if (kind == 2) {  // ReadBit / ReadInt failed: ("", nil)
  } else if (room < sc.cap[i] || hin_off[i + 1] - hin_off[i] < sc.hsz[i]) {
    // the output region, or the packed Huffman input (overlapping payloads
    // can total more than the block), was cut short by the buffer's end
    st = MHQ_STR_NOSPACE;
  } else if (kind == 1) {
    len = out_len[i];
    if (status[i] == MHQ_LIT_INVALID) {
      st = MHQ_STR_INVALID;  // ("", "invalid Huffman coding")
      len = 0;
    } else if (len == 0) {
      st = MHQ_STR_EOF;  // io.ReadFull into len*8/5+1 >= 1 bytes read nothing: io.EOF
    }
  } else {
    const uint64_t take = sc.take[i];
    if (take == 0 && sc.declared[i] > 0) {
      st = MHQ_STR_EOF;  // the block ended before the payload: io.EOF
    } else {
      const uint8_t *src = blk + sc.start[i];
      uint8_t *dst = out + out_off[i];
      for (uint64_t k = 0; k < take; k++) dst[k] = src[k];
      len = (uint32_t)take;
    }
  }
  out_len[i] = len;
  status[i] = st;
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
  for (uint64_t j = 0; j < L; j++) dst[k + j] = src[j];
  status[i] = MHQ_STR_OK;
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

hipError_t launch_read_strings(const DevTables &t, const uint8_t *blk, uint64_t blk_len, const uint64_t *pos,
                               const uint64_t *limit, const uint8_t *prefix, uint64_t n, uint8_t *out,
                               uint64_t out_cap, uint64_t *out_off, uint32_t *out_len, uint8_t *status,
                               uint64_t *next, hipStream_t s) {
  if (n == 0) {
    return hipMemsetAsync(out_off, 0, sizeof(uint64_t), s);
  }
  ReadScratch sc{};
  uint64_t *hin_off = nullptr;
  uint8_t *hin = nullptr;
  hipError_t e = hipSuccess;
#define TRY(x)                   \
  do {                           \
    e = (x);                     \
    if (e != hipSuccess) goto done; \
  } while (0)
  TRY(scratch(&sc.start, n, s));
  TRY(scratch(&sc.take, n, s));
  TRY(scratch(&sc.declared, n, s));
  TRY(scratch(&sc.cap, n, s));
  TRY(scratch(&sc.hsz, n, s));
  TRY(scratch(&sc.kind, n, s));
  TRY(scratch(&hin_off, n + 1, s));
  TRY(scratch(&hin, blk_len + 16, s));
  read_parse_kernel<<<blocks(n), kT, 0, s>>>(blk, blk_len, pos, limit, prefix, n, sc, next);
  TRY(hipGetLastError());
  // output regions: capacities back to back; the packed Huffman input
  TRY(launch_offsets(sc.cap, n, 0, out_off, nullptr, s));
  TRY(launch_offsets(sc.hsz, n, 0, hin_off, nullptr, s));
  clamp_offsets_kernel<<<blocks(n + 1), kT, 0, s>>>(out_off, n + 1, out_cap);
  clamp_offsets_kernel<<<blocks(n + 1), kT, 0, s>>>(hin_off, n + 1, blk_len);
  gather_huff_kernel<<<blocks(n), kT, 0, s>>>(blk, sc, n, hin_off, hin);
  TRY(hipGetLastError());
  TRY(launch_decode(t, hin, hin_off, 0, n, out, out_off, 0, out_len, status, s));
  read_finish_kernel<<<blocks(n), kT, 0, s>>>(blk, sc, n, out_off, hin_off, out, out_len, status);
  TRY(hipGetLastError());
done:
  (void)hipFreeAsync(sc.start, s);
  (void)hipFreeAsync(sc.take, s);
  (void)hipFreeAsync(sc.declared, s);
  (void)hipFreeAsync(sc.cap, s);
  (void)hipFreeAsync(sc.hsz, s);
  (void)hipFreeAsync(sc.kind, s);
  (void)hipFreeAsync(hin_off, s);
  (void)hipFreeAsync(hin, s);
  return e;
}

hipError_t launch_write_strings(const DevTables &t, const uint8_t *in, const uint64_t *in_off, uint64_t n,
                                const uint8_t *prefix, const uint8_t *lead, uint32_t choice, uint8_t *out,
                                uint64_t out_cap, uint64_t *out_off, uint8_t *status, hipStream_t s) {
  if (n == 0) {
    return hipMemsetAsync(out_off, 0, sizeof(uint64_t), s);
  }
  uint32_t *enc_len = nullptr, *frame = nullptr;
  uint64_t *enc_off = nullptr;
  uint8_t *enc = nullptr, *huff = nullptr;
  uint64_t enc_total = 0, base = 0;
  hipError_t e = hipSuccess;
  TRY(scratch(&enc_len, n, s));
  TRY(scratch(&frame, n, s));
  TRY(scratch(&enc_off, n + 1, s));
  TRY(scratch(&huff, n, s));
  TRY(launch_encode_len(t, in, in_off, 0, n, enc_len, s));
  TRY(hipMemcpyAsync(&base, in_off, sizeof(uint64_t), hipMemcpyDeviceToHost, s));
  TRY(launch_offsets(enc_len, n, 0, enc_off, nullptr, s));
  TRY(hipMemcpyAsync(&enc_total, enc_off + n, sizeof(uint64_t), hipMemcpyDeviceToHost, s));
  TRY(hipStreamSynchronize(s));
  TRY(scratch(&enc, enc_total + 16, s));
  TRY(launch_encode(t, in, in_off, 0, n, enc, enc_off, 0, s));
  write_size_kernel<<<blocks(n), kT, 0, s>>>(in_off, enc_len, prefix, choice, n, frame, huff);
  TRY(hipGetLastError());
  TRY(launch_offsets(frame, n, 0, out_off, nullptr, s));
  if (out) {
    write_frame_kernel<<<blocks(n), kT, 0, s>>>(in, in_off, enc, enc_off, prefix, lead, huff, n, out_off, out_cap,
                                                  out, status);
    TRY(hipGetLastError());
  }
done:
#undef TRY
  (void)hipFreeAsync(enc_len, s);
  (void)hipFreeAsync(frame, s);
  (void)hipFreeAsync(enc_off, s);
  (void)hipFreeAsync(enc, s);
  (void)hipFreeAsync(huff, s);
  (void)base;
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
