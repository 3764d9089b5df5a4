// huff_encode.hip -- gfx950 batch encode of RFC 7541 Huffman literals.
//
// Semantics: HuffmanCompressor.Write + Pad (hc/huffman.go:23-37) over
// bitWriter (io/bitio.go:72-149): codes MSB-first, the last octet padded with
// 1 bits; encode_len is ceil(sum of code lengths / 8), the size the Auto
// choice compares with the raw length (hc/io.go:172).
//
// Structure (one workgroup = kWaves wave64s, the code table in LDS): each
// wave walks tiles of kTileLits literals staged in its LDS slice.  A tile's
// bytes are processed in rounds of 1 KiB: lane l takes the 16-byte chunk
// 64r + l, looks up the 16 codes, and a wave prefix sum of the chunk bit
// totals places every byte's code in the tile's bit stream (S = running sum
// of code lengths over the tile).  A literal's bit offset is S minus S at its
// first byte, so a lane never waits for another lane's bytes: the work is
// perfectly balanced whatever the literal lengths.  Output words are
// assembled in registers and OR-ed into the zeroed staging area (words at
// chunk and literal boundaries are shared), then written back with aligned
// 16-B stores.
#include <hip/hip_runtime.h>

#include "huff_common.h"
#include "huff_kernels.h"
#include "huff_table.h"

namespace mhq {
namespace {

using namespace dev;

constexpr int kWaves = 8;
constexpr int kThreads = kWave * kWaves;
constexpr int kTileLits = 256;
constexpr int kInCap = 6144;   // staged input bytes per wave (incl. 16-B alignment slack)
constexpr int kOutCap = 6144;  // staged output bytes per wave (encode only)
constexpr int kChunks = kInCap / 16;

struct WaveSmem {
  uint32_t in_w[kInCap / 4];
  uint32_t out_w[kOutCap / 4 + 4];
  uint2 rec[kTileLits + 2];   // per boundary: (input byte index, output byte index)
  uint32_t sstart[kTileLits]; // S at the literal's first byte
  uint32_t obits[kTileLits];  // encoded bits per literal (encode_len)
  uint16_t lit_at[kChunks];   // literal holding the first byte of each chunk
};
struct Smem {
  uint2 code[256];  // (code left-aligned in 32 bits, length)
  WaveSmem w[kWaves];
};

// Appends `len` bits (MSB-aligned in `cla`) at bit position bp of the LDS
// word stream `ow`; acc holds this lane's bits of word bp>>5 (MSB-aligned in
// its upper half).  Complete words are OR-ed out.
__device__ __forceinline__ void put_bits(uint32_t *ow, uint64_t &acc, uint32_t &bp, uint32_t cla, uint32_t len) {
  const uint32_t sh = bp & 31u;
  acc |= ((uint64_t)cla << 32) >> sh;
  if (sh + len >= 32u) {
    atomicOr(&ow[bp >> 5], __builtin_bswap32((uint32_t)(acc >> 32)));
    acc <<= 32;
  }
  bp += len;
}

// OR-s out the partial word at bp (if any bits of it are pending).
__device__ __forceinline__ void put_flush(uint32_t *ow, uint64_t acc, uint32_t bp) {
  if (bp & 31u) atomicOr(&ow[bp >> 5], __builtin_bswap32((uint32_t)(acc >> 32)));
}

template <bool kEmit>
__global__ __launch_bounds__(kThreads) void encode_kernel(
    const uint8_t *__restrict__ in, const uint64_t *__restrict__ in_off, uint64_t in_bias, uint64_t n,
    uint8_t *__restrict__ out, const uint64_t *__restrict__ out_off, uint64_t out_bias,
    uint32_t *__restrict__ enc_len, const uint32_t *__restrict__ g_code, const uint8_t *__restrict__ g_len,
    uint64_t ntiles) {
  __shared__ Smem sm;
  const int tid = threadIdx.x;
  const int wave = __builtin_amdgcn_readfirstlane(tid / kWave);
  const int lane = tid % kWave;
  for (int i = tid; i < 256; i += kThreads) {
    const uint32_t L = g_len[i];
    sm.code[i] = make_uint2(g_code[i] << (32u - L), L);
  }
  __syncthreads();
  WaveSmem &ws = sm.w[wave];
  const uint64_t stride = (uint64_t)gridDim.x * kWaves;

  for (uint64_t t = (uint64_t)blockIdx.x * kWaves + wave; t < ntiles; t += stride) {
    const uint64_t s = t * kTileLits;
    const uint32_t cnt = (uint32_t)min((uint64_t)kTileLits, n - s);
    TileOffsets<kTileLits> off;
    off.load(in_off, kEmit ? out_off : nullptr, s, cnt, lane);
    uint32_t cur = 0;
    while (cur < cnt) {
      const uint64_t ic = in_off[s + cur];
      const uint64_t oc = kEmit ? out_off[s + cur] : 0;
      const uint8_t *ia = in + (ic - in_bias);
      uint8_t *oa = kEmit ? out + (oc - out_bias) : nullptr;
      const uint32_t idelta = (uint32_t)((uintptr_t)ia & 15u);
      const uint32_t odelta = kEmit ? (uint32_t)((uintptr_t)oa & 15u) : 0u;
      const uint32_t end = off.fit(cur, cnt, ic, kInCap - idelta, oc, kEmit ? kOutCap - odelta : ~0ull, lane);
      if (end == cur) {  // one literal larger than the slice: lane 0 walks it in global memory
        if (lane == 0) {
          const uint64_t L = in_off[s + cur + 1] - ic;
          if (kEmit) {
            const uint64_t cap = out_off[s + cur + 1] - oc;
            uint64_t acc = 0, o = 0;
            uint32_t nacc = 0;
            for (uint64_t i = 0; i < L; i++) {
              const uint2 cl = sm.code[ia[i]];
              acc = (acc << cl.y) | (cl.x >> (32u - cl.y));
              nacc += cl.y;
              while (nacc >= 8) {
                nacc -= 8;
                if (o < cap) oa[o] = (uint8_t)(acc >> nacc);
                o++;
              }
            }
            if (nacc && o < cap) oa[o] = (uint8_t)((acc << (8 - nacc)) | ((1u << (8 - nacc)) - 1u));
          } else {
            uint64_t bits = 0;
            for (uint64_t i = 0; i < L; i++) bits += sm.code[ia[i]].y;
            enc_len[s + cur] = (uint32_t)((bits + 7u) >> 3);
          }
        }
        cur++;
        continue;
      }
      const uint32_t m = end - cur;
#pragma unroll
      for (int k = 0; k < TileOffsets<kTileLits>::kPer; k++) {
        const uint32_t j = (uint32_t)lane + (uint32_t)k * kWave;
        if (j >= cur && j <= end)
          ws.rec[j - cur] = make_uint2((uint32_t)(off.io[k] - ic) + idelta,
                                       kEmit ? (uint32_t)(off.oo[k] - oc) + odelta : 0u);
      }
      const uint32_t in_bytes = (uint32_t)(in_off[s + end] - ic) + idelta;
      const uint32_t out_bytes = kEmit ? (uint32_t)(out_off[s + end] - oc) + odelta : 0u;
      stage_in<false, false>(ws.in_w, 0, ia - idelta, in_bytes, lane);
      if (kEmit) zero_lds(ws.out_w, out_bytes, lane);
      for (uint32_t j = lane; j < m; j += kWave) ws.obits[j] = 0;
      wave_sync();
      // literal holding the first byte of each chunk
      for (uint32_t j = lane; j < m; j += kWave) {
        const uint32_t a = ws.rec[j].x, b = ws.rec[j + 1].x;
        for (uint32_t c = (a + 15u) >> 4; (c << 4) < b; c++) ws.lit_at[c] = (uint16_t)j;
      }
      wave_sync();

      const uint32_t x_lo = ws.rec[0].x, x_hi = ws.rec[m].x;
      const uint32_t c_lo = x_lo >> 4, c_hi = (x_hi + 15u) >> 4;
      uint32_t carry = 0;  // S at the start of this round
      for (uint32_t c0 = c_lo; c0 < c_hi; c0 += kWave) {
        const uint32_t c = c0 + (uint32_t)lane;
        const bool live = c < c_hi;
        const uint32_t x0 = c << 4;
        u32x4 v = live ? *(const u32x4 *)(ws.in_w + 4u * c) : u32x4{0u, 0u, 0u, 0u};
        uint32_t lit0 = (live && x0 >= x_lo) ? ws.lit_at[c] : 0u;
        // pass 1: code lengths of the chunk's bytes
        uint32_t cla[16], len[16];
        uint32_t tot = 0;
#pragma unroll
        for (int i = 0; i < 16; i++) {
          const uint32_t x = x0 + (uint32_t)i;
          const uint32_t byte = (v[i >> 2] >> ((i & 3) * 8)) & 0xffu;
          const bool in_tile = live && x >= x_lo && x < x_hi;
          const uint2 cl = sm.code[byte];
          cla[i] = cl.x;
          len[i] = in_tile ? cl.y : 0u;
          tot += len[i];
        }
        // exclusive wave scan of chunk totals
        uint32_t incl = tot;
#pragma unroll
        for (int d = 1; d < kWave; d <<= 1) {
          const uint32_t y = __shfl_up(incl, d);
          if (lane >= d) incl += y;
        }
        const uint32_t base = carry + incl - tot;
        carry += __shfl(incl, kWave - 1);
        // pass 2a: S at literal starts inside this chunk; encoded bits of literals ending here
        {
          uint32_t lit = lit0, sacc = base;
          uint32_t lo = ws.rec[lit0].x, hi = ws.rec[lit0 + 1].x;  // current literal's byte range
#pragma unroll
          for (int i = 0; i < 16; i++) {
            const uint32_t x = x0 + (uint32_t)i;
            if (live && x >= x_lo && x < x_hi) {
              while (x >= hi) {
                lit++;
                lo = hi;
                hi = ws.rec[lit + 1].x;
              }
              if (x == lo) ws.sstart[lit] = sacc;
            }
            sacc += len[i];
          }
        }
        wave_sync();
        {
          uint32_t lit = lit0, sacc = base;
          uint32_t lo = ws.rec[lit0].x, hi = ws.rec[lit0 + 1].x;  // current literal's byte range
          uint32_t ss = ws.sstart[lit0];
          uint64_t acc = 0;
          uint32_t bp = 0;
          bool open = false;  // bit buffer positioned in a literal's region
#pragma unroll
          for (int i = 0; i < 16; i++) {
            const uint32_t x = x0 + (uint32_t)i;
            if (live && x >= x_lo && x < x_hi) {
              bool moved = false;
              while (x >= hi) {
                lit++;
                lo = hi;
                hi = ws.rec[lit + 1].x;
                moved = true;
              }
              if (moved) ss = ws.sstart[lit];
              if (kEmit) {
                if (!open || x == lo) {
                  if (open) put_flush(ws.out_w, acc, bp);
                  acc = 0;
                  bp = ws.rec[lit].y * 8u + (sacc - ss);
                  open = true;
                }
                put_bits(ws.out_w, acc, bp, cla[i], len[i]);
              }
              if (x + 1u == hi) {  // the literal's last byte: Pad(0xff)
                const uint32_t bits = sacc + len[i] - ss;
                ws.obits[lit] = bits;
                if (kEmit) {
                  const uint32_t pad = (8u - (bp & 7u)) & 7u;
                  if (pad) put_bits(ws.out_w, acc, bp, 0xffffffffu << (32u - pad), pad);
                }
              }
            }
            sacc += len[i];
          }
          if (kEmit && open) put_flush(ws.out_w, acc, bp);
        }
        wave_sync();
      }
      if (kEmit) {
        store_out(oa - odelta, (const uint8_t *)ws.out_w, odelta, out_bytes, lane);
      } else {
        for (uint32_t j = lane; j < m; j += kWave) enc_len[s + cur + j] = (ws.obits[j] + 7u) >> 3;
      }
      wave_sync();
      cur = end;
    }
  }
}

}  // namespace

hipError_t launch_encode_len(const DevTables &t, const uint8_t *in, const uint64_t *in_off, uint64_t in_bias,
                             uint64_t n, uint32_t *enc_len, hipStream_t s) {
  if (n == 0) return hipSuccess;
  const uint64_t ntiles = (n + kTileLits - 1) / kTileLits;
  encode_kernel<false><<<dim3(dev::tile_grid(ntiles, kWaves, MHQ_PER_CU)), dim3(kThreads), 0, s>>>(
      in, in_off, in_bias, n, nullptr, nullptr, 0, enc_len, t.code, t.len, ntiles);
  return hipGetLastError();
}

hipError_t launch_encode(const DevTables &t, const uint8_t *in, const uint64_t *in_off, uint64_t in_bias,
                         uint64_t n, uint8_t *out, const uint64_t *out_off, uint64_t out_bias, hipStream_t s) {
  if (n == 0) return hipSuccess;
  const uint64_t ntiles = (n + kTileLits - 1) / kTileLits;
  encode_kernel<true><<<dim3(dev::tile_grid(ntiles, kWaves, MHQ_PER_CU)), dim3(kThreads), 0, s>>>(
      in, in_off, in_bias, n, out, out_off, out_bias, nullptr, t.code, t.len, ntiles);
  return hipGetLastError();
}

}  // namespace mhq
