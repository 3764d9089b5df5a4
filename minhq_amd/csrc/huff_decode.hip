// huff_decode.hip -- gfx950 batch decode of RFC 7541 Huffman literals.
//
// Semantics: hc/huffman.go:102-121 (HuffmanDecompressor.Read, one tree step
// per bit) driven to EOF as Reader.ReadString does (hc/io.go:85-96); see the
// contract in SURVEY.md §8a and the CPU restatement oracle/huff_oracle.c.
//   * every complete code emits its byte; a partial code at the end of the
//     literal (padding or otherwise) is dropped without checks;
//   * 30 one-bits reach the childless node where EOS would be
//     (hc/huffman.go:63-76): one more bit of input is "invalid Huffman coding";
//   * Read stops as soon as its buffer is full (hc/huffman.go:104).
//
// Structure: one workgroup per CU; its waves work independently (no
// workgroup barrier after the table load).  A wave takes a tile of up to 128
// consecutive literals at a time (tiles handed out by an LDS counter) and
// decodes it with two literals per lane:
//   * staging: the tile's offsets and input bytes are loaded into registers
//     one tile ahead (offsets two tiles ahead), so HBM latency hides behind
//     the decode of the current tile.  Input lands in the wave's LDS slice as
//     byte-swapped words (word k = stream bits 32k..32k+31, MSB first); the
//     output is assembled in a zeroed LDS copy of the tile's output region
//     (global layout) and leaves as aligned 16-B stores, with out_len/status
//     as coalesced stores, when the next tile starts;
//   * balance: a counting sort by encoded length (descending) inside the
//     wave; lane t decodes rank t, then rank 127-t, so every lane's two
//     literals add up to about the same length and the 64 lanes of a wave
//     run loops of about the same length;
//   * each step reads the two staged words holding a literal's bit position
//     and forms its next 32 bits (bits past the literal's end read as ones,
//     so the loop needs no end test: WinBuf3); a probe reads LUT1 with the
//     next 12 bits (one or two codes of <= 12 bits) or, for longer codes, LUT2
//     by count of leading ones; output bytes gather in a 64-bit register and
//     are OR-ed into the staging one word per step, so literals that share a
//     word need no ordering;
//   * a tile a little over the slices is decoded in pieces that fit; a tile
//     of long literals streams, every lane on a literal of its own through a
//     private LDS window (decode_tile_long).
#include <hip/hip_runtime.h>


#include "huff_decode_dev.h"

namespace mhq {
namespace {

using namespace dev;

template <bool kGaps>
__global__ __launch_bounds__(kT) void decode_kernel(const uint8_t *__restrict__ in, const uint64_t *__restrict__ in_off,
                                                    const uint32_t *__restrict__ in_end, StrFinish str,
                                                    uint64_t in_bias, uint64_t n, uint8_t *__restrict__ out,
                                                    const uint64_t *__restrict__ out_off, uint64_t out_bias,
                                                    uint32_t *__restrict__ out_len, uint8_t *__restrict__ status,
                                                    const uint32_t *__restrict__ g_lut1,
                                                    const uint16_t *__restrict__ g_lut2,
                                                    const uint8_t *__restrict__ g_len, uint64_t per_block,
                                                    uint32_t tl0) {
  __shared__ Smem sm;
  decode_body<kGaps>(sm, in, in_off, in_end, str, in_bias, n, out, out_off, out_bias, out_len, status, g_lut1, g_lut2,
                     g_len, per_block, tl0);
}

// ---- batches of long literals: the streamed form alone, 16 waves per CU ----
// When the mean literal is too long for tiles of 64 to fit the staging
// slices (config 5: 438 encoded bytes), every tile of decode_kernel streams
// through decode_tile_long, which needs only its per-lane windows -- not the
// slices, the records or the sort -- and its loop is latency-bound at the
// decode kernel's 12 waves per CU.  This kernel runs the same per-lane
// windows (128 B a lane) with the tables only: 16 waves per CU, tiles of 64
// literals (one a lane) taken from an LDS counter.
#ifndef MHQ_DEC_LW_WAVES  // waves per workgroup of the long-literal form
#define MHQ_DEC_LW_WAVES 16
#endif
#ifndef MHQ_DEC_LW_WORDS  // a lane's window in words (32: 128 B, 16: 64 B)
#define MHQ_DEC_LW_WORDS 32
#endif
#ifndef MHQ_DEC_LW_PEND  // its output groups pending for wave-wide stores (OutAccGT)
#define MHQ_DEC_LW_PEND 2
#endif
#ifndef MHQ_DEC_LW_BLOCKS  // its workgroups per CU
#define MHQ_DEC_LW_BLOCKS 1
#endif
constexpr int kLWaves = MHQ_DEC_LW_WAVES;
constexpr uint32_t kLWords = MHQ_DEC_LW_WORDS;
struct LongWin {
  uint32_t in_w[kWave * kLWords];
};
struct SmemL {
  uint32_t lut1[kLut1Size];
  uint16_t lut2[kLut2Size];
  uint8_t clen[256];
  uint32_t next_tile;
  LongWin w[kLWaves];
};

__global__ __launch_bounds__(kLWaves * kWave, MHQ_DEC_LW_BLOCKS) void decode_long_kernel(
    const uint8_t *__restrict__ in, const uint64_t *__restrict__ in_off, uint64_t in_bias, uint64_t n,
    uint8_t *__restrict__ out, const uint64_t *__restrict__ out_off, uint64_t out_bias, uint32_t *__restrict__ out_len,
    uint8_t *__restrict__ status, const uint32_t *__restrict__ g_lut1, const uint16_t *__restrict__ g_lut2,
    const uint8_t *__restrict__ g_len, uint64_t per_block) {
  __shared__ SmemL sm;
  const uint32_t tid = threadIdx.x, lane = tid % kWave, wave = tid / kWave;
  const uint64_t L0 = (uint64_t)blockIdx.x * per_block;
  if (L0 >= n) return;
  const uint64_t L1 = min(L0 + per_block, n);
  static_assert(kLut2Size / 8 <= kLWaves * kWave, "table copy shape");
  for (uint32_t i = tid; i < (uint32_t)(kLut1Size / 4); i += kLWaves * kWave) ((u32x4 *)sm.lut1)[i] = ((const u32x4 *)g_lut1)[i];
  if (tid < (uint32_t)(kLut2Size / 8)) ((u32x4 *)sm.lut2)[tid] = ((const u32x4 *)g_lut2)[tid];
  if (tid < 64u) ((uint32_t *)sm.clen)[tid] = ((const uint32_t *)g_len)[tid];
  if (tid == 0) sm.next_tile = kLWaves;
  __syncthreads();
  const uint32_t ntiles = (uint32_t)((L1 - L0 + kWave - 1) / kWave);
  uint32_t tile = wave;
  while (tile < ntiles) {
    const uint64_t s = L0 + (uint64_t)tile * kWave;
    const uint32_t cnt = (uint32_t)min((uint64_t)kWave, L1 - s);
    decode_tile_long_body<false, SmemL, LongWin, kLWords, MHQ_DEC_LW_PEND>(sm, sm.w[wave], in, in_off, nullptr,
                                                                      in_bias, out, out_off, out_bias, out_len,
                                                                      status, s, cnt, lane);
    uint32_t t = 0;
    if (lane == 0) t = atomicAdd(&sm.next_tile, 1u);
    tile = __builtin_amdgcn_readfirstlane(t);
  }
}

}  // namespace

#ifdef MHQ_DIAG_TIMELINE
extern "C" int mhq_diag_timeline(unsigned long long *out, int n) {
  const int m = n < 1024 * 16 * kTlSlots ? n : 1024 * 16 * kTlSlots;
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_tl), m * sizeof(unsigned long long)) == hipSuccess ? kTlSlots : -1;
}
#endif

hipError_t launch_decode(const DevTables &t, const uint8_t *in, const uint64_t *in_off, uint64_t in_bias,
                         uint64_t n, uint8_t *out, const uint64_t *out_off, uint64_t out_bias,
                         uint32_t *out_len, uint8_t *status, hipStream_t s, const uint32_t *in_end,
                         const StrFinish *str, uint64_t in_bytes) {
  if (n == 0) return hipSuccess;
  const int form = decode_form();
  if (!in_end && form == kDecodeStream)
    return launch_decode_stream(t, in, in_off, in_bias, n, out, out_off, out_bias, out_len, status, s);
  if (!in_end && in_bytes > (uint64_t)kLongMean * n) {  // every tile would stream: the long-literal form
    const uint64_t cus = (uint64_t)dev::device_cus();
    const uint64_t blocks = cus * MHQ_DEC_LW_BLOCKS;
    const uint64_t per_block = (((n + blocks - 1) / blocks + kWave - 1) / kWave) * kWave;
    const unsigned grid = (unsigned)((n + per_block - 1) / per_block);
    decode_long_kernel<<<dim3(grid), dim3(kLWaves * kWave), 0, s>>>(in, in_off, in_bias, n, out, out_off, out_bias,
                                                                     out_len, status, t.lut1, t.lut2, t.len, per_block);
    return hipGetLastError();
  }
  // One workgroup per CU, each a contiguous range of whole wave tiles.  The
  // tile length (<= kTile) is chosen so that every wave gets the same number
  // of tiles: no wave idles through a last, partial round.  (A shorter first
  // round of tiles, 86 + 128 + 128 literals per wave on the north star instead
  // of 3 x 114, was 1 us slower: the opening does not shorten with its bytes.)
  const uint64_t cus = (uint64_t)dev::device_cus();
  const uint64_t slots = cus * kWaves;
  const uint64_t rounds = (n + slots * kTile - 1) / (slots * kTile);
  const uint64_t tl = std::max<uint64_t>(1, (n + slots * rounds - 1) / (slots * rounds));
  const uint64_t per_block = (((n + cus - 1) / cus + tl - 1) / tl) * tl;
  const unsigned grid = (unsigned)((n + per_block - 1) / per_block);
  if (in_end)
    decode_kernel<true><<<dim3(grid), dim3(kT), 0, s>>>(in, in_off, in_end, str ? *str : StrFinish{}, in_bias, n, out,
                                                        out_off, out_bias,
                                                        out_len, status, t.lut1, t.lut2, t.len, per_block,
                                                        (uint32_t)tl);
  else
    decode_kernel<false><<<dim3(grid), dim3(kT), 0, s>>>(in, in_off, nullptr, StrFinish{}, in_bias, n, out, out_off,
                                                         out_bias,
                                                         out_len, status, t.lut1, t.lut2, t.len, per_block,
                                                         (uint32_t)tl);
  return hipGetLastError();
}

#ifdef MHQ_DBG_BOUNDS
MHQ_DBG_READER(mhq_dbg_bounds_decode)
#endif

}  // namespace mhq
