// huff_kernels.h -- launchers for the gfx950 Huffman batch kernels.
// Internal to libmhq_huff.so; the public surface is include/mhq_huff.h.
#pragma once
#include <hip/hip_runtime.h>

#include <atomic>
#include <stdint.h>

#include "../../include/mhq_huff.h"

namespace mhq {

// Device copies of the tables built by build_tables() (huff_table.h).
struct DevTables {
  const uint32_t *code;  // [256]
  const uint8_t *len;    // [256]
  const uint32_t *lut1;  // [kLut1Size]
  const uint16_t *lut2;  // [kLut2Size]
};

// All offsets arrays have n+1 entries; literal i occupies
// base[off[i] - bias .. off[i+1] - bias).
// encode_len's block: with `block_sums` not null, block k writes
// (sum of enc_len, sum of floor(8*enc_len/5)) over literals
// [k*kLenSumBlock, (k+1)*kLenSumBlock) to block_sums[2k], [2k+1]
// (ceil(n/kLenSumBlock) pairs), the first pass of the offsets scan.
constexpr int kLenSumBlock = 256;
hipError_t launch_encode_len(const DevTables &t, const uint8_t *in, const uint64_t *in_off,
                             uint64_t in_bias, uint64_t n, uint32_t *enc_len, hipStream_t s,
                             uint64_t *block_sums = nullptr);
// launch_offsets over encode_len's block sums (no reduce pass).  block_sums
// is scratch of offsets_sums_scratch_bytes(n) bytes, encode_len's sums first
// (scanned in place).
size_t offsets_sums_scratch_bytes(uint64_t n);
hipError_t launch_offsets_sums(const uint32_t *enc_len, uint64_t n, uint64_t *block_sums, uint64_t base,
                               uint64_t *out_off, uint64_t *cap_off, hipStream_t s);
hipError_t launch_encode(const DevTables &t, const uint8_t *in, const uint64_t *in_off,
                         uint64_t in_bias, uint64_t n, uint8_t *out, const uint64_t *out_off,
                         uint64_t out_bias, hipStream_t s);
// encode_len + the offsets scan (out_off, cap_off from base) + encode in ONE
// launch (enc_packed.hip), for batches under 2^29 plaintext bytes: out holds
// the encodings from out_off[0] = base on, out_cap bytes (a literal whose
// region ends past it is not written).  slots: encode_packed_slot_bytes(n)
// bytes that only look-backs use, tag: this call's, in 1 .. 2^30 - 1, never
// held by a slot of an earlier call on the buffer (take_slots, mhq_api.cpp).
// in_bytes must be in_off[n] - in_off[0]: otherwise nothing is encoded and
// out_off[n] = UINT64_MAX.
size_t encode_packed_slot_bytes(uint64_t n);
// Polls of an unpublished predecessor before a look-back computes its sum
// itself (enc_packed.hip, read_strings.hip's fallback).
uint32_t lookback_help_polls();
hipError_t launch_encode_packed(const DevTables &t, const uint8_t *in, const uint64_t *in_off, uint64_t in_bias,
                                uint64_t n, uint64_t base, uint32_t *enc_len, uint64_t *out_off, uint64_t *cap_off,
                                uint8_t *out, uint64_t out_cap, uint64_t *slots, uint32_t tag, hipStream_t s,
                                uint64_t in_bytes);
// in_end (optional): literal i is in[in_off[i] - in_bias .. e_i - in_bias), e_i
// the first position at or after in_off[i] whose low 32 bits are in_end[i]
// (literals under 4 GiB); e_i <= in_off[i + 1] when the literals are in order
// (any order decodes; in-order tiles are the fast ones), in_off[n] >= every
// e_i.  str (with in_end): read_strings' strings, see StrFinish.
// read_strings' per-string data for the in_end decode (str_frame.hip): with
// `kind`, each write of out_len / status applies ReadString's outcome
// (str_outcome), and each workgroup ends by finishing its literal range --
// raw payloads copied out, raw EOFs, regions cut short at out_cap -- when the
// parse stored `gen` to *finish_needed (some string is raw) or the output is
// cut (out_off[n] >= out_cap).
struct StrFinish {
  const uint8_t *kind = nullptr;
  const uint64_t *start = nullptr, *next = nullptr;
  const uint32_t *hend = nullptr;
  const uint8_t *blk = nullptr;
  uint64_t out_cap = 0;
  const uint64_t *finish_needed = nullptr;
  uint64_t gen = 0;
  // the workgroup's own range sets the tile-length means and the cut test
  // (the fused read's fallback: no other workgroup's data is read)
  bool local = false;
};
hipError_t launch_decode(const DevTables &t, const uint8_t *in, const uint64_t *in_off,
                         uint64_t in_bias, uint64_t n, uint8_t *out, const uint64_t *out_off,
                         uint64_t out_bias, uint32_t *out_len, uint8_t *status, hipStream_t s,
                         const uint32_t *in_end = nullptr, const StrFinish *str = nullptr, uint64_t in_bytes = 0);
// The streamed decode (huff_decode_stream.hip): launch_decode's form for the
// plain decode (no in_end) when kDecodeStream is set.
hipError_t launch_decode_stream(const DevTables &t, const uint8_t *in, const uint64_t *in_off, uint64_t in_bias,
                                uint64_t n, uint8_t *out, const uint64_t *out_off, uint64_t out_bias,
                                uint32_t *out_len, uint8_t *status, hipStream_t s);
// Which form launch_decode takes for the plain decode: kDecodeAuto (the tile
// kernel, or the long-literal kernel when in_bytes shows a mean over
// kLongMean), kDecodeTile (the tile kernel, huff_decode.hip), kDecodeStream
// (huff_decode_stream.hip).
// Set by mhq_set_decode_form (tests, A/B runs) or MHQ_DECODE_FORM at load.
enum DecodeForm { kDecodeAuto = 0, kDecodeTile = 1, kDecodeStream = 2 };
int decode_form();
int set_decode_form(int form);  // the previous form, -1 for an unknown one
// Test hook (mhq_debug_poison_scratch): read_strings poisons its fallback
// word and look-back slots with round 4's matching forms before each call.
extern std::atomic<int> debug_poison_scratch;
// in_bytes (the batch's encoded bytes, 0 if unknown): a mean literal over
// kLongMean bytes takes the long-literal form (decode_long_kernel)
#ifndef MHQ_DEC_LONG_MEAN
#define MHQ_DEC_LONG_MEAN 64
#endif
constexpr uint64_t kLongMean = MHQ_DEC_LONG_MEAN;
// read_strings in one pass (str_frame.hip, MHQ_RS_FUSED): the frames parsed
// from each staged tile, decoded in place, raw payloads copied, every output
// written; strings out of block order (or a header past the next string's
// pos) store gen to *fallback, and the caller then runs the multi-pass
// pipeline gated on it.  sc_*: the parse of tiles too long to stage (read by
// their streamed decode).
hipError_t launch_read_fused(const DevTables &t, const uint8_t *blk, uint64_t blk_len, const uint64_t *pos,
                             const uint64_t *limit, const uint8_t *prefix, uint64_t n, uint8_t *out,
                             uint64_t *out_off, uint32_t *out_len, uint8_t *status, uint64_t *next,
                             uint64_t *sc_start, uint32_t *sc_hend, uint8_t *sc_kind, uint64_t *fallback,
                             uint64_t *wg_agg, uint64_t gen, hipStream_t s);
// The fallback of launch_read_fused, one launch that returns at once unless
// *fallback == gen (strings out of block order): parse, the regions back to
// back (a decoupled look-back over per-workgroup capacity sums) and the
// decode, per workgroup range.  wg_agg / wg_fin: kReadFallbackMaxWgs words
// each; launch_read_fused clears wg_agg (the look-back slots) for it, and the
// published sums carry a never-zero tag of gen.
constexpr unsigned kReadFallbackMaxWgs = 1024;
hipError_t launch_read_fallback(const DevTables &t, const uint8_t *blk, uint64_t blk_len, const uint64_t *pos,
                                const uint64_t *limit, const uint8_t *prefix, uint64_t n, uint8_t *out,
                                uint64_t out_cap, uint64_t *out_off, uint32_t *out_len, uint8_t *status,
                                uint64_t *next, uint64_t *sc_start, uint32_t *sc_hend, uint8_t *sc_kind,
                                uint64_t *fallback, uint64_t *wg_agg, uint64_t *wg_fin, uint64_t gen, hipStream_t s);
// out_off[i] = base + sum_{j<i} enc_len[j]; cap_off[i] = base + sum_{j<i} floor(8*enc_len[j]/5)
// (either output may be null).  Scratch: offsets_scratch_bytes(n) bytes, or
// null for a hipMallocAsync on `s`.
size_t offsets_scratch_bytes(uint64_t n);
hipError_t launch_offsets(const uint32_t *enc_len, uint64_t n, uint64_t base, uint64_t *out_off,
                          uint64_t *cap_off, hipStream_t s, void *scratch = nullptr);
// oa[i] = min(sum_{j<i} a[j], lim_a), ob[i] = min(sum_{j<i} b[j], lim_b) in one scan
// (a, b 16-B aligned); scratch: offsets_pair_scratch_bytes(n) bytes, or null
// for a hipMallocAsync on s.
size_t offsets_pair_scratch_bytes(uint64_t n);
hipError_t launch_offsets_pair(const uint32_t *a, const uint32_t *b, uint64_t n, uint64_t lim_a, uint64_t lim_b,
                               uint64_t *oa, uint64_t *ob, void *scratch, hipStream_t s);
// launch_offsets_pair over per-kLenSumBlock (sum a, sum b) pairs its producer
// wrote to block_sums (offsets_sums_scratch_bytes(n) bytes; no reduce pass).
// With `gate`, the pass does nothing unless *gate == gen when it runs.
hipError_t launch_offsets_pair_sums(const uint32_t *a, const uint32_t *b, uint64_t n, uint64_t *block_sums,
                                    uint64_t lim_a, uint64_t lim_b, uint64_t *oa, uint64_t *ob, hipStream_t s,
                                    const uint64_t *gate = nullptr, uint64_t gen = 0);
// read_strings' fallback layout: out_off[i] = min(sum_{j<i} cap_j, lim), cap_j
// the output capacity of framed string j recomputed from its parse (kind & 3:
// 1 Huffman floor(8*take/5) with take the low word of hend - start, 0 raw
// next - start, 2 none), over the per-kLenSumBlock sums its parse wrote; only
// when *gate == gen.
hipError_t launch_read_caps_sums(const uint64_t *start, const uint32_t *hend, const uint64_t *next,
                                 const uint8_t *kind, uint64_t n, uint64_t *block_sums, uint64_t lim,
                                 uint64_t *out_off, hipStream_t s, const uint64_t *gate, uint64_t gen);
// cap_off[i] = base + sum_{j<i} floor(8*(in_off[j+1]-in_off[j])/5): decode capacities
// for a batch whose encoded offsets are known.
// Batch ReadString / WriteStringRaw (str_frame.hip); see include/mhq_huff.h.
// read_strings' scratch: read_strings_scratch_bytes(n, blk_len) bytes, or null
// for one hipMallocAsync of them on s.
size_t read_strings_scratch_bytes(uint64_t n, uint64_t blk_len);
hipError_t launch_read_strings(const DevTables &t, const uint8_t *blk, uint64_t blk_len, const uint64_t *pos,
                               const uint64_t *limit, const uint8_t *prefix, uint64_t n, uint8_t *out,
                               uint64_t out_cap, uint64_t *out_off, uint32_t *out_len, uint8_t *status,
                               uint64_t *next, hipStream_t s, void *scratch = nullptr);
// write_strings' scratch: write_strings_scratch_bytes(n, out ? out_cap : 0)
// bytes, or null for one hipMallocAsync of them on s.
size_t write_strings_scratch_bytes(uint64_t n, uint64_t out_cap);
hipError_t launch_write_strings(const DevTables &t, const uint8_t *in, const uint64_t *in_off, uint64_t n,
                                const uint8_t *prefix, const uint8_t *lead, uint32_t choice, uint8_t *out,
                                uint64_t out_cap, uint64_t *out_off, uint8_t *status, hipStream_t s,
                                void *scratch = nullptr);
// Batch ReadInt / WriteInt (str_frame.hip); see include/mhq_huff.h.
hipError_t launch_read_ints(const uint8_t *blk, const uint64_t *pos, const uint64_t *limit, const uint8_t *prefix,
                            uint64_t n, int index, uint64_t *value, uint64_t *next, uint8_t *status, hipStream_t s);
hipError_t launch_write_ints(const uint64_t *value, const uint8_t *prefix, const uint8_t *lead, uint64_t n,
                             uint8_t *out, uint64_t out_cap, uint64_t *out_off, uint8_t *status, hipStream_t s);
// Batch HTTP/3 (draft) varints and frame headers (str_frame.hip); see include/mhq_huff.h.
hipError_t launch_read_varints(const uint8_t *blk, const uint64_t *pos, const uint64_t *limit, uint64_t n,
                               uint64_t *value, uint64_t *next, uint8_t *status, hipStream_t s);
hipError_t launch_read_frames(const uint8_t *blk, const uint64_t *pos, const uint64_t *limit, uint64_t n,
                              uint8_t *type, uint64_t *payload_len, uint64_t *payload_pos, uint8_t *status,
                              hipStream_t s);
hipError_t launch_write_varints(const uint64_t *value, uint64_t n, uint8_t *out, uint64_t out_cap,
                                uint64_t *out_off, uint8_t *status, hipStream_t s);
hipError_t launch_capacity(const uint64_t *in_off, uint64_t n, uint64_t base, uint64_t *cap_off,
                           hipStream_t s);

}  // namespace mhq
