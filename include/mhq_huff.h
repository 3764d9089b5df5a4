/*
 * mhq_huff.h -- C ABI of libmhq_huff.so, the MI355X (gfx950) batch codec for
 * HPACK/QPACK Huffman string literals (RFC 7541 Appendix B).
 *
 * This is the drop-in boundary behind minhq's hc/huffman.go +
 * hc/huffmantable.go.  The reference's streaming, one-literal surface
 *   hc.NewHuffmanCompressor / (*HuffmanCompressor).Write / .Pad
 *                                         (hc/huffman.go:18-37)
 *   hc.NewHuffmanDecompressor / (*HuffmanDecompressor).Read
 *                                         (hc/huffman.go:96-121)
 * stays in Go; a cgo shim adds the batch entry points
 *   hc.HuffmanEncodeBatch(lits [][]byte) [][]byte
 *   hc.HuffmanDecodeBatch(enc  [][]byte) ([][]byte, []error)
 * on top of the functions below.  Per literal the results are byte-for-byte
 * those of Write+Pad and of Read-to-EOF respectively.
 *
 * Layout of a batch: n literals packed back to back; literal i is
 * in[in_off[i] - in_off[0] .. in_off[i+1] - in_off[0]) for the host-memory
 * entry points (in points at literal 0), and in[in_off[i] .. in_off[i+1]) for
 * the device entry points.  Offsets are non-decreasing uint64 arrays of n+1
 * entries.  Output regions follow the same convention with out_off.
 *
 * Ownership: every buffer is caller-owned and used only for the duration of
 * the call (host entry points) or until the work on `stream` completes
 * (device entry points).  The library never retains a caller pointer.
 * Threading: every entry point may be called concurrently on one context.
 * Errors: entry points return MHQ_OK (0) or a negative MHQ_E* code;
 * mhq_strerror() gives its text.  Per-literal decode outcomes go to status[].
 */
#ifndef MHQ_HUFF_H
#define MHQ_HUFF_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define MHQ_OK 0
#define MHQ_EINVAL (-22)  /* bad argument (null pointer, bad device index) */
#define MHQ_ENOMEM (-12)  /* host or device allocation failed */
#define MHQ_ENODEV (-19)  /* no usable gfx950 device */
#define MHQ_EHIP (-1000)  /* a HIP runtime call failed: MHQ_EHIP - hipError_t */

/* Per-literal decode status (status[] entries). */
#define MHQ_LIT_OK 0      /* ran to the end of the literal (io.EOF), or the output region filled */
#define MHQ_LIT_INVALID 1 /* errors.New("invalid Huffman coding"), hc/huffman.go:112 */

typedef struct mhq_ctx mhq_ctx;

/* Opens a context on `ndev` devices (0 = every visible device).  Builds the
 * immutable code/decode tables once and uploads them to each device. */
int mhq_open(mhq_ctx **out, int ndev);
/* Same, on an explicit list of HIP device ordinals (one process per GPU:
 * rank r opens {r}).  Context device index k is ordinals[k]. */
int mhq_open_devices(mhq_ctx **out, const int *ordinals, int count);
void mhq_close(mhq_ctx *ctx);
int mhq_device_count(const mhq_ctx *ctx);
const char *mhq_strerror(int rc);

/* The 256-entry code table as the kernels use it (hc/huffmantable.go:9-267):
 * len[s] bits, value code[s] right-justified.  For tests and tooling. */
int mhq_code_table(uint8_t *len, uint32_t *code);

/* ---------------- host-memory batches (PCIe-inclusive path) ---------------
 * The batch is sharded over the context's devices by encoded bytes.  When
 * every buffer of a call is pinned, device-mapped host memory (mhq_host_alloc,
 * hipHostMalloc, torch pin_memory) the kernels read and write it in place
 * over PCIe, one launch per shard; otherwise (pageable memory) each shard is
 * copied in, processed and copied back in pipelined chunks.  Synchronous. */

/* Pinned, device-mapped host memory for the host-memory calls: buffers from
 * here take the in-place route (no Go/C heap buffer can).  NULL when the
 * allocation fails or no device is visible.  A replacement for the C.malloc
 * of the cgo shim; free with mhq_host_free. */
void *mhq_host_alloc(size_t bytes);
void mhq_host_free(void *p);

/* enc_len[i] = encoded bytes of literal i = ceil(sum of code lengths / 8).
 * Replaces the sizing done by bytes.Buffer in hc/io.go:157-171; drives the
 * Auto choice (hc/io.go:172: Huffman iff enc_len < raw length). */
int mhq_huff_encode_len(mhq_ctx *ctx, const uint8_t *in, const uint64_t *in_off, uint64_t n,
                        uint32_t *enc_len);

/* HuffmanCompressor.Write + Pad per literal (hc/huffman.go:23-37): codes
 * MSB-first, final octet padded with 1 bits.  out_off[i+1]-out_off[i] must be
 * at least enc_len[i]; bytes past enc_len[i] in a region are unspecified (the
 * host forms: zero when the call stages through device buffers, the caller's
 * old contents when it runs in place on pinned buffers).  An
 * empty region (out_off[i+1] == out_off[i]) skips literal i: nothing of it is
 * written (a caller encoding a subset places only that subset). */
int mhq_huff_encode(mhq_ctx *ctx, const uint8_t *in, const uint64_t *in_off, uint64_t n, uint8_t *out,
                    const uint64_t *out_off);

/* HuffmanDecompressor.Read until EOF per literal (hc/huffman.go:102-121),
 * into a region of capacity out_off[i+1]-out_off[i] (floor(8*len/5) always
 * suffices; hc/io.go:87 allocates len*8/5+1).  Writes out_len[i] and
 * status[i].  Trailing partial codes (padding) are dropped without checks,
 * as in the reference.  Bytes past out_len[i] in a region are unspecified:
 * zero when the call stages through device buffers (pageable memory), the
 * caller's old contents when it runs in place on pinned buffers; compare
 * out_len[i] bytes only. */
int mhq_huff_decode(mhq_ctx *ctx, const uint8_t *in, const uint64_t *in_off, uint64_t n, uint8_t *out,
                    const uint64_t *out_off, uint32_t *out_len, uint8_t *status);

/* ---------------- device-resident batches ---------------------------------
 * Same semantics; every pointer is device memory on device `dev` of the
 * context; `stream` is a hipStream_t (NULL = the null stream).  Asynchronous:
 * the call only enqueues work on `stream`. */
int mhq_huff_encode_len_dev(mhq_ctx *ctx, int dev, const uint8_t *in, const uint64_t *in_off, uint64_t n,
                            uint32_t *enc_len, void *stream);
/* out_off[i] = base + sum_{j<i} enc_len[j] (n+1 entries) and, if cap_off is
 * not NULL, cap_off[i] = base + sum_{j<i} floor(8*enc_len[j]/5): the
 * encode output offsets and the matching decode capacities. */
int mhq_huff_offsets_dev(mhq_ctx *ctx, int dev, const uint32_t *enc_len, uint64_t n, uint64_t base,
                         uint64_t *out_off, uint64_t *cap_off, void *stream);
/* mhq_huff_encode_len_dev followed by mhq_huff_offsets_dev (cap_off may be
 * NULL), with the scan's first pass folded into the sizing kernel: the whole
 * output layout of an encode in two launches.  Replaces the sizing half of
 * hc/io.go:157-172 (the temp-buffer encode that Auto mode measures) for a
 * batch, plus the placement the caller would otherwise do on the host. */
int mhq_huff_encode_layout_dev(mhq_ctx *ctx, int dev, const uint8_t *in, const uint64_t *in_off, uint64_t n,
                               uint64_t base, uint32_t *enc_len, uint64_t *out_off, uint64_t *cap_off,
                               void *stream);
/* The encode side of a batch in one call: enc_len[i], out_off (from base,
 * n+1 entries), cap_off (may be NULL) as mhq_huff_encode_layout_dev writes
 * them, and the encodings as mhq_huff_encode_dev writes them, literal i at
 * out[out_off[i] - base].  in_bytes must be in_off[n] - in_off[0] (the
 * device checks: a batch whose offsets disagree is not encoded and gets
 * out_off[n] = UINT64_MAX); out_cap (out's size in bytes) must be at least
 * 30 * in_bytes / 8 + n, the most any n literals of in_bytes plaintext
 * bytes encode to (each pads to whole bytes), MHQ_EINVAL otherwise.  A batch of short literals (mean up to
 * 40 bytes, under 2^29 bytes) takes ONE launch that stages each range of
 * literals once: sized, placed by a look-back over the ranges before it,
 * encoded (enc_packed.hip); other batches take the layout call and the
 * encode.  Replaces hc/io.go:157-172's sizing and hc/huffman.go:23-37's
 * Write + Pad for a batch, plus the placement the caller would do. */
int mhq_huff_encode_packed_dev(mhq_ctx *ctx, int dev, const uint8_t *in, const uint64_t *in_off, uint64_t n,
                               uint64_t in_bytes, uint64_t base, uint32_t *enc_len, uint64_t *out_off,
                               uint64_t *cap_off, uint8_t *out, uint64_t out_cap, void *stream);
/* cap_off[i] = base + sum_{j<i} floor(8*(in_off[j+1]-in_off[j])/5). */
int mhq_huff_capacity_dev(mhq_ctx *ctx, int dev, const uint64_t *in_off, uint64_t n, uint64_t base,
                          uint64_t *cap_off, void *stream);
int mhq_huff_encode_dev(mhq_ctx *ctx, int dev, const uint8_t *in, const uint64_t *in_off, uint64_t n,
                        uint8_t *out, const uint64_t *out_off, void *stream);
int mhq_huff_decode_dev(mhq_ctx *ctx, int dev, const uint8_t *in, const uint64_t *in_off, uint64_t n,
                        uint8_t *out, const uint64_t *out_off, uint32_t *out_len, uint8_t *status,
                        void *stream);
/* mhq_huff_decode_dev for a caller that knows the batch's encoded bytes
 * in_bytes = in_off[n] - in_off[0] (0: unknown, the same as
 * mhq_huff_decode_dev): a mean literal over 64 encoded bytes then takes the
 * long-literal form of the kernel (every tile would stream through per-lane
 * windows anyway; that form runs them at 16 waves per CU instead of 12).
 * Same results either way; the host-memory mhq_huff_decode reads in_bytes
 * from its offsets itself. */
int mhq_huff_decode_sized_dev(mhq_ctx *ctx, int dev, const uint8_t *in, const uint64_t *in_off, uint64_t n,
                              uint64_t in_bytes, uint8_t *out, const uint64_t *out_off, uint32_t *out_len,
                              uint8_t *status, void *stream);
/* Tuning and test hook (no reference counterpart): the kernel form of the
 * plain batch decode (mhq_huff_decode*, not the framed strings).
 * MHQ_DECODE_AUTO: the per-wave tile kernel (huff_decode.hip), or the
 * long-literal kernel when in_bytes shows a mean over 64 encoded bytes;
 * MHQ_DECODE_TILE: the tile kernel for every batch;
 * MHQ_DECODE_STREAM: the streamed decode (huff_decode_stream.hip) for every
 * batch.  Results are the
 * same in every form.  Process-wide; returns the previous form, or
 * MHQ_EINVAL for an unknown one.  MHQ_DECODE_FORM=auto|tile|stream in the
 * environment sets the initial form. */
#define MHQ_DECODE_AUTO 0
#define MHQ_DECODE_TILE 1
#define MHQ_DECODE_STREAM 2
int mhq_set_decode_form(int form);

/* Test hook (no reference counterpart): while set, every read_strings call
 * first fills its fallback word and look-back slots with stale values that
 * match the call in round 4's compare forms (tests/test_strings.py::
 * test_read_poisoned_scratch).  Process-wide; returns the previous setting. */
int mhq_debug_poison_scratch(int on);

/* ---------------- string literals: H bit + prefix integer + payload --------
 * Batch Reader.ReadString(prefix) and Writer.WriteStringRaw(s, prefix, choice)
 * (hc/io.go:73-97, 153-197) with the prefix integers of Reader.ReadInt /
 * Writer.WriteInt (hc/io.go:25-55, 110-137).  A string literal starts on an
 * octet whose low prefix+1 bits hold the H bit and the length prefix; the bits
 * above belong to the caller's opcode (HPACK: prefix 7; QPACK: 7/5/3 after
 * 1/3/5-bit opcodes, hc/qpackdecoder.go:127,163,340). */

/* Per-string outcome of a read (status[]), in ReadString's terms. */
#define MHQ_STR_OK 0      /* (string, nil); also ("", nil) when the H bit or the length cannot be read */
#define MHQ_STR_INVALID 1 /* ("", "invalid Huffman coding") */
#define MHQ_STR_EOF 2     /* ("", io.EOF): nothing decoded from a Huffman literal, or a raw one cut to 0 bytes */
#define MHQ_STR_NOSPACE 3 /* the output buffer could not hold this string (not a reference outcome) */

/* HuffmanCodingChoice (hc/io.go:140-150). */
#define MHQ_HUFF_AUTO 0   /* Huffman iff strictly shorter (hc/io.go:172) */
#define MHQ_HUFF_ALWAYS 1
#define MHQ_HUFF_NEVER 2

/* Reads n string literals from blk[0..blk_len): literal i starts at byte
 * pos[i] (its H bit is bit 7-prefix[i] of that octet) and may use bytes up to
 * limit[i] (the end of its header block: the LimitedReader's underlying EOF
 * truncates the payload silently).  The call writes out_off[0..n] (string i is
 * out[out_off[i] .. out_off[i]+out_len[i]); the regions are disjoint and in
 * string order), out_len[i], status[i] and next[i] (the byte after the
 * payload).  When the strings lie in block order (every payload ends at or
 * before the next string's pos, as in a header block) region i starts at
 * floor(8*start/5) of its payload start and out_off[n] = floor(8*blk_len/5):
 * no scan is needed.  Otherwise the regions are laid back to back, each of
 * floor(8*take/5) (Huffman) or take (raw) bytes.  out_cap must be at least
 * blk_len*8/5 + 1 (enough for any set of non-overlapping literals).  Device
 * pointers; asynchronous on `stream`. */
int mhq_read_strings_dev(mhq_ctx *ctx, int dev, const uint8_t *blk, uint64_t blk_len, const uint64_t *pos,
                         const uint64_t *limit, const uint8_t *prefix, uint64_t n, uint8_t *out, uint64_t out_cap,
                         uint64_t *out_off, uint32_t *out_len, uint8_t *status, uint64_t *next, void *stream);

/* Frames n strings (string i is in[in_off[i]..in_off[i+1])) as
 * WriteStringRaw(s, prefix[i], choice) after opcode bits lead[i] (the
 * 7-prefix[i] bits above the H bit).  Writes out_off[0..n] (frame i is
 * out[out_off[i]..out_off[i+1])) and, when out is not NULL, the frames and
 * status[i] (MHQ_STR_OK, or MHQ_STR_NOSPACE past out_cap).  With out NULL only
 * out_off is computed (size query).  Device pointers; asynchronous on `stream`
 * (no synchronisation inside: only payloads whose frames fit out_cap are
 * encoded, into device scratch of about out_cap bytes -- kept per stream up
 * to 64 MiB, taken in stream order for the call above that). */
int mhq_write_strings_dev(mhq_ctx *ctx, int dev, const uint8_t *in, const uint64_t *in_off, uint64_t n,
                          const uint8_t *prefix, const uint8_t *lead, int choice, uint8_t *out, uint64_t out_cap,
                          uint64_t *out_off, uint8_t *status, void *stream);

/* Host-memory forms of the two calls above (device 0 of the context,
 * synchronous).  Same arguments and layout, host pointers; out_off is written
 * by the call. */
int mhq_read_strings(mhq_ctx *ctx, const uint8_t *blk, uint64_t blk_len, const uint64_t *pos, const uint64_t *limit,
                     const uint8_t *prefix, uint64_t n, uint8_t *out, uint64_t out_cap, uint64_t *out_off,
                     uint32_t *out_len, uint8_t *status, uint64_t *next);
int mhq_write_strings(mhq_ctx *ctx, const uint8_t *in, const uint64_t *in_off, uint64_t n, const uint8_t *prefix,
                      const uint8_t *lead, int choice, uint8_t *out, uint64_t out_cap, uint64_t *out_off,
                      uint8_t *status);

/* ---------------- prefix integers ------------------------------------------
 * Batch Reader.ReadInt / ReadIndex(prefix) and Writer.WriteInt(v, prefix)
 * (hc/io.go:25-67, 110-137), the integers of every HPACK/QPACK instruction
 * (prefixes 3..8: hc/hpack.go:84-130, hc/qpackdecoder.go:145-393).  An integer
 * starts on an octet whose low prefix bits hold its prefix; the bits above
 * belong to the caller's opcode.  Sequential within a header block, the
 * integers of many blocks (or the ones a host pre-pass has located) batch. */

/* Per-integer outcome (status[]). */
#define MHQ_INT_OK 0
#define MHQ_INT_EOF 1      /* the block ended inside the integer (ReadBits: io.EOF) */
#define MHQ_INT_OVERFLOW 2 /* ErrIntegerOverflow (hc/io.go:12,46; ReadIndex: hc/io.go:63) */
#define MHQ_INT_BADARG 3   /* prefix outside 1..8 (not a reference outcome) */
#define MHQ_INT_NOSPACE 4  /* write: the frame does not fit out_cap (not a reference outcome) */

/* Reads n integers from blk: integer i starts at byte pos[i] and may use bytes
 * up to limit[i].  Writes value[i], next[i] (the byte after the integer; pos[i]
 * on error) and status[i].  index != 0 applies ReadIndex's check (value above
 * the largest int64 -> MHQ_INT_OVERFLOW).  Device pointers; asynchronous on
 * `stream`. */
int mhq_read_ints_dev(mhq_ctx *ctx, int dev, const uint8_t *blk, const uint64_t *pos, const uint64_t *limit,
                      const uint8_t *prefix, uint64_t n, int index, uint64_t *value, uint64_t *next,
                      uint8_t *status, void *stream);
/* Writes n integers as WriteInt(value[i], prefix[i]) after opcode bits lead[i]
 * (the 8-prefix[i] bits above the prefix), back to back: integer i is
 * out[out_off[i] .. out_off[i+1]).  out NULL: out_off only (size query).
 * Device pointers; asynchronous on `stream`. */
int mhq_write_ints_dev(mhq_ctx *ctx, int dev, const uint64_t *value, const uint8_t *prefix, const uint8_t *lead,
                       uint64_t n, uint8_t *out, uint64_t out_cap, uint64_t *out_off, uint8_t *status,
                       void *stream);
/* Host-memory forms (device 0 of the context, synchronous). */
int mhq_read_ints(mhq_ctx *ctx, const uint8_t *blk, uint64_t blk_len, const uint64_t *pos, const uint64_t *limit,
                  const uint8_t *prefix, uint64_t n, int index, uint64_t *value, uint64_t *next, uint8_t *status);
int mhq_write_ints(mhq_ctx *ctx, const uint64_t *value, const uint8_t *prefix, const uint8_t *lead, uint64_t n,
                   uint8_t *out, uint64_t out_cap, uint64_t *out_off, uint8_t *status);

/* ---------------- HTTP/3 (draft) frame varints -----------------------------
 * Batch frameReader.ReadVarint / ReadFrame's header and frameWriter.WriteVarint
 * (frame.go:72-92, 128-152): a 2-bit length code (1, 2, 4 or 8 octets), then
 * the value MSB first; a frame header is the payload length as a varint and a
 * type octet. */
#define MHQ_VARINT_OK 0
#define MHQ_VARINT_EOF 1       /* the block ended inside the varint (or before a frame's type octet) */
#define MHQ_VARINT_TOO_LARGE 2 /* write: value >= 2^62, ErrTooLarge (frame.go:52,131-132) */
#define MHQ_VARINT_NOSPACE 3   /* write: past out_cap (not a reference outcome) */

/* Varint i at byte pos[i], reading no byte at or past limit[i]: value[i],
 * next[i] (pos[i] on EOF), status[i].  Device pointers, async on `stream`. */
int mhq_read_varints_dev(mhq_ctx *ctx, int dev, const uint8_t *blk, const uint64_t *pos, const uint64_t *limit,
                         uint64_t n, uint64_t *value, uint64_t *next, uint8_t *status, void *stream);
/* Frame header i at byte pos[i]: type[i], payload_len[i] (as declared),
 * payload_pos[i] (the byte after the type octet; pos[i] on EOF), status[i]. */
int mhq_read_frames_dev(mhq_ctx *ctx, int dev, const uint8_t *blk, const uint64_t *pos, const uint64_t *limit,
                        uint64_t n, uint8_t *type, uint64_t *payload_len, uint64_t *payload_pos, uint8_t *status,
                        void *stream);
/* Writes value[i] as the shortest varint, back to back: varint i is
 * out[out_off[i] .. out_off[i+1]) (empty for a value >= 2^62, status
 * MHQ_VARINT_TOO_LARGE).  out NULL: out_off only (size query). */
int mhq_write_varints_dev(mhq_ctx *ctx, int dev, const uint64_t *value, uint64_t n, uint8_t *out, uint64_t out_cap,
                          uint64_t *out_off, uint8_t *status, void *stream);
/* Host-memory forms (device 0 of the context, synchronous). */
int mhq_read_varints(mhq_ctx *ctx, const uint8_t *blk, uint64_t blk_len, const uint64_t *pos, const uint64_t *limit,
                     uint64_t n, uint64_t *value, uint64_t *next, uint8_t *status);
int mhq_read_frames(mhq_ctx *ctx, const uint8_t *blk, uint64_t blk_len, const uint64_t *pos, const uint64_t *limit,
                    uint64_t n, uint8_t *type, uint64_t *payload_len, uint64_t *payload_pos, uint8_t *status);
int mhq_write_varints(mhq_ctx *ctx, const uint64_t *value, uint64_t n, uint8_t *out, uint64_t out_cap,
                      uint64_t *out_off, uint8_t *status);

#ifdef __cplusplus
}
#endif
#endif /* MHQ_HUFF_H */
