/*
 * huff_oracle.c -- TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement of minhq's Go Huffman path, used as the parity checker for
 * the HIP product library (minhq_amd/libmhq_huff.so) and as the "port" CPU
 * baseline in bench.py.  Only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg may load this library.  Nothing in minhq_amd/ links it.
 *
 * Pinning: the Go reference cannot be built or run in this pipeline (no Go
 * toolchain).  This restatement is pinned by the reference's
 * own known-answer vectors, extracted into tests/golden/ by
 * tests/golden/make_golden.py (hc/huffman_test.go:12-28, hc/io_test.go:76-87,
 * io/bitio_test.go:25-45, Huffman literals embedded in hc/testcases_test.go
 * and hc/qpack_test.go, and the code table hc/huffmantable.go:9-267).
 *
 * Every function cites the reference lines it follows.
 */
#include "huff_oracle.h"

#include <pthread.h>
#include <stdlib.h>
#include <string.h>

/* ------------------------------------------------------------------------ */
/* Code table: hc/huffmantable.go:9-267 (RFC 7541 Appendix B).               */
/* The code is canonical, so it is stored as lengths only and the code       */
/* values are rebuilt in (length, symbol) order.  tests/golden/              */
/* huffman_table.json (extracted from the reference) pins the result.        */
/* EOS (symbol 256, hc/huffmantable.go:266) is absent, as in the reference.  */
/* ------------------------------------------------------------------------ */
static const uint8_t k_code_len[256] = {
    13, 23, 28, 28, 28, 28, 28, 28, 28, 24, 30, 28, 28, 30, 28, 28,
    28, 28, 28, 28, 28, 28, 30, 28, 28, 28, 28, 28, 28, 28, 28, 28,
    6,  10, 10, 12, 13, 6,  8,  11, 10, 10, 8,  11, 8,  6,  6,  6,
    5,  5,  5,  6,  6,  6,  6,  6,  6,  6,  7,  8,  15, 6,  12, 10,
    13, 6,  7,  7,  7,  7,  7,  7,  7,  7,  7,  7,  7,  7,  7,  7,
    7,  7,  7,  7,  7,  7,  7,  7,  8,  7,  8,  13, 19, 13, 14, 6,
    15, 5,  6,  5,  6,  5,  6,  6,  6,  5,  7,  7,  6,  6,  6,  5,
    6,  7,  6,  5,  5,  6,  7,  7,  7,  7,  7,  15, 11, 14, 13, 28,
    20, 22, 20, 20, 22, 22, 22, 23, 22, 23, 23, 23, 23, 23, 24, 23,
    24, 24, 22, 23, 24, 23, 23, 23, 23, 21, 22, 23, 22, 23, 23, 24,
    22, 21, 20, 22, 22, 23, 23, 21, 23, 22, 22, 24, 21, 22, 23, 23,
    21, 21, 22, 21, 23, 22, 23, 23, 20, 22, 22, 22, 23, 22, 22, 23,
    26, 26, 20, 19, 22, 23, 22, 25, 26, 26, 26, 27, 27, 26, 24, 25,
    19, 21, 26, 27, 27, 26, 27, 24, 21, 21, 26, 26, 28, 27, 27, 27,
    20, 24, 20, 21, 22, 21, 21, 23, 22, 22, 25, 25, 24, 24, 26, 23,
    26, 27, 26, 26, 27, 27, 27, 27, 27, 28, 27, 27, 27, 27, 27, 26,
};

typedef struct {
  uint8_t len;
  uint32_t val; /* right-justified, as huffmanTableItem (hc/huffmantable.go:3-6) */
} orc_item;

static orc_item g_table[256];

/* Decoder tree: hc/huffman.go:40-44 (huffmanDecoderNode). */
typedef struct orc_node {
  int32_t next[2]; /* index into g_nodes, -1 == nil */
  uint8_t leaf;
  uint8_t val;
} orc_node;

#define ORC_MAX_NODES 1024
static orc_node g_nodes[ORC_MAX_NODES];
static int g_nnodes;
static int32_t g_root = -1;
static pthread_once_t g_once = PTHREAD_ONCE_INIT;

static int32_t new_node(void) {
  int32_t id = g_nnodes++;
  g_nodes[id].next[0] = g_nodes[id].next[1] = -1;
  g_nodes[id].leaf = 0;
  g_nodes[id].val = 0;
  return id;
}

/* makeLayer: hc/huffman.go:46-79.  Scans all 256 entries in symbol order,
 * attaches leaves for codes that end one level down, returns early once both
 * children are leaves, and recurses into nil children only if some code
 * extends below this prefix ("found").  The all-ones prefix of length 30
 * (where EOS would sit) finds nothing and stays a childless non-leaf. */
static int32_t make_layer(uint32_t prefix, uint8_t prefix_len) {
  int32_t layer = new_node();
  int found = 0;
  for (int i = 0; i < 256; i++) {
    const orc_item e = g_table[i];
    if (e.len < prefix_len + 1) continue;
    if ((e.val >> (e.len - prefix_len)) != prefix) continue;
    uint32_t arity = (e.val >> (e.len - prefix_len - 1)) & 1u;
    if (e.len == prefix_len + 1) {
      int32_t child = new_node();
      g_nodes[child].leaf = 1;
      g_nodes[child].val = (uint8_t)i;
      g_nodes[layer].next[arity] = child;
      if (g_nodes[layer].next[arity ^ 1u] != -1) return layer;
    }
    found = 1;
  }
  if (found) {
    if (g_nodes[layer].next[0] == -1) {
      int32_t c = make_layer(prefix << 1, prefix_len + 1);
      g_nodes[layer].next[0] = c;
    }
    if (g_nodes[layer].next[1] == -1) {
      int32_t c = make_layer((prefix << 1) | 1u, prefix_len + 1);
      g_nodes[layer].next[1] = c;
    }
  }
  return layer;
}

/* Table-driven decode (CPU baseline beside the restated Go loop):
 * g_fast[w] is the symbol and length of the code (<= ORC_FAST_BITS bits) that
 * starts the ORC_FAST_BITS-bit window w, found by walking the same tree; 0 if
 * the code is longer (then the tree walk takes over). */
#define ORC_FAST_BITS 12
typedef struct {
  uint8_t sym, len;
} orc_fast;
static orc_fast g_fast[1u << ORC_FAST_BITS];

static void build_fast_lut(void) {
  for (uint32_t w = 0; w < (1u << ORC_FAST_BITS); w++) {
    int32_t node = g_root;
    g_fast[w].len = 0;
    for (int b = 0; b < ORC_FAST_BITS; b++) {
      node = g_nodes[node].next[(w >> (ORC_FAST_BITS - 1 - b)) & 1u];
      if (node < 0) break;
      if (g_nodes[node].leaf) {
        g_fast[w].sym = g_nodes[node].val;
        g_fast[w].len = (uint8_t)(b + 1);
        break;
      }
    }
  }
}

/* The reference initialises lazily and without synchronisation
 * (hc/huffman.go:81-87); here it is built exactly once (pthread_once) so the
 * threaded CPU baseline is race free. */
static void init_once(void) {
  /* canonical rebuild of hc/huffmantable.go values */
  int order[256];
  for (int i = 0; i < 256; i++) order[i] = i;
  for (int i = 1; i < 256; i++) { /* insertion sort by (len, sym) */
    int s = order[i], j = i - 1;
    while (j >= 0 && (k_code_len[order[j]] > k_code_len[s])) {
      order[j + 1] = order[j];
      j--;
    }
    order[j + 1] = s;
  }
  uint32_t code = 0;
  uint8_t prev = k_code_len[order[0]];
  for (int i = 0; i < 256; i++) {
    int s = order[i];
    if (i > 0) code = (code + 1u) << (k_code_len[s] - prev);
    prev = k_code_len[s];
    g_table[s].len = k_code_len[s];
    g_table[s].val = code;
  }
  g_nnodes = 0;
  g_root = make_layer(0, 0);
  build_fast_lut();
}

void orc_init(void) { pthread_once(&g_once, init_once); }

void orc_table(uint8_t *len, uint32_t *val) {
  orc_init();
  for (int i = 0; i < 256; i++) {
    len[i] = g_table[i].len;
    val[i] = g_table[i].val;
  }
}

int orc_tree_nodes(void) {
  orc_init();
  return g_nnodes;
}

/* ------------------------------------------------------------------------ */
/* Bit writer: io/bitio.go:17-149 (bitWriter), writing into a caller buffer. */
/* ------------------------------------------------------------------------ */
typedef struct {
  uint8_t *out;
  size_t cap;
  size_t written;
  uint64_t saved;
  uint8_t saved_bits;
} orc_bw;

/* writeByteInternal: io/bitio.go:41-56 (ByteWriter fast path). */
static int bw_write_byte(orc_bw *bw, uint8_t c) {
  if (bw->written >= bw->cap) return ORC_ERR_SHORT_WRITE;
  bw->out[bw->written++] = c;
  return 0;
}

/* writeSaved: io/bitio.go:59-69. */
static int bw_write_saved(orc_bw *bw) {
  while (bw->saved_bits >= 8) {
    uint8_t x = (uint8_t)(bw->saved >> (bw->saved_bits - 8));
    int err = bw_write_byte(bw, x);
    if (err) return err;
    bw->saved_bits -= 8;
  }
  return 0;
}

/* WriteBits: io/bitio.go:72-105. */
static int bw_write_bits(orc_bw *bw, uint64_t v, uint8_t count) {
  if (count > 64) return ORC_ERR_TOO_LARGE;
  if (count < 64 && v >= (1ull << count)) return ORC_ERR_TOO_LARGE;
  if (bw->saved_bits + count < 8) {
    bw->saved_bits += count;
    bw->saved = (bw->saved << count) | v;
    return 0;
  }
  int err = bw_write_saved(bw);
  if (err) return err;
  uint8_t remainder = (uint8_t)(count + bw->saved_bits - 8);
  /* Go: byte((saved << (8-savedBits)) | (v >> remainder)); shifts >= 64 give 0 */
  uint64_t hi = bw->saved << (8 - bw->saved_bits);
  uint64_t lo = remainder >= 64 ? 0 : (v >> remainder);
  err = bw_write_byte(bw, (uint8_t)(hi | lo));
  if (err) return err;
  bw->saved = v;
  bw->saved_bits = remainder;
  (void)bw_write_saved(bw);
  return 0;
}

/* Pad: io/bitio.go:135-149. */
static int bw_pad(orc_bw *bw, uint8_t pad) {
  if (bw->saved_bits > 0) {
    int err = bw_write_saved(bw);
    if (err) return err;
    err = bw_write_bits(bw, (uint64_t)(pad >> bw->saved_bits), (uint8_t)(8 - bw->saved_bits));
    if (err) return err;
    bw->saved = 0;
    bw->saved_bits = 0;
  }
  return 0;
}

/* Exposed for the io/bitio_test.go:25-45 vectors. */
struct orc_bitwriter {
  orc_bw bw;
};

orc_bitwriter *orc_bw_new(uint8_t *out, size_t cap) {
  orc_bitwriter *w = (orc_bitwriter *)calloc(1, sizeof(*w));
  if (!w) return NULL;
  w->bw.out = out;
  w->bw.cap = cap;
  return w;
}
int orc_bw_write_bits(orc_bitwriter *w, uint64_t v, uint8_t count) {
  return bw_write_bits(&w->bw, v, count);
}
int orc_bw_pad(orc_bitwriter *w, uint8_t pad) { return bw_pad(&w->bw, pad); }
size_t orc_bw_written(orc_bitwriter *w) { return w->bw.written; }
void orc_bw_free(orc_bitwriter *w) { free(w); }

/* ------------------------------------------------------------------------ */
/* Huffman compressor: hc/huffman.go:18-37.                                  */
/* ------------------------------------------------------------------------ */
size_t orc_huff_encoded_len(const uint8_t *in, size_t len) {
  orc_init();
  uint64_t bits = 0;
  for (size_t i = 0; i < len; i++) bits += g_table[in[i]].len;
  return (size_t)((bits + 7) / 8);
}

int orc_huff_encode(const uint8_t *in, size_t len, uint8_t *out, size_t cap, size_t *out_len) {
  orc_init();
  orc_bw bw = {out, cap, 0, 0, 0};
  for (size_t i = 0; i < len; i++) { /* Write: hc/huffman.go:23-32 */
    const orc_item e = g_table[in[i]];
    int err = bw_write_bits(&bw, (uint64_t)e.val, e.len);
    if (err) {
      *out_len = bw.written;
      return err;
    }
  }
  int err = bw_pad(&bw, 0xff); /* Pad: hc/huffman.go:35-37 */
  *out_len = bw.written;
  return err;
}

/* ------------------------------------------------------------------------ */
/* Huffman decompressor: hc/huffman.go:90-121 over bitReader.ReadBit         */
/* (io/bitio.go:174-214).  One tree step per bit.                            */
/* Returns ORC_OK when the input ran out (EOF) or the output filled, and     */
/* ORC_INVALID on a nil child (hc/huffman.go:111-113); *out_len is the count */
/* of bytes produced before that point in both cases.                        */
/* ------------------------------------------------------------------------ */
int orc_huff_decode(const uint8_t *in, size_t len, uint8_t *out, size_t cap, size_t *out_len) {
  orc_init();
  int32_t cursor = g_root;
  size_t i = 0;      /* bytes emitted */
  size_t pos = 0;    /* next input byte (readByteInternal) */
  uint64_t saved = 0;
  uint8_t saved_bits = 0;
  while (i < cap) {
    /* ReadBit: io/bitio.go:202-214 */
    if (saved_bits == 0) {
      if (pos >= len) break; /* reader error (io.EOF): Read returns (i, err) */
      saved = (saved << 8) | in[pos++];
      saved_bits += 8;
    }
    saved_bits--;
    uint32_t b = (uint32_t)(saved >> saved_bits) & 1u;
    cursor = g_nodes[cursor].next[b];
    if (cursor == -1) {
      *out_len = i;
      return ORC_INVALID;
    }
    if (g_nodes[cursor].leaf) {
      out[i++] = g_nodes[cursor].val;
      cursor = g_root;
    }
  }
  *out_len = i;
  return ORC_OK;
}

/* Same results as orc_huff_decode, a table lookup per code of <= 12 bits:
 * the next 12 bits (zeros past the end) index g_fast; a code that fits the
 * literal is taken whole, anything else (a longer code, the end of the
 * literal, the EOS prefix) goes one symbol through the bit-serial tree walk,
 * so the end-of-literal, INVALID and buffer-full rules are the reference's. */
int orc_huff_decode_fast(const uint8_t *in, size_t len, uint8_t *out, size_t cap, size_t *out_len) {
  orc_init();
  const uint64_t end = (uint64_t)len * 8u;
  uint64_t pos = 0;
  size_t n = 0;
  while (n < cap && pos < end) {
    /* 32 bits from pos, MSB first, zeros past the end */
    const uint64_t byte = pos >> 3;
    uint64_t v = 0;
    for (int k = 0; k < 5; k++) v = (v << 8) | (byte + (uint64_t)k < len ? in[byte + (uint64_t)k] : 0u);
    const uint32_t win = (uint32_t)(v >> (8u - (pos & 7u)));
    const orc_fast e = g_fast[win >> (32 - ORC_FAST_BITS)];
    if (e.len && (uint64_t)e.len <= end - pos) {
      out[n++] = e.sym;
      pos += e.len;
      continue;
    }
    int32_t node = g_root; /* one symbol, bit by bit (hc/huffman.go:104-119) */
    for (;;) {
      if (pos >= end) goto done; /* EOF inside a code: partial code dropped */
      const uint32_t bit = (in[pos >> 3] >> (7u - (pos & 7u))) & 1u;
      pos++;
      node = g_nodes[node].next[bit];
      if (node < 0) {
        *out_len = n;
        return ORC_INVALID;
      }
      if (g_nodes[node].leaf) {
        out[n++] = g_nodes[node].val;
        break;
      }
    }
  }
done:
  *out_len = n;
  return ORC_OK;
}

/* ------------------------------------------------------------------------ */
/* String level: Reader.ReadInt / ReadString (hc/io.go:25-55, 73-97) and    */
/* Writer.WriteInt / WriteStringRaw (hc/io.go:110-137, 153-197).             */
/* The input is a byte-aligned string literal whose first octet carries     */
/* (8 - 1 - prefix) bits that belong to the caller's opcode; this helper    */
/* starts at the H bit position given by `skip_bits` (0..7).                */
/* ------------------------------------------------------------------------ */
typedef struct {
  const uint8_t *in;
  size_t len, pos;
  uint64_t saved;
  uint8_t saved_bits;
} orc_br;

static int br_read_byte_internal(orc_br *br, uint8_t *b) {
  if (br->pos >= br->len) return ORC_ERR_EOF;
  *b = br->in[br->pos++];
  return 0;
}

/* ReadBits: io/bitio.go:217-246 */
static int br_read_bits(orc_br *br, uint8_t count, uint64_t *out) {
  if (count > 64) return ORC_ERR_TOO_LARGE;
  while (br->saved_bits + 8 <= count) {
    uint8_t b;
    int err = br_read_byte_internal(br, &b);
    if (err) return err;
    br->saved = (br->saved << 8) | b;
    br->saved_bits += 8;
  }
  if (br->saved_bits >= count) {
    br->saved_bits -= count;
    uint64_t mask = count == 0 ? 0 : (~0ull >> (64 - count));
    *out = (br->saved >> br->saved_bits) & mask;
    return 0;
  }
  uint64_t result = br->saved_bits == 0 ? 0 : (br->saved & (~0ull >> (64 - br->saved_bits)));
  uint8_t remainder = count - br->saved_bits;
  uint8_t b;
  int err = br_read_byte_internal(br, &b);
  if (err) return err;
  br->saved = b;
  br->saved_bits = 8 - remainder;
  *out = (result << remainder) | (br->saved >> (8 - remainder));
  return 0;
}

/* ReadInt: hc/io.go:25-55 */
static int br_read_int(orc_br *br, uint8_t prefix, uint64_t *out) {
  uint64_t v;
  int err = br_read_bits(br, prefix, &v);
  if (err) return err;
  if (v < ((1ull << prefix) - 1)) {
    *out = v;
    return 0;
  }
  for (uint8_t s = 0; s < 64; s += 7) {
    uint64_t b;
    err = br_read_bits(br, 8, &b);
    if (err) return err;
    if (s == 63 && (b > 1 || (b == 1 && ((v >> 63) == 1)))) return ORC_ERR_OVERFLOW;
    v += (b & 0x7f) << s;
    if ((b & 0x80) == 0) break;
  }
  *out = v;
  return 0;
}

/* Reader.ReadInt(prefix) after `skip_bits` opcode bits (hc/io.go:25-55):
 * ORC_OK with *out and *consumed (whole octets read), ORC_ERR_EOF when the
 * input ends inside the integer, ORC_ERR_OVERFLOW (hc/io.go:46). */
int orc_read_int(const uint8_t *in, size_t len, uint8_t skip_bits, uint8_t prefix, uint64_t *out,
                 size_t *consumed) {
  orc_br br = {in, len, 0, 0, 0};
  uint64_t tmp;
  *out = 0;
  *consumed = 0;
  if (skip_bits) {
    int err = br_read_bits(&br, skip_bits, &tmp);
    if (err) return err;
  }
  int err = br_read_int(&br, prefix, out);
  if (err) {
    *out = 0;
    return err;
  }
  *consumed = br.pos;
  return ORC_OK;
}

int orc_read_string(const uint8_t *in, size_t len, uint8_t skip_bits, uint8_t prefix,
                    uint8_t *out, size_t cap, size_t *out_len, size_t *consumed) {
  orc_init();
  orc_br br = {in, len, 0, 0, 0};
  uint64_t tmp;
  *out_len = 0;
  *consumed = 0;
  if (skip_bits && br_read_bits(&br, skip_bits, &tmp)) return ORC_OK;
  uint64_t h;
  if (br_read_bits(&br, 1, &h)) return ORC_OK;          /* hc/io.go:74-77: ("", nil) */
  uint64_t n;
  if (br_read_int(&br, prefix, &n)) return ORC_OK;      /* hc/io.go:78-81: ("", nil) */
  /* LimitedReader{R: hr, N: len} (hc/io.go:82); the prefix ends on an octet
   * boundary in every HPACK/QPACK use, so the payload is the next n bytes,
   * truncated silently at the end of the input. */
  size_t start = br.pos;
  size_t avail = len - start;
  size_t take = n < avail ? (size_t)n : avail;
  *consumed = start + take;
  if (h) {
    /* buf = make([]byte, len*8/5+1); io.ReadFull (hc/io.go:85-93) */
    size_t need = (size_t)(n * 8 / 5 + 1);
    size_t got = 0;
    int st = orc_huff_decode(in + start, take, out, need < cap ? need : cap, &got);
    if (st == ORC_INVALID) return ORC_INVALID;          /* ("", err) */
    if (got == 0 && need > 0) return ORC_ERR_EOF;       /* io.ReadFull: io.EOF */
    *out_len = got;
    return ORC_OK;
  }
  if (take == 0 && n > 0) return ORC_ERR_EOF;
  if (take > cap) return ORC_ERR_SHORT_WRITE;
  memcpy(out, in + start, take);
  *out_len = take;
  return ORC_OK;
}

/* WriteInt: hc/io.go:110-137 */
static int bw_write_int(orc_bw *bw, uint64_t p, uint8_t prefix) {
  uint64_t ones = (1ull << prefix) - 1;
  if (p < ones) return bw_write_bits(bw, p, prefix);
  int err = bw_write_bits(bw, ones, prefix);
  if (err) return err;
  p -= ones;
  for (int done = 0; !done;) {
    uint8_t b = (uint8_t)(p & 0x7f);
    p >>= 7;
    if (p > 0) b |= 0x80;
    else done = 1;
    err = bw_write_bits(bw, b, 8);
    if (err) return err;
  }
  return 0;
}

/* Writer.WriteInt(v, prefix) after `lead_bits` opcode bits of value `lead`
 * (hc/io.go:110-137), flushed to whole octets. */
int orc_write_int(uint64_t v, uint8_t lead, uint8_t lead_bits, uint8_t prefix, uint8_t *out, size_t cap,
                  size_t *out_len) {
  orc_bw bw;
  memset(&bw, 0, sizeof(bw));
  bw.out = out;
  bw.cap = cap;
  int err = lead_bits ? bw_write_bits(&bw, lead, lead_bits) : 0;
  if (!err) err = bw_write_int(&bw, v, prefix);
  *out_len = bw.written;
  return err;
}

/* ------------------------------------------------------------------------ */
/* HTTP/3 (draft) frame varints (frame.go:72-92, 128-152).                   */
/* ------------------------------------------------------------------------ */

/* ReadVarint (frame.go:72-79): a 2-bit length code, then (8 << code) - 2
 * value bits, MSB first. */
int orc_read_varint(const uint8_t *in, size_t len, uint64_t *out, size_t *consumed) {
  orc_br br = {in, len, 0, 0, 0};
  uint64_t code;
  *out = 0;
  *consumed = 0;
  int err = br_read_bits(&br, 2, &code);
  if (err) return err;
  err = br_read_bits(&br, (uint8_t)((8u << code) - 2u), out);
  if (err) {
    *out = 0;
    return err;
  }
  *consumed = br.pos;
  return ORC_OK;
}

/* WriteVarint (frame.go:128-152): the shortest of 1, 2, 4, 8 octets;
 * values >= 2^62 are ErrTooLarge. */
int orc_write_varint(uint64_t v, uint8_t *out, size_t cap, size_t *out_len) {
  orc_bw bw;
  memset(&bw, 0, sizeof(bw));
  bw.out = out;
  bw.cap = cap;
  *out_len = 0;
  uint8_t size;
  if (v >= (1ull << 62)) return ORC_ERR_TOO_LARGE;
  if (v >= (1ull << 30)) size = 3;
  else if (v >= (1ull << 14)) size = 2;
  else if (v >= (1ull << 6)) size = 1;
  else size = 0;
  int err = bw_write_bits(&bw, size, 2);
  if (!err) err = bw_write_bits(&bw, v, (uint8_t)((1u << size) * 8u - 2u));
  *out_len = bw.written;
  return err;
}

/* ReadFrame's header (frame.go:81-92): the payload length as a varint, then
 * the type octet; the payload is the next `len` octets (a LimitedReader). */
int orc_read_frame(const uint8_t *in, size_t len, uint8_t *type, uint64_t *plen, size_t *hdr_len) {
  size_t used = 0;
  *type = 0;
  *plen = 0;
  *hdr_len = 0;
  int err = orc_read_varint(in, len, plen, &used);
  if (err) return err;
  if (used >= len) {
    *plen = 0;
    return ORC_ERR_EOF;
  }
  *type = in[used];
  *hdr_len = used + 1;
  return ORC_OK;
}

/* WriteStringRaw: hc/io.go:153-197.  choice: 0 Auto, 1 Always, 2 Never
 * (hc/io.go:140-150).  Writes H bit + prefix integer + payload starting on an
 * octet boundary after `lead_bits` opcode bits (value `lead`). */
int orc_write_string(const uint8_t *s, size_t len, uint8_t lead, uint8_t lead_bits,
                     uint8_t prefix, int choice, uint8_t *out, size_t cap, size_t *out_len) {
  orc_init();
  orc_bw bw = {out, cap, 0, 0, 0};
  uint8_t *tmp = NULL;
  size_t l = len;
  const uint8_t *payload = s;
  uint64_t hbit = 0;
  *out_len = 0;
  if (choice != 2) {
    size_t enc_cap = orc_huff_encoded_len(s, len);
    tmp = (uint8_t *)malloc(enc_cap ? enc_cap : 1);
    size_t enc_len = 0;
    int err = orc_huff_encode(s, len, tmp, enc_cap, &enc_len);
    if (err) {
      free(tmp);
      return err;
    }
    if (choice == 1 || enc_len < len) { /* strict less-than: hc/io.go:172 */
      payload = tmp;
      l = enc_len;
      hbit = 1;
    }
  }
  int err = 0;
  if (lead_bits) err = bw_write_bits(&bw, lead, lead_bits);
  if (!err) err = bw_write_bits(&bw, hbit, 1);
  if (!err) err = bw_write_int(&bw, (uint64_t)l, prefix);
  for (size_t i = 0; !err && i < l; i++) err = bw_write_bits(&bw, payload[i], 8);
  free(tmp);
  *out_len = bw.written;
  return err;
}

/* ------------------------------------------------------------------------ */
/* Batch drivers (the CPU baseline): literal i is in[in_off[i]..in_off[i+1]). */
/* Threads take contiguous literal ranges; the per-literal work is exactly   */
/* the restated Go loop above.                                               */
/* ------------------------------------------------------------------------ */
typedef struct {
  int op; /* 0 len, 1 encode, 2 decode, 3 table-driven decode */
  const uint8_t *in;
  const uint64_t *in_off;
  uint8_t *out;
  const uint64_t *out_off;
  uint32_t *lens;
  uint8_t *status;
  uint64_t lo, hi;
  int rc;
} orc_job;

static void *orc_worker(void *arg) {
  orc_job *j = (orc_job *)arg;
  j->rc = 0;
  for (uint64_t i = j->lo; i < j->hi; i++) {
    const uint8_t *src = j->in + j->in_off[i];
    size_t n = (size_t)(j->in_off[i + 1] - j->in_off[i]);
    if (j->op == 0) {
      j->lens[i] = (uint32_t)orc_huff_encoded_len(src, n);
    } else if (j->op == 1) {
      size_t cap = (size_t)(j->out_off[i + 1] - j->out_off[i]), got = 0;
      int err = orc_huff_encode(src, n, j->out + j->out_off[i], cap, &got);
      if (err) j->rc = err;
    } else {
      size_t cap = (size_t)(j->out_off[i + 1] - j->out_off[i]), got = 0;
      int st = j->op == 2 ? orc_huff_decode(src, n, j->out + j->out_off[i], cap, &got)
                          : orc_huff_decode_fast(src, n, j->out + j->out_off[i], cap, &got);
      j->lens[i] = (uint32_t)got;
      j->status[i] = (uint8_t)(st == ORC_INVALID ? 1 : 0);
    }
  }
  return NULL;
}

static int orc_run(int op, const uint8_t *in, const uint64_t *in_off, uint64_t n, uint8_t *out,
                   const uint64_t *out_off, uint32_t *lens, uint8_t *status, int nthreads) {
  orc_init();
  if (nthreads < 1) nthreads = 1;
  if ((uint64_t)nthreads > n) nthreads = n ? (int)n : 1;
  orc_job *jobs = (orc_job *)calloc((size_t)nthreads, sizeof(orc_job));
  pthread_t *tids = (pthread_t *)calloc((size_t)nthreads, sizeof(pthread_t));
  if (!jobs || !tids) {
    free(jobs);
    free(tids);
    return ORC_ERR_NOMEM;
  }
  for (int t = 0; t < nthreads; t++) {
    jobs[t] = (orc_job){op, in, in_off, out, out_off, lens, status,
                        n * (uint64_t)t / (uint64_t)nthreads, n * (uint64_t)(t + 1) / (uint64_t)nthreads, 0};
    if (nthreads == 1) orc_worker(&jobs[t]);
    else pthread_create(&tids[t], NULL, orc_worker, &jobs[t]);
  }
  int rc = 0;
  for (int t = 0; t < nthreads; t++) {
    if (nthreads > 1) pthread_join(tids[t], NULL);
    if (jobs[t].rc) rc = jobs[t].rc;
  }
  free(jobs);
  free(tids);
  return rc;
}

int orc_encode_len_batch(const uint8_t *in, const uint64_t *in_off, uint64_t n, uint32_t *enc_len,
                         int nthreads) {
  return orc_run(0, in, in_off, n, NULL, NULL, enc_len, NULL, nthreads);
}
int orc_encode_batch(const uint8_t *in, const uint64_t *in_off, uint64_t n, uint8_t *out,
                     const uint64_t *out_off, int nthreads) {
  return orc_run(1, in, in_off, n, out, out_off, NULL, NULL, nthreads);
}
int orc_decode_batch(const uint8_t *in, const uint64_t *in_off, uint64_t n, uint8_t *out,
                     const uint64_t *out_off, uint32_t *out_len, uint8_t *status, int nthreads) {
  return orc_run(2, in, in_off, n, out, out_off, out_len, status, nthreads);
}
int orc_decode_fast_batch(const uint8_t *in, const uint64_t *in_off, uint64_t n, uint8_t *out,
                          const uint64_t *out_off, uint32_t *out_len, uint8_t *status, int nthreads) {
  return orc_run(3, in, in_off, n, out, out_off, out_len, status, nthreads);
}
