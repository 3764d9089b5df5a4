/* huff_oracle.h -- TEST INFRASTRUCTURE ONLY (see huff_oracle.c header). */
#ifndef MHQ_HUFF_ORACLE_H
#define MHQ_HUFF_ORACLE_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

enum {
  ORC_OK = 0,
  ORC_INVALID = 1,          /* errors.New("invalid Huffman coding"), hc/huffman.go:112 */
  ORC_ERR_EOF = -1,         /* io.EOF */
  ORC_ERR_TOO_LARGE = -2,   /* bytes.ErrTooLarge, io/bitio.go:73-77 */
  ORC_ERR_SHORT_WRITE = -3, /* io.ErrShortWrite */
  ORC_ERR_OVERFLOW = -4,    /* ErrIntegerOverflow, hc/io.go:12 */
  ORC_ERR_NOMEM = -5,
};

void orc_init(void);
void orc_table(uint8_t *len, uint32_t *val);
int orc_tree_nodes(void);

typedef struct orc_bitwriter orc_bitwriter;
orc_bitwriter *orc_bw_new(uint8_t *out, size_t cap);
int orc_bw_write_bits(orc_bitwriter *w, uint64_t v, uint8_t count);
int orc_bw_pad(orc_bitwriter *w, uint8_t pad);
size_t orc_bw_written(orc_bitwriter *w);
void orc_bw_free(orc_bitwriter *w);

size_t orc_huff_encoded_len(const uint8_t *in, size_t len);
int orc_huff_encode(const uint8_t *in, size_t len, uint8_t *out, size_t cap, size_t *out_len);
int orc_huff_decode(const uint8_t *in, size_t len, uint8_t *out, size_t cap, size_t *out_len);

int orc_read_int(const uint8_t *in, size_t len, uint8_t skip_bits, uint8_t prefix, uint64_t *out,
                 size_t *consumed);
int orc_write_int(uint64_t v, uint8_t lead, uint8_t lead_bits, uint8_t prefix, uint8_t *out, size_t cap,
                  size_t *out_len);
int orc_read_varint(const uint8_t *in, size_t len, uint64_t *out, size_t *consumed);
int orc_write_varint(uint64_t v, uint8_t *out, size_t cap, size_t *out_len);
int orc_read_frame(const uint8_t *in, size_t len, uint8_t *type, uint64_t *plen, size_t *hdr_len);
int orc_read_string(const uint8_t *in, size_t len, uint8_t skip_bits, uint8_t prefix,
                    uint8_t *out, size_t cap, size_t *out_len, size_t *consumed);
int orc_write_string(const uint8_t *s, size_t len, uint8_t lead, uint8_t lead_bits,
                     uint8_t prefix, int choice, uint8_t *out, size_t cap, size_t *out_len);

int orc_encode_len_batch(const uint8_t *in, const uint64_t *in_off, uint64_t n, uint32_t *enc_len,
                         int nthreads);
int orc_encode_batch(const uint8_t *in, const uint64_t *in_off, uint64_t n, uint8_t *out,
                     const uint64_t *out_off, int nthreads);
int orc_decode_batch(const uint8_t *in, const uint64_t *in_off, uint64_t n, uint8_t *out,
                     const uint64_t *out_off, uint32_t *out_len, uint8_t *status, int nthreads);
/* Table-driven decode with orc_huff_decode's results (CPU baseline only). */
int orc_huff_decode_fast(const uint8_t *in, size_t len, uint8_t *out, size_t cap, size_t *out_len);
int orc_decode_fast_batch(const uint8_t *in, const uint64_t *in_off, uint64_t n, uint8_t *out,
                          const uint64_t *out_off, uint32_t *out_len, uint8_t *status, int nthreads);

#ifdef __cplusplus
}
#endif
#endif
