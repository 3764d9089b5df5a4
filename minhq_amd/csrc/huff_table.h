// huff_table.h -- RFC 7541 Appendix B canonical Huffman code and the decode
// tables the gfx950 kernels stage into LDS.
//
// The code itself is hc/huffmantable.go:9-267 (256 symbols, EOS at
// hc/huffmantable.go:266 deliberately absent).  It is canonical, so only the
// code lengths are stored; code values are rebuilt in (length, symbol) order,
// exactly as the reference's values were assigned (checked against the
// reference table by tests/test_oracle.py::test_product_tables_match_reference).
#pragma once
#include <stdint.h>

namespace mhq {

constexpr int kLut1Bits = 12;                 // first-level multi-symbol LUT index width
constexpr int kLut1Size = 1 << kLut1Bits;     // 4096 x u32 = 16 KiB of LDS
constexpr int kLut2SubBits = 5;               // bits after the first 0 of a long code
constexpr int kLut2Size = 32 << kLut2SubBits; // [leading ones 0..31][5 bits] x u16
constexpr int kEosOnes = 30;                  // all-ones prefix where EOS would be
// A code starting with kLongOnes ones is longer than kLut1Bits (the 12-bit
// codes 0xffa/0xffb have 9): its LUT1 entry is 0, so a decoder may go to LUT2
// at once.  build_tables() checks it.
constexpr int kLongOnes = 10;

// LUT1 entry layout (u32), one field per byte so the decode loop can use
// each field straight from the entry (a 64-bit shift takes its count from
// bits [5:0]; SDWA operands select a byte or half-word):
//   [7:0] total bits  [15:8] 8 * nsym  [23:16] sym0  [31:24] sym1 (0 for one-symbol entries)
// An entry of 0: the first code is longer than 12 bits (or is the all-ones EOS
// prefix) -> LUT2 path.
constexpr uint32_t lut1_entry(uint32_t s0, uint32_t s1, uint32_t tot, uint32_t ns) {
  return ns ? (tot | ((ns * 8u) << 8) | (s0 << 16) | (s1 << 24)) : 0u;
}
// LUT2 entry layout (u16): [7:0] sym  [12:8] len (0 = no code).

static const uint8_t kCodeLen[256] = {
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

struct Tables {
  uint32_t code[256];   // right-justified code value (huffmanTableItem.val)
  uint8_t len[256];     // code length (huffmanTableItem.len)
  uint32_t lut1[kLut1Size];
  uint16_t lut2[kLut2Size];
};

// Builds every table once on the host; returns false if the code violates an
// assumption the kernels rely on (it cannot for the fixed RFC 7541 code).
bool build_tables(Tables *t);

}  // namespace mhq
