// huff_table.cpp -- host-side construction of the code and decode tables.
#include "huff_table.h"

#include <algorithm>
#include <string.h>

namespace mhq {

namespace {

// Decodes one code from the MSB-aligned `bits`-wide window `w` by direct
// comparison against every code (host only, run once per table entry).
// Returns the symbol, or -1 if no code of length <= bits is a prefix of w.
int match_code(const Tables &t, uint32_t w, int bits, int *len_out) {
  for (int s = 0; s < 256; s++) {
    int L = t.len[s];
    if (L > bits) continue;
    if ((w >> (bits - L)) == t.code[s]) {
      *len_out = L;
      return s;
    }
  }
  return -1;
}

}  // namespace

bool build_tables(Tables *t) {
  memset(t, 0, sizeof(*t));
  // Canonical code values: codes assigned in (length, symbol) order.
  int order[256];
  for (int i = 0; i < 256; i++) order[i] = i;
  std::stable_sort(order, order + 256, [](int a, int b) { return kCodeLen[a] < kCodeLen[b]; });
  uint32_t code = 0;
  int prev = kCodeLen[order[0]];
  for (int i = 0; i < 256; i++) {
    int s = order[i];
    if (i > 0) code = (code + 1u) << (kCodeLen[s] - prev);
    prev = kCodeLen[s];
    t->code[s] = code;
    t->len[s] = kCodeLen[s];
  }

  // every code with kLongOnes leading ones is longer than LUT1's index
  for (int s = 0; s < 256; s++) {
    const uint32_t top = t->code[s] << (32 - t->len[s]);
    if (top >= (~0u << (32 - kLongOnes)) && t->len[s] <= kLut1Bits) return false;
  }

  // LUT1: up to two symbols from the next 12 bits.
  for (uint32_t idx = 0; idx < (uint32_t)kLut1Size; idx++) {
    int l0 = 0;
    int s0 = match_code(*t, idx, kLut1Bits, &l0);
    if (s0 < 0) {
      t->lut1[idx] = lut1_entry(0, 0, 0, 0);
      continue;
    }
    int rest = kLut1Bits - l0;
    uint32_t wrest = idx & ((1u << rest) - 1u);
    int l1 = 0;
    int s1 = rest > 0 ? match_code(*t, wrest, rest, &l1) : -1;
    if (s1 >= 0)
      t->lut1[idx] = lut1_entry((uint32_t)s0, (uint32_t)s1, (uint32_t)(l0 + l1), 2);
    else
      t->lut1[idx] = lut1_entry((uint32_t)s0, 0, (uint32_t)l0, 1);
  }

  // LUT2: codes longer than 12 bits, keyed by their count of leading ones
  // and the (at most 5) bits that follow the first zero.
  for (int s = 0; s < 256; s++) {
    int L = t->len[s];
    if (L <= kLut1Bits) continue;
    uint32_t c = t->code[s];
    int ones = 0;
    while (ones < L && ((c >> (L - 1 - ones)) & 1u)) ones++;
    if (ones >= L || ones >= 32) return false;  // an all-ones code: only EOS, absent
    int rest = L - ones - 1;
    if (rest > kLut2SubBits) return false;
    uint32_t rbits = c & ((1u << rest) - 1u);
    uint32_t base = (uint32_t)ones << kLut2SubBits;
    uint32_t lo = rbits << (kLut2SubBits - rest);
    uint32_t span = 1u << (kLut2SubBits - rest);
    for (uint32_t k = 0; k < span; k++) {
      uint16_t &slot = t->lut2[base + lo + k];
      if (slot != 0) return false;  // not prefix free
      slot = (uint16_t)(s | (L << 8));
    }
  }
  // Every 12-bit window that LUT1 cannot resolve must start with >= 10 ones
  // (checked implicitly by the kernels' use of LUT2); the LUT2 rows the
  // kernels may index are 0..31, all present.
  return true;
}

}  // namespace mhq
