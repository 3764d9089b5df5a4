// ubench_loop.hip -- inner-loop variants of the short-literal decode, timed
// alone on an LDS-resident hdr-like stream (no literal ends), chip-wide.
//
// Variants (template V):
//   0  the kernel's masked step pair (BitBufM / OutAcc / Pend: two 12-bit
//      LUT1 probes per step, LUT2 branch in the second step, refill, ds_or)
//   1  variant 0 with two independent chains per lane, interleaved
//   2  one 8-bit probe per symbol (T8, 16 bank-interleaved copies), four
//      probes per step, LUT2 at the step's first probe only
//   3  variant 0 with a third LUT1 probe per step
//   4-11  variant 0 with one change (kMode below); 12 one output store per two steps
// Prints G symbols/s chip-wide and cycles per step per wave for 8/12/16
// waves per CU.  Every variant checks its bytes against the symbol stream.
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I minhq_amd/csrc \
//     tools/ubench/ubench_loop.hip minhq_amd/csrc/huff_table.cpp -o tools/ubench/ubench_loop
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <vector>

#include "huff_table.h"

#define CHECK(x)                                                                        \
  do {                                                                                  \
    hipError_t e_ = (x);                                                                \
    if (e_ != hipSuccess) {                                                             \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      exit(1);                                                                          \
    }                                                                                   \
  } while (0)

using namespace mhq;

constexpr int kStreamBytes = 32768;
constexpr int kStreamWords = kStreamBytes / 4;
constexpr int kOutWords = 4096;
constexpr int kT8Copies = 16;

struct Smem {
  uint32_t lut1[kLut1Size];
  uint16_t lut2[kLut2Size];
  uint32_t t8[256 * kT8Copies];
  uint32_t lut1x2[2 * kLut1Size];  // LUT1 twice, interleaved: entry i of copy c at 2i + c
  uint32_t in_w[kStreamWords + 8];  // byte-swapped words (MSB-first stream)
  uint32_t out_w[kOutWords];
};

__device__ __forceinline__ uint32_t ones_past(int32_t d) {
  const uint32_t c = (uint32_t)min(max(d, 0), 32);
  return (uint32_t)(0xffffffffull >> c);
}

struct BitBufM {
  uint64_t bb;
  int32_t left, rem;
  uint32_t wi;
  __device__ __forceinline__ void init(const uint32_t *words, uint32_t p0, uint32_t endbit) {
    const uint32_t k = p0 >> 5;
    const int32_t e = (int32_t)endbit - (int32_t)(32u * k);
    const uint32_t w0 = words[k] | ones_past(e), w1 = words[k + 1] | ones_past(e - 32);
    bb = (((uint64_t)w0 << 32) | w1) << (p0 & 31u);
    rem = e - 64;
    wi = k + 2u;
    left = (int32_t)(endbit - p0);
  }
  __device__ __forceinline__ void refill(uint32_t w) {
    const int32_t nb = left - rem;
    const bool need = nb <= 32;
    bb |= (uint64_t)(need ? (w | ones_past(rem)) : 0u) << ((uint32_t)(32 - nb) & 63u);
    rem -= need ? 32 : 0;
    wi += need ? 1u : 0u;
  }
  __device__ __forceinline__ uint32_t top32() const { return (uint32_t)(bb >> 32); }
  __device__ __forceinline__ void consume(uint32_t e) {
    bb <<= (e & 63u);
    left -= (int32_t)(e & 0xffu);
  }
};

struct OutAcc {
  uint64_t acc;
  uint32_t ow, ab;
  __device__ __forceinline__ void init(uint32_t optr) {
    acc = 0;
    ow = optr >> 2;
    ab = (optr & 3u) * 8u;
  }
  __device__ __forceinline__ void put(uint32_t syms, uint32_t nbits) {
    acc |= (uint64_t)syms << ab;
    ab += nbits;
  }
};

struct Pend {
  uint32_t ow, v;
};

__device__ __forceinline__ uint32_t long_code(const uint16_t *lut2, uint32_t win, uint32_t &sym) {
  const uint32_t nw = ~win;
  const uint32_t c = nw ? (uint32_t)__builtin_clz(nw) : 32u;
  if (c >= (uint32_t)kEosOnes) return 0;
  const uint32_t e2 = lut2[(c << kLut2SubBits) | ((win << (c + 1)) >> (32 - kLut2SubBits))];
  sym = e2 & 0xffu;
  return e2 >> 8;
}

// kMode: 0 plain; 4 both probes from a global (L1-resident) LUT1; 5 the
// second probe from it; 6 LUT1 from two copies by lane parity; 7 no output
// ds_or; 8 no refill read (timing only).
template <bool kLong, bool kP3, int kMode = 0>
__device__ __forceinline__ uint32_t lut1_probe(const Smem &sm, const uint32_t *__restrict__ glut, uint32_t S,
                                               uint32_t lane, int which) {
  const uint32_t i = S >> (32 - kLut1Bits);
  if (kMode == 4 || (kMode == 5 && which == 2)) return glut[i];
  if (kMode == 6) return sm.lut1x2[2u * i + (lane & 1u)];
  return sm.lut1[i];
}
template <bool kLong, bool kP3, int kMode = 0>
__device__ __forceinline__ bool masked_step(const Smem &sm, uint32_t *otgt, BitBufM &in, OutAcc &out, Pend &pend,
                                            bool &stop, const uint32_t *__restrict__ glut = nullptr,
                                            uint32_t lane = 0) {
  const uint32_t S = in.top32();
  stop = S >= 0xfffffffcu;
  uint32_t e = lut1_probe<kLong, kP3, kMode>(sm, glut, S, lane, 1);
  if (kMode == 9) otgt[pend.ow & (kOutWords - 1u)] = pend.v;
  else if (kMode == 10) { if (pend.v) otgt[pend.ow & (kOutWords - 1u)] = pend.v; }
  else if (kMode == 11) { if (pend.v) atomicOr(&otgt[pend.ow & (kOutWords - 1u)], pend.v); }
  else if (kMode != 7) atomicOr(&otgt[pend.ow & (kOutWords - 1u)], pend.v);
  const uint32_t w = kMode == 8 ? in.wi * 0x9e3779b9u : sm.in_w[in.wi];
  bool lng = false;
  if (kLong && ((e == 0u) & !stop)) {
    uint32_t sym = 0;
    const uint32_t L = long_code(sm.lut2, S, sym);
    e = L | (8u << 8) | (sym << 16);
    lng = true;
  }
  out.put(e >> 16, (e >> 8) & 0xffu);
  in.consume(e);
  uint32_t e2 = lut1_probe<kLong, kP3, kMode>(sm, glut, in.top32(), lane, 2);
  e2 = lng ? 0u : e2;
  out.put(e2 >> 16, (e2 >> 8) & 0xffu);
  in.consume(e2);
  if (kP3) {
    uint32_t e3 = sm.lut1[in.top32() >> (32 - kLut1Bits)];
    const int32_t nb = in.left - in.rem;
    const bool take = (int32_t)(e3 & 0xffu) + 2 <= nb && out.ab + ((e3 >> 8) & 0xffu) <= 63u;
    e3 = take ? e3 : 0u;
    out.put(e3 >> 16, (e3 >> 8) & 0xffu);
    in.consume(e3);
  }
  in.refill(w);
  const bool ok = in.left >= 0;
  pend.ow = out.ow;
  pend.v = ok ? (uint32_t)out.acc : 0u;
  if (kMode == 10 || kMode == 11) pend.v = out.ab >= 32u ? pend.v | 1u : 0u;  // (timing only)
  out.acc >>= out.ab & 32u;
  out.ow += out.ab >> 5;
  out.ab &= 31u;
  return stop || !ok;
}

// T8 step: refill to >= 33 bits, probe 0 reads T8 and LUT2 together (a code
// of 10+ bits ends the step), probes 1..3 T8 only (<= 8 bits each).
__device__ __forceinline__ bool t8_step(const Smem &sm, uint32_t *otgt, BitBufM &in, OutAcc &out, Pend &pend,
                                        uint32_t lane16) {
  const uint32_t S = in.top32();
  const bool stop = S >= 0xfffffffcu;
  uint32_t e = sm.t8[((S >> 24) << 4) | lane16];
  const uint32_t nw = ~S;
  const uint32_t c = min(nw ? (uint32_t)__builtin_clz(nw) : 32u, (uint32_t)kEosOnes - 1u);
  const uint32_t l2 = sm.lut2[(c << kLut2SubBits) | ((S << (c + 1u)) >> (32 - kLut2SubBits))];
  atomicOr(&otgt[pend.ow & (kOutWords - 1u)], pend.v);
  const uint32_t w = sm.in_w[in.wi];
  const bool lng = e == 0u;
  e = lng ? (stop ? 0u : ((l2 >> 8) | (8u << 8) | ((l2 & 0xffu) << 16))) : e;
  out.put(e >> 16, (e >> 8) & 0xffu);
  in.consume(e);
#pragma unroll
  for (int k = 0; k < 3; k++) {
    uint32_t ek = sm.t8[((in.top32() >> 24) << 4) | lane16];
    ek = lng ? 0u : ek;
    out.put(ek >> 16, (ek >> 8) & 0xffu);
    in.consume(ek);
  }
  in.refill(w);
  const bool ok = in.left >= 0;
  pend.ow = out.ow;
  pend.v = ok ? (uint32_t)out.acc : 0u;
  out.acc >>= out.ab & 32u;
  out.ow += out.ab >> 5;
  out.ab &= 31u;
  return stop || !ok;
}

struct Chain {
  BitBufM in;
  OutAcc out;
  Pend pend;
  uint32_t ow0, p0, endbit, bits;
  __device__ void init(const Smem &sm, uint32_t p, uint32_t eb, uint32_t optr) {
    p0 = p;
    endbit = eb;
    in.init(sm.in_w, p, eb);
    out.init(optr);
    ow0 = out.ow;
    pend = Pend{out.ow, 0u};
    bits = 0;
  }
  __device__ __forceinline__ void wrap(const Smem &sm) {
    if (in.left < 4096) {  // restart at the chain's start (rare)
      bits += (out.ow - ow0) * 32u + out.ab;
      in.init(sm.in_w, p0, endbit);
      out.ow = ow0;
      out.ab = 0;
      out.acc = 0;
    }
  }
  __device__ uint32_t total() const { return bits + (out.ow - ow0) * 32u + out.ab; }
};

template <int V>
__device__ uint32_t run(Smem &sm, uint32_t p0, uint32_t p1, uint32_t eb, uint32_t iters, uint32_t lane,
                        const uint32_t *__restrict__ glut) {
  Chain a, b;
  a.init(sm, p0, eb, (threadIdx.x & 1023u) * 60u);  // 15-word stride: banks spread
  if (V == 1) b.init(sm, p1, eb, (threadIdx.x & 1023u) * 60u + 30u * 1024u);
  bool stop;
  for (uint32_t i = 0; i < iters; i++) {
    if (V == 12) {  // one output store per two steps (timing only: the first step stores nothing)
      masked_step<false, false, 7>(sm, sm.out_w, a.in, a.out, a.pend, stop, glut, lane);
      masked_step<true, false, 0>(sm, sm.out_w, a.in, a.out, a.pend, stop, glut, lane);
    } else if (V >= 4) {
      masked_step<false, false, V>(sm, sm.out_w, a.in, a.out, a.pend, stop, glut, lane);
      masked_step<true, false, V>(sm, sm.out_w, a.in, a.out, a.pend, stop, glut, lane);
    } else if (V == 0 || V == 1 || V == 3) {
      masked_step<false, V == 3>(sm, sm.out_w, a.in, a.out, a.pend, stop);
      if (V == 1) masked_step<false, false>(sm, sm.out_w, b.in, b.out, b.pend, stop);
      masked_step<true, V == 3>(sm, sm.out_w, a.in, a.out, a.pend, stop);
      if (V == 1) masked_step<true, false>(sm, sm.out_w, b.in, b.out, b.pend, stop);
    } else {
      t8_step(sm, sm.out_w, a.in, a.out, a.pend, lane & 15u);
    }
    a.wrap(sm);
    if (V == 1) b.wrap(sm);
  }
  return a.total() + (V == 1 ? b.total() : 0u);
}

// Correctness: one chain per lane decodes from its start for `iters` steps
// into a private global region; the host compares with the symbol stream.
template <int V>
__global__ __launch_bounds__(1024) void check_kernel(const uint32_t *g_lut1, const uint16_t *g_lut2,
                                                     const uint32_t *g_t8, const uint32_t *g_words,
                                                     const uint32_t *starts, uint32_t *g_out) {
  __shared__ Smem sm;
  const uint32_t tid = threadIdx.x;
  for (uint32_t i = tid; i < kLut1Size; i += blockDim.x) sm.lut1[i] = g_lut1[i];
  for (uint32_t i = tid; i < kLut2Size; i += blockDim.x) sm.lut2[i] = g_lut2[i];
  for (uint32_t i = tid; i < 256 * kT8Copies; i += blockDim.x) sm.t8[i] = g_t8[i];
  for (uint32_t i = tid; i < 2 * kLut1Size; i += blockDim.x) sm.lut1x2[i] = g_lut1[i >> 1];
  for (uint32_t i = tid; i < kStreamWords + 8; i += blockDim.x) sm.in_w[i] = i < kStreamWords ? g_words[i] : ~0u;
  for (uint32_t i = tid; i < kOutWords; i += blockDim.x) sm.out_w[i] = 0;
  __syncthreads();
  const uint32_t lane = tid & 63u;
  Chain a;
  a.init(sm, starts[tid], kStreamBytes * 8u - 64u, tid * 4u * 16u);  // 64 B per thread: 16 words
  bool stop;
  for (int i = 0; i < 6; i++) {  // <= 48 symbols: fits 64 bytes
    if (V == 2)
      t8_step(sm, sm.out_w, a.in, a.out, a.pend, lane & 15u);
    else
      masked_step<true, V == 3>(sm, sm.out_w, a.in, a.out, a.pend, stop);
  }
  atomicOr(&sm.out_w[a.pend.ow & (kOutWords - 1u)], a.pend.v);
  atomicOr(&sm.out_w[a.out.ow & (kOutWords - 1u)], (uint32_t)a.out.acc);  // the partial word
  __syncthreads();
  for (uint32_t k = 0; k < 16; k++) g_out[tid * 17 + k] = sm.out_w[(tid * 16 + k) & (kOutWords - 1u)];
  g_out[tid * 17 + 16] = (a.out.ow - tid * 16u) * 4u + a.out.ab / 8u;  // bytes decoded
}

template <int V>
__global__ __launch_bounds__(1024) void ubench(const uint32_t *g_lut1, const uint16_t *g_lut2, const uint32_t *g_t8,
                                               const uint32_t *g_words, const uint32_t *starts, uint32_t nstarts,
                                               uint32_t iters, uint32_t *sink, unsigned long long *sym_bits,
                                               unsigned long long *cycles) {
  __shared__ Smem sm;
  const uint32_t tid = threadIdx.x;
  for (uint32_t i = tid; i < kLut1Size; i += blockDim.x) sm.lut1[i] = g_lut1[i];
  for (uint32_t i = tid; i < kLut2Size; i += blockDim.x) sm.lut2[i] = g_lut2[i];
  for (uint32_t i = tid; i < 256 * kT8Copies; i += blockDim.x) sm.t8[i] = g_t8[i];
  for (uint32_t i = tid; i < 2 * kLut1Size; i += blockDim.x) sm.lut1x2[i] = g_lut1[i >> 1];
  for (uint32_t i = tid; i < kStreamWords + 8; i += blockDim.x) sm.in_w[i] = i < kStreamWords ? g_words[i] : ~0u;
  for (uint32_t i = tid; i < kOutWords; i += blockDim.x) sm.out_w[i] = 0;
  __syncthreads();
  const uint32_t g = blockIdx.x * blockDim.x + tid;
  const uint32_t p0 = starts[(g * 7919u) % nstarts];
  const uint32_t p1 = starts[(g * 104729u + 17u) % nstarts];
  const unsigned long long t0 = clock64();
  const uint32_t bits = run<V>(sm, p0, p1, kStreamBytes * 8u - 64u, iters, tid & 63u, g_lut1);
  const unsigned long long t1 = clock64();
  __syncthreads();
  sink[g & ((1u << 20) - 1u)] = bits + sm.out_w[tid & (kOutWords - 1u)];
  atomicAdd(sym_bits, (unsigned long long)bits);
  if ((tid & 63u) == 0) atomicAdd(cycles, t1 - t0);
}

static uint64_t rng_state = 0x1234567;
static uint64_t rnd() {
  rng_state ^= rng_state << 13;
  rng_state ^= rng_state >> 7;
  rng_state ^= rng_state << 17;
  return rng_state;
}

int main(int argc, char **argv) {
  const uint32_t iters = argc > 1 ? (uint32_t)atoi(argv[1]) : 1000;
  Tables t;
  if (!build_tables(&t)) return 1;
  // T8: codes of <= 8 bits from the top 8 bits: len | 8 << 8 | sym << 16, 0 otherwise
  std::vector<uint32_t> t8(256 * kT8Copies, 0);
  for (uint32_t idx = 0; idx < 256; idx++) {
    uint32_t ent = 0;
    for (int s = 0; s < 256; s++) {
      const int L = t.len[s];
      if (L <= 8 && (idx >> (8 - L)) == t.code[s]) ent = (uint32_t)L | (8u << 8) | ((uint32_t)s << 16);
    }
    for (int c = 0; c < kT8Copies; c++) t8[idx * kT8Copies + c] = ent;
  }
  // LUT2 must also hold the 10..12-bit codes for T8
  std::vector<uint16_t> lut2(t.lut2, t.lut2 + kLut2Size);
  for (int s = 0; s < 256; s++) {
    const int L = t.len[s];
    if (L < 10 || L > kLut1Bits) continue;
    const uint32_t c = t.code[s];
    int ones = 0;
    while (ones < L && ((c >> (L - 1 - ones)) & 1u)) ones++;
    const int rest = L - ones - 1;
    if (rest > kLut2SubBits) return 2;
    const uint32_t base = (uint32_t)ones << kLut2SubBits, lo = (c & ((1u << rest) - 1u)) << (kLut2SubBits - rest);
    for (uint32_t k = 0; k < (1u << (kLut2SubBits - rest)); k++) {
      if (lut2[base + lo + k] != 0) return 3;
      lut2[base + lo + k] = (uint16_t)(s | (L << 8));
    }
  }
  static const int hist[95] = {163, 0, 0, 0, 0, 0, 0, 0, 18, 18, 36, 1, 41, 162, 181, 165, 183, 74, 19, 0, 36, 72, 36, 0,
                               37, 1, 107, 75, 0, 22, 0, 0, 0, 0, 2, 1, 1, 18, 19, 36, 0, 0, 0, 0, 0, 19, 19, 0,
                               2, 0, 0, 21, 37, 19, 0, 36, 0, 1, 0, 0, 0, 0, 0, 4, 0, 331, 45, 343, 115, 540, 57, 180,
                               163, 198, 4, 41, 135, 78, 326, 301, 187, 22, 211, 130, 324, 61, 38, 125, 41, 22, 36,
                               0, 0, 0, 0};
  std::vector<double> cdf(95);
  double tot = 0, acc = 0;
  for (int i = 0; i < 95; i++) tot += hist[i] + 1;
  for (int i = 0; i < 95; i++) cdf[i] = (acc += (hist[i] + 1) / tot);
  std::vector<uint8_t> bytes(kStreamBytes, 0);
  std::vector<uint32_t> starts;
  std::vector<int> symat;  // symbol index of each start
  std::vector<uint8_t> syms;
  uint64_t bit = 0;
  const uint64_t limit = (uint64_t)kStreamBytes * 8 - 64;
  while (true) {
    const double u = (rnd() >> 11) * (1.0 / 9007199254740992.0);
    int s = 0;
    while (s < 94 && cdf[s] < u) s++;
    const int sym = 0x20 + s;
    const int L = t.len[sym];
    if (bit + L > limit) break;
    if (bit < (uint64_t)kStreamBytes * 8 / 2) {
      starts.push_back((uint32_t)bit);
      symat.push_back((int)syms.size());
    }
    syms.push_back((uint8_t)sym);
    for (int b = L - 1; b >= 0; b--, bit++)
      if ((t.code[sym] >> b) & 1u) bytes[bit >> 3] |= (uint8_t)(0x80u >> (bit & 7));
  }
  std::vector<uint32_t> words(kStreamWords);
  for (int i = 0; i < kStreamWords; i++)
    words[i] = (uint32_t)bytes[4 * i] << 24 | bytes[4 * i + 1] << 16 | bytes[4 * i + 2] << 8 | bytes[4 * i + 3];
  uint32_t *d_lut1, *d_t8, *d_words, *d_starts, *d_sink, *d_out;
  uint16_t *d_lut2;
  unsigned long long *d_cyc, *d_bits;
  CHECK(hipMalloc(&d_lut1, sizeof(t.lut1)));
  CHECK(hipMalloc(&d_lut2, lut2.size() * 2));
  CHECK(hipMalloc(&d_t8, t8.size() * 4));
  CHECK(hipMalloc(&d_words, words.size() * 4));
  CHECK(hipMalloc(&d_starts, starts.size() * 4));
  CHECK(hipMalloc(&d_sink, (1 << 20) * 4));
  CHECK(hipMalloc(&d_out, 1024 * 17 * 4));
  CHECK(hipMalloc(&d_cyc, 8));
  CHECK(hipMalloc(&d_bits, 8));
  CHECK(hipMemcpy(d_lut1, t.lut1, sizeof(t.lut1), hipMemcpyHostToDevice));
  CHECK(hipMemcpy(d_lut2, lut2.data(), lut2.size() * 2, hipMemcpyHostToDevice));
  CHECK(hipMemcpy(d_t8, t8.data(), t8.size() * 4, hipMemcpyHostToDevice));
  CHECK(hipMemcpy(d_words, words.data(), words.size() * 4, hipMemcpyHostToDevice));
  CHECK(hipMemcpy(d_starts, starts.data(), starts.size() * 4, hipMemcpyHostToDevice));
  int dev = 0, cus = 0;
  CHECK(hipGetDevice(&dev));
  CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
  // correctness of the step variants (one chain per lane, from starts[tid])
  auto verify = [&](int v) {
    if (v == 0) check_kernel<0><<<1, 256>>>(d_lut1, d_lut2, d_t8, d_words, d_starts, d_out);
    if (v == 2) check_kernel<2><<<1, 256>>>(d_lut1, d_lut2, d_t8, d_words, d_starts, d_out);
    if (v == 3) check_kernel<3><<<1, 256>>>(d_lut1, d_lut2, d_t8, d_words, d_starts, d_out);
    CHECK(hipDeviceSynchronize());
    std::vector<uint32_t> o(256 * 17);
    CHECK(hipMemcpy(o.data(), d_out, o.size() * 4, hipMemcpyDeviceToHost));
    int bad = 0;
    long total = 0;
    for (int tid = 0; tid < 256; tid++) {
      const uint32_t nb = o[tid * 17 + 16];
      total += nb;
      const uint8_t *b8 = (const uint8_t *)&o[tid * 17];
      for (uint32_t k = 0; k < nb && k < 64; k++)
        if (b8[k] != syms[symat[tid] + k]) {
          bad++;
          break;
        }
    }
    printf("variant %d check: %s (%.1f bytes per chain in 6 steps)\n", v, bad ? "MISMATCH" : "ok", total / 256.0);
    if (bad) exit(1);
  };
  verify(0);
  verify(2);
  verify(3);
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  const int wavess[] = {8, 12, 16};
  const char *only = argc > 2 ? argv[2] : nullptr;  // comma-separated variants to time (default: all but 2, 3)
  for (int v = 0; v < 13; v++) {
    if (only) {
      char key[8];
      snprintf(key, sizeof key, "%d", v);
      bool hit = false;
      for (const char *p = only; *p;) {
        const char *q = strchr(p, ',');
        const size_t len = q ? (size_t)(q - p) : strlen(p);
        if (len == strlen(key) && !strncmp(p, key, len)) hit = true;
        p += len + (q ? 1 : 0);
      }
      if (!hit) continue;
    } else if (v >= 2 && v <= 3) {
      continue;
    }
    for (int waves : wavess) {
      auto launch = [&]() {
        dim3 grid(cus), block(waves * 64);
        const uint32_t ns = (uint32_t)starts.size();
        if (v == 0) ubench<0><<<grid, block>>>(d_lut1, d_lut2, d_t8, d_words, d_starts, ns, iters, d_sink, d_bits, d_cyc);
        if (v == 1) ubench<1><<<grid, block>>>(d_lut1, d_lut2, d_t8, d_words, d_starts, ns, iters, d_sink, d_bits, d_cyc);
        if (v == 2) ubench<2><<<grid, block>>>(d_lut1, d_lut2, d_t8, d_words, d_starts, ns, iters, d_sink, d_bits, d_cyc);
        if (v == 3) ubench<3><<<grid, block>>>(d_lut1, d_lut2, d_t8, d_words, d_starts, ns, iters, d_sink, d_bits, d_cyc);
        if (v == 4) ubench<4><<<grid, block>>>(d_lut1, d_lut2, d_t8, d_words, d_starts, ns, iters, d_sink, d_bits, d_cyc);
        if (v == 5) ubench<5><<<grid, block>>>(d_lut1, d_lut2, d_t8, d_words, d_starts, ns, iters, d_sink, d_bits, d_cyc);
        if (v == 6) ubench<6><<<grid, block>>>(d_lut1, d_lut2, d_t8, d_words, d_starts, ns, iters, d_sink, d_bits, d_cyc);
        if (v == 7) ubench<7><<<grid, block>>>(d_lut1, d_lut2, d_t8, d_words, d_starts, ns, iters, d_sink, d_bits, d_cyc);
        if (v == 9) ubench<9><<<grid, block>>>(d_lut1, d_lut2, d_t8, d_words, d_starts, ns, iters, d_sink, d_bits, d_cyc);
        if (v == 10) ubench<10><<<grid, block>>>(d_lut1, d_lut2, d_t8, d_words, d_starts, ns, iters, d_sink, d_bits, d_cyc);
        if (v == 12) ubench<12><<<grid, block>>>(d_lut1, d_lut2, d_t8, d_words, d_starts, ns, iters, d_sink, d_bits, d_cyc);
        if (v == 11) ubench<11><<<grid, block>>>(d_lut1, d_lut2, d_t8, d_words, d_starts, ns, iters, d_sink, d_bits, d_cyc);
        if (v == 8) ubench<8><<<grid, block>>>(d_lut1, d_lut2, d_t8, d_words, d_starts, ns, iters, d_sink, d_bits, d_cyc);
      };
      launch();
      CHECK(hipDeviceSynchronize());
      CHECK(hipMemset(d_cyc, 0, 8));
      CHECK(hipMemset(d_bits, 0, 8));
      const int reps = 5;
      CHECK(hipEventRecord(e0));
      for (int r = 0; r < reps; r++) launch();
      CHECK(hipEventRecord(e1));
      CHECK(hipEventSynchronize(e1));
      float ms = 0;
      CHECK(hipEventElapsedTime(&ms, e0, e1));
      unsigned long long cyc = 0, bits = 0;
      CHECK(hipMemcpy(&cyc, d_cyc, 8, hipMemcpyDeviceToHost));
      CHECK(hipMemcpy(&bits, d_bits, 8, hipMemcpyDeviceToHost));
      const double symbols = (double)bits / 8.0;
      const double wave_cyc = (double)cyc / ((double)cus * waves * reps);
      printf("variant %d waves/CU %2d: %7.3f ms  %8.1f G sym/s  cycles/iter/wave %6.1f  sym/iter/lane %.2f\n", v,
             waves, ms / reps, symbols / (ms * 1e-3) / 1e9, wave_cyc / iters,
             symbols / ((double)cus * waves * 64 * reps * iters));
    }
  }
  return 0;
}
