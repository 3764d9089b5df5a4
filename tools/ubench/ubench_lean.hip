// ubench_lean.hip -- the "lean" short-literal decode step, timed alone on an
// LDS-resident hdr-like stream (no literal ends), against ubench_loop's
// variant 0 (the round-2 kernel's step).
//
// Lean step:
//   * the bit buffer is LSB-first (staged words bit-reversed), with the next
//     stream bit at bit 2: a LUT1 probe's LDS address is bb & 0x3ffc (one
//     VALU), consumption is one 64-bit right shift, a refill shifts the word
//     left by the valid-bit count (+2);
//   * LUT1L entry: [7:0] bits, [15:8] symbol count, [31:16] the symbols:
//     every probe stores its two symbol bytes straight to the output staging
//     (ds_write_b16_d16_hi at the byte pointer) and advances the pointer by
//     the count; a one-symbol probe's second byte is overwritten by the next
//     probe's first.  No output accumulator.
// Variants: 0 two probes per step; 1 three probes per step (refill before
// the third when needed).
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I minhq_amd/csrc \
//     tools/ubench/ubench_lean.hip minhq_amd/csrc/huff_table.cpp -o tools/ubench/ubench_lean
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

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
constexpr int kOutBytes = 65536;

struct Smem {
  uint32_t lut1[kLut1Size];        // LUT1L, indexed by the bit-reversed 12-bit window
  uint16_t lut2[kLut2Size];        // LUT2L: [leading ones][5 bits after the first zero, LSB-first]
  uint32_t in_w[kStreamWords + 8];  // LSB-first words: bit j of word k = stream bit 32k + j
  uint8_t out[kOutBytes];
};

typedef uint16_t u16u __attribute__((aligned(1)));

// ones at the bit positions >= r of an LSB-first word (r clamped to [0, 32])
__device__ __forceinline__ uint32_t ones_from(int32_t r) {
  const uint32_t c = (uint32_t)min(max(r, 0), 32);
  return (uint32_t)(~0ull << c);
}

// bb: stream bits from bit 2 up (bits 0-1 junk); left = endbit - p; rem2 =
// endbit - kb - 2 (kb: first stream bit not yet in bb), so the valid-bit
// count + 2 is left - rem2.
struct LeanBuf {
  uint64_t bb;
  int32_t left, rem2;
  uint32_t wi;
  // Tops the buffer up when it holds <= 30 valid bits (the next word enters
  // at bit valid + 2 = left - rem2); bits at or past the literal's end are ones.
  __device__ __forceinline__ void refill(uint32_t w) {
    const int32_t nb2 = left - rem2;
    const bool need = nb2 <= 32;
    const uint32_t wm = need ? (w | ones_from(rem2 + 2)) : 0u;
    bb |= (uint64_t)wm << ((uint32_t)nb2 & 63u);
    rem2 -= need ? 32 : 0;
    wi += need ? 1u : 0u;
  }
  __device__ __forceinline__ void init(const uint32_t *words, uint32_t p0, uint32_t endbit) {
    const uint32_t k = p0 >> 5;
    const int32_t e = (int32_t)endbit - (int32_t)(32u * k);
    bb = ((uint64_t)((words[k] | ones_from(e)) >> (p0 & 31u))) << 2;  // 32 - (p0 & 31) valid bits
    left = (int32_t)(endbit - p0);
    rem2 = e - 32 - 2;
    wi = k + 1u;
    refill(words[wi]);
  }
};

// LUT1L probe address: bb & 0x3ffc is 4 x the 12-bit window (byte address).
__device__ __forceinline__ uint32_t lut_at(const Smem &sm, uint64_t bb) {
  const uint32_t a = (uint32_t)bb & 0x3ffcu;
  return *(const uint32_t *)((const uint8_t *)sm.lut1 + a);
}

// Lean buffer with the round-2 output accumulator (64-bit, one ds_or per
// step): LUT1L entries with 8 * n in [15:8].
struct Acc {
  uint64_t acc;
  uint32_t ow, ab, pow, pv;
};
template <bool kLong>
__device__ __forceinline__ bool lean_acc_step(Smem &sm, LeanBuf &in, Acc &o, uint32_t &wnext) {
  const uint32_t lo = (uint32_t)in.bb;
  const bool stop = (lo | 3u) == 0xffffffffu;
  uint32_t e = lut_at(sm, in.bb);
  atomicOr((uint32_t *)(sm.out + (o.pow & 0xfffcu)), o.pv);
  const uint32_t w = wnext;
  bool lng = false;
  if (kLong && ((e == 0u) & !stop)) {
    const uint64_t x = in.bb >> 2;
    const uint32_t c = (uint32_t)__builtin_ctz(~(uint32_t)x);
    const uint32_t sub = (uint32_t)(x >> (c + 1u)) & 31u;
    const uint32_t e2 = sm.lut2[(c << kLut2SubBits) | sub];
    e = (e2 >> 8) | (8u << 8) | ((e2 & 0xffu) << 16);
    lng = true;
  }
  o.acc |= (uint64_t)(e >> 16) << o.ab;
  o.ab += (e >> 8) & 0xffu;
  in.bb >>= (e & 63u);
  uint32_t e2 = lut_at(sm, in.bb);
  e2 = lng ? 0u : e2;
  o.acc |= (uint64_t)(e2 >> 16) << o.ab;
  o.ab += (e2 >> 8) & 0xffu;
  in.bb >>= (e2 & 63u);
  in.left -= (int32_t)((e & 0xffu) + (e2 & 0xffu));
  in.refill(w);
  wnext = sm.in_w[in.wi];
  const bool ok = in.left >= 0;
  o.pow = o.ow * 4u;
  o.pv = ok ? (uint32_t)o.acc : 0u;
  o.acc >>= o.ab & 32u;
  o.ow += o.ab >> 5;
  o.ab &= 31u;
  return stop || !ok;
}

// One lean step (two probes, or three).  Returns true when the literal ended.
template <bool kLong, int kProbes>
__device__ __forceinline__ bool lean_step(Smem &sm, LeanBuf &in, uint32_t &optr, uint32_t &wnext) {
  const uint32_t lo = (uint32_t)in.bb;
  const bool stop = (lo | 3u) == 0xffffffffu;  // >= 30 ones: the EOS prefix
  uint32_t e = lut_at(sm, in.bb);
  const uint32_t w = wnext;
  bool lng = false;
  if (kLong && ((e == 0u) & !stop)) {  // a code of 13..29 bits
    const uint64_t x = in.bb >> 2;
    const uint32_t c = (uint32_t)__builtin_ctz(~(uint32_t)x);
    const uint32_t sub = (uint32_t)(x >> (c + 1u)) & 31u;
    const uint32_t e2 = sm.lut2[(c << kLut2SubBits) | sub];
    e = (e2 >> 8) | (1u << 8) | ((e2 & 0xffu) << 16);
    lng = true;
  }
  if (kProbes == 4) {  // byte stores (always aligned)
    sm.out[optr] = (uint8_t)(e >> 16);
    sm.out[optr + 1] = (uint8_t)(e >> 24);
  } else {
    *(u16u *)(sm.out + optr) = (uint16_t)(e >> 16);
  }
  optr += (e >> 8) & 0xffu;
  in.bb >>= (e & 63u);
  uint32_t e2 = lut_at(sm, in.bb);
  e2 = lng ? 0u : e2;
  if (kProbes == 4) {
    sm.out[optr] = (uint8_t)(e2 >> 16);
    sm.out[optr + 1] = (uint8_t)(e2 >> 24);
  } else {
    *(u16u *)(sm.out + optr) = (uint16_t)(e2 >> 16);
  }
  optr += (e2 >> 8) & 0xffu;
  in.bb >>= (e2 & 63u);
  uint32_t tot = (e & 0xffu) + (e2 & 0xffu);
  if (kProbes == 3) {
    // a third probe when 12 more bits are surely valid (>= 31 after the
    // refill, <= 24 consumed: needs nb - consumed >= 12)
    uint32_t e3 = lut_at(sm, in.bb);
    const int32_t nbv = in.left - in.rem2 - 2 - (int32_t)tot;
    e3 = (nbv >= 12 && !lng) ? e3 : 0u;
    *(u16u *)(sm.out + optr) = (uint16_t)(e3 >> 16);
    optr += (e3 >> 8) & 0xffu;
    in.bb >>= (e3 & 63u);
    tot += e3 & 0xffu;
  }
  in.left -= (int32_t)tot;
  in.refill(w);
  wnext = sm.in_w[in.wi];
  return stop || in.left < 0;
}

struct Chain {
  LeanBuf in;
  uint32_t optr, o0, p0, endbit, total, wnext;
  __device__ void init(const Smem &sm, uint32_t p, uint32_t eb, uint32_t o) {
    p0 = p;
    endbit = eb;
    in.init(sm.in_w, p, eb);
    optr = o0 = o;
    total = 0;
    wnext = sm.in_w[in.wi];
  }
  __device__ __forceinline__ void wrap(const Smem &sm, uint32_t omask) {
    if (in.left < 4096) {
      total += optr - o0;
      in.init(sm.in_w, p0, endbit);
      wnext = sm.in_w[in.wi];
      optr = o0;
    }
    if (optr - o0 > omask) {  // keep the writes in the lane's window
      total += optr - o0;
      optr = o0;
    }
  }
};

__device__ void load_tables(Smem &sm, const uint32_t *g_lut1, const uint16_t *g_lut2, const uint32_t *g_words) {
  const uint32_t tid = threadIdx.x;
  for (uint32_t i = tid; i < kLut1Size; i += blockDim.x) sm.lut1[i] = g_lut1[i];
  for (uint32_t i = tid; i < kLut2Size; i += blockDim.x) sm.lut2[i] = g_lut2[i];
  for (uint32_t i = tid; i < kStreamWords + 8; i += blockDim.x) sm.in_w[i] = i < kStreamWords ? g_words[i] : ~0u;
  __syncthreads();
}

template <int kProbes>
__global__ __launch_bounds__(256) void check_kernel(const uint32_t *g_lut1, const uint16_t *g_lut2,
                                                    const uint32_t *g_words, const uint32_t *starts,
                                                    uint8_t *g_out, uint32_t *g_n) {
  __shared__ Smem sm;
  load_tables(sm, g_lut1, g_lut2, g_words);
  const uint32_t tid = threadIdx.x;
  Chain a;
  a.init(sm, starts[tid], kStreamBytes * 8u - 64u, tid * 256u);
  for (int i = 0; i < 8; i++) lean_step<true, kProbes>(sm, a.in, a.optr, a.wnext);
  __syncthreads();
  for (uint32_t k = 0; k < 64; k++) g_out[tid * 64 + k] = sm.out[tid * 256 + k];
  g_n[tid] = a.optr - tid * 256u;
}

template <int kProbes>
__global__ __launch_bounds__(1024) void ubench(const uint32_t *g_lut1, const uint16_t *g_lut2, const uint32_t *g_words,
                                               const uint32_t *starts, uint32_t nstarts, uint32_t iters,
                                               uint32_t *sink, unsigned long long *sym_total,
                                               unsigned long long *cycles) {
  __shared__ Smem sm;
  load_tables(sm, g_lut1, g_lut2, g_words);
  const uint32_t tid = threadIdx.x;
  const uint32_t g = blockIdx.x * blockDim.x + tid;
  Chain a;
  a.init(sm, starts[(g * 7919u) % nstarts], kStreamBytes * 8u - 64u, (tid & 1023u) * 60u);  // 15-word stride: banks spread
  const unsigned long long t0 = clock64();
  Acc o{0, a.o0 / 4u, 0, a.o0, 0};
  const uint32_t ow0 = o.ow;
  for (uint32_t i = 0; i < iters; i++) {
    if (kProbes == 12) {
      lean_acc_step<false>(sm, a.in, o, a.wnext);
      lean_acc_step<true>(sm, a.in, o, a.wnext);
      if (a.in.left < 4096) {
        a.total += (o.ow - ow0) * 4u + o.ab / 8u;
        a.in.init(sm.in_w, a.p0, a.endbit);
        a.wnext = sm.in_w[a.in.wi];
        o.ow = ow0;
        o.ab = 0;
        o.acc = 0;
      }
      if (o.ow - ow0 > 8u) {
        a.total += (o.ow - ow0) * 4u;
        o.ow = ow0;
      }
    } else {
      lean_step<false, kProbes>(sm, a.in, a.optr, a.wnext);
      lean_step<true, kProbes>(sm, a.in, a.optr, a.wnext);
      a.wrap(sm, 32u);
    }
  }
  const unsigned long long t1 = clock64();
  __syncthreads();
  const uint32_t n = kProbes == 12 ? a.total + (o.ow - ow0) * 4u + o.ab / 8u : a.total + a.optr - a.o0;
  sink[g & ((1u << 20) - 1u)] = n + sm.out[tid];
  atomicAdd(sym_total, (unsigned long long)n);
  if ((tid & 63u) == 0) atomicAdd(cycles, t1 - t0);
}

static uint64_t rng_state = 0x1234567;
static uint64_t rnd() {
  rng_state ^= rng_state << 13;
  rng_state ^= rng_state >> 7;
  rng_state ^= rng_state << 17;
  return rng_state;
}
static uint32_t bitrev(uint32_t x, int n) {
  uint32_t r = 0;
  for (int i = 0; i < n; i++) r |= ((x >> i) & 1u) << (n - 1 - i);
  return r;
}

int main(int argc, char **argv) {
  const uint32_t iters = argc > 1 ? (uint32_t)atoi(argv[1]) : 1000;
  Tables t;
  if (!build_tables(&t)) return 1;
  // LUT1L: index = bit-reversed 12-bit window; entry bits | n << 8 | syms << 16
  std::vector<uint32_t> lut1l(kLut1Size);
  for (uint32_t i = 0; i < (uint32_t)kLut1Size; i++) {
    const uint32_t e = t.lut1[bitrev(i, kLut1Bits)];
    const uint32_t n = (e >> 8) & 0xffu;  // 8 * nsym
    lut1l[i] = e ? ((e & 0xffu) | ((n / 8u) << 8) | (e & 0xffff0000u)) : 0u;
  }
  // LUT2L: [c][sub] with sub LSB-first
  std::vector<uint16_t> lut2l(kLut2Size);
  for (uint32_t c = 0; c < 32; c++)
    for (uint32_t s = 0; s < 32; s++) lut2l[(c << kLut2SubBits) | bitrev(s, kLut2SubBits)] = t.lut2[(c << kLut2SubBits) | s];
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
  std::vector<int> symat;
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
  // LSB-first words: bit j of word k = stream bit 32k + j
  std::vector<uint32_t> words(kStreamWords);
  for (int i = 0; i < kStreamWords; i++) {
    const uint32_t be = (uint32_t)bytes[4 * i] << 24 | bytes[4 * i + 1] << 16 | bytes[4 * i + 2] << 8 | bytes[4 * i + 3];
    words[i] = bitrev(be, 32);
  }
  uint32_t *d_lut1, *d_words, *d_starts, *d_sink, *d_n;
  uint16_t *d_lut2;
  uint8_t *d_out;
  unsigned long long *d_cyc, *d_sym;
  CHECK(hipMalloc(&d_lut1, lut1l.size() * 4));
  CHECK(hipMalloc(&d_lut2, lut2l.size() * 2));
  CHECK(hipMalloc(&d_words, words.size() * 4));
  CHECK(hipMalloc(&d_starts, starts.size() * 4));
  CHECK(hipMalloc(&d_sink, (1 << 20) * 4));
  CHECK(hipMalloc(&d_out, 256 * 64));
  CHECK(hipMalloc(&d_n, 256 * 4));
  CHECK(hipMalloc(&d_cyc, 8));
  CHECK(hipMalloc(&d_sym, 8));
  CHECK(hipMemcpy(d_lut1, lut1l.data(), lut1l.size() * 4, hipMemcpyHostToDevice));
  CHECK(hipMemcpy(d_lut2, lut2l.data(), lut2l.size() * 2, hipMemcpyHostToDevice));
  CHECK(hipMemcpy(d_words, words.data(), words.size() * 4, hipMemcpyHostToDevice));
  CHECK(hipMemcpy(d_starts, starts.data(), starts.size() * 4, hipMemcpyHostToDevice));
  int dev = 0, cus = 0;
  CHECK(hipGetDevice(&dev));
  CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
  for (int v = 0; v < 2; v++) {
    if (v == 0) check_kernel<2><<<1, 256>>>(d_lut1, d_lut2, d_words, d_starts, d_out, d_n);
    else check_kernel<3><<<1, 256>>>(d_lut1, d_lut2, d_words, d_starts, d_out, d_n);
    CHECK(hipDeviceSynchronize());
    std::vector<uint8_t> o(256 * 64);
    std::vector<uint32_t> nn(256);
    CHECK(hipMemcpy(o.data(), d_out, o.size(), hipMemcpyDeviceToHost));
    CHECK(hipMemcpy(nn.data(), d_n, nn.size() * 4, hipMemcpyDeviceToHost));
    int bad = 0;
    long total = 0;
    for (int tid = 0; tid < 256; tid++) {
      total += nn[tid];
      for (uint32_t k = 0; k < nn[tid] && k < 64; k++)
        if (o[tid * 64 + k] != syms[symat[tid] + k]) {
          if (bad < 3) printf("  lane %d byte %u: got %02x want %02x\n", tid, k, o[tid * 64 + k], syms[symat[tid] + k]);
          bad++;
          break;
        }
    }
    printf("lean %d-probe check: %s (%.1f bytes per chain in 8 steps)\n", v + 2, bad ? "MISMATCH" : "ok",
           total / 256.0);
    if (bad) return 1;
  }
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  const int wavess[] = {8, 12, 16};
  for (int v = 3; v >= 0; v--) {
    if (v == 1) continue;
    if (v == 2) {  // the accumulator variant wants 8 * n in [15:8]
      for (auto &x : lut1l) x = x ? ((x & 0xffff00ffu) | ((((x >> 8) & 0xffu) * 8u) << 8)) : 0u;
      CHECK(hipMemcpy(d_lut1, lut1l.data(), lut1l.size() * 4, hipMemcpyHostToDevice));
    }
    for (int waves : wavess) {
      auto launch = [&]() {
        dim3 grid(cus), block(waves * 64);
        const uint32_t ns = (uint32_t)starts.size();
        if (v == 0) ubench<2><<<grid, block>>>(d_lut1, d_lut2, d_words, d_starts, ns, iters, d_sink, d_sym, d_cyc);
        else if (v == 1) ubench<3><<<grid, block>>>(d_lut1, d_lut2, d_words, d_starts, ns, iters, d_sink, d_sym, d_cyc);
        else if (v == 3) ubench<4><<<grid, block>>>(d_lut1, d_lut2, d_words, d_starts, ns, iters, d_sink, d_sym, d_cyc);
        else ubench<12><<<grid, block>>>(d_lut1, d_lut2, d_words, d_starts, ns, iters, d_sink, d_sym, d_cyc);
      };
      launch();
      CHECK(hipDeviceSynchronize());
      CHECK(hipMemset(d_cyc, 0, 8));
      CHECK(hipMemset(d_sym, 0, 8));
      const int reps = 5;
      CHECK(hipEventRecord(e0));
      for (int r = 0; r < reps; r++) launch();
      CHECK(hipEventRecord(e1));
      CHECK(hipEventSynchronize(e1));
      float ms = 0;
      CHECK(hipEventElapsedTime(&ms, e0, e1));
      unsigned long long cyc = 0, symbols = 0;
      CHECK(hipMemcpy(&cyc, d_cyc, 8, hipMemcpyDeviceToHost));
      CHECK(hipMemcpy(&symbols, d_sym, 8, hipMemcpyDeviceToHost));
      const double wave_cyc = (double)cyc / ((double)cus * waves * reps);
      printf("lean %d waves/CU %2d: %7.3f ms  %8.1f G sym/s  cycles/iter/wave %6.1f  sym/iter/lane %.2f\n", v == 2 ? 12 : (v == 3 ? 4 : v + 2),
             waves, ms / reps, (double)symbols / (ms * 1e-3) / 1e9, wave_cyc / iters,
             (double)symbols / ((double)cus * waves * 64 * reps * iters));
    }
  }
  return 0;
}
