// ubench_decode.hip -- inner-loop microbenchmark for the decode probe chain.
//
// Every lane decodes `probes` LUT1 probes of an hdr-like Huffman stream staged
// in LDS (one workgroup per CU, `waves` waves), starting at a symbol boundary
// of its own.  Variants of the loop body are template instances; the result is
// probes per second and shader cycles per wave-probe, so loop shapes and
// occupancies can be compared without the tile framework around them.
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I minhq_amd/csrc \
//     tools/ubench/ubench_decode.hip minhq_amd/csrc/huff_table.cpp -o ubench
//   ./ubench [probes=4000]
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include <vector>

#include "huff_table.h"

#define CHECK(x)                                                                    \
  do {                                                                              \
    hipError_t e_ = (x);                                                            \
    if (e_ != hipSuccess) {                                                         \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      exit(1);                                                                      \
    }                                                                               \
  } while (0)

using namespace mhq;

constexpr int kStreamBytes = 32768;
constexpr uint32_t kLut1Null = 0u;  // (variants 0-4 predate the byte-field LUT1 layout; time 5-8 only)
constexpr int kStreamWords = kStreamBytes / 4;

struct Smem {
  uint32_t lutL[kLut1Size];
  uint32_t lut1[kLut1Size];
  uint16_t lut2[kLut2Size];
  alignas(16) uint32_t in_w[kStreamWords + 8];
  uint32_t out_w[2048];
};

__device__ __forceinline__ uint32_t long_code(const uint16_t *lut2, uint32_t win, uint32_t &sym) {
  const uint32_t nw = ~win;
  const uint32_t c = nw ? (uint32_t)__builtin_clz(nw) : 32u;
  if (c >= (uint32_t)kEosOnes) return 0;
  const uint32_t e2 = lut2[(c << kLut2SubBits) | ((win << (c + 1)) >> (32 - kLut2SubBits))];
  sym = e2 & 0xffu;
  return e2 >> 8;
}

struct BitBuf {
  uint64_t bb;
  uint32_t p, kb, w;
  const uint32_t *in_w;
  __device__ __forceinline__ void init(const uint32_t *words, uint32_t p0) {
    in_w = words;
    p = p0;
    const uint32_t k = p0 >> 5;
    bb = (((uint64_t)in_w[k] << 32) | in_w[k + 1]) << (p0 & 31u);
    kb = (k + 2u) * 32u;
    w = in_w[k + 2u];
  }
  __device__ __forceinline__ void refill() {
    const uint32_t nb = kb - p;
    const bool need = nb <= 32u;
    bb |= (uint64_t)(need ? w : 0u) << ((32u - nb) & 63u);
    kb += need ? 32u : 0u;
    w = in_w[kb >> 5];
  }
  __device__ __forceinline__ uint32_t top32() const { return (uint32_t)(bb >> 32); }
  __device__ __forceinline__ void consume(uint32_t n) {
    bb <<= n;
    p += n;
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
  __device__ __forceinline__ void flush(uint32_t *out_w) {
    atomicOr(&out_w[ow & 2047u], (uint32_t)acc);
    const bool full = ab >= 32u;
    acc = full ? (acc >> 32) : acc;
    ow += full ? 1u : 0u;
    ab &= 31u;
  }
};

// Variant 0: register bit buffer, inline long-code branch per probe, output
// accumulator flushed with ds_or every 2 probes (the production loop).
// Variant 1: as 0 without output (checksum of symbols only).
// Variant 2: as 0, one long-code check per 2 probes (long entries consume 0).
// Variant 3: as 1 but two independent chains per lane.
// Variant 4: window read from LDS per probe (ds_read2 + shift), no output.
template <int V>
__device__ uint32_t run(const Smem &sm, uint32_t *out_w, uint32_t p0, uint32_t p1, uint32_t probes, uint32_t lane) {
  uint32_t chk = 0;
  if constexpr (V == 0 || V == 1 || V == 2) {
    BitBuf in;
    in.init(sm.in_w, p0);
    OutAcc out;
    out.init(lane * 128u);
    for (uint32_t i = 0; i < probes; i += 2) {
      if constexpr (V == 2) {
        uint32_t e = sm.lut1[in.top32() >> (32 - kLut1Bits)];
        out.put(e & 0xffffu, (e >> 26) & 31u);
        in.consume((e >> 16) & 31u);
        e = sm.lut1[in.top32() >> (32 - kLut1Bits)];
        if ((int32_t)e >= 0) {
          in.refill();
          uint32_t sym = 0;
          const uint32_t L = long_code(sm.lut2, in.top32(), sym);
          out.put(sym, 8u);
          in.consume(L);
          e = kLut1Null;
        }
        out.put(e & 0xffffu, (e >> 26) & 31u);
        in.consume((e >> 16) & 31u);
      } else {
#pragma unroll
        for (int u = 0; u < 2; u++) {
          uint32_t e = sm.lut1[in.top32() >> (32 - kLut1Bits)];
          if ((int32_t)e >= 0) {
            in.refill();
            uint32_t sym = 0;
            const uint32_t L = long_code(sm.lut2, in.top32(), sym);
            out.put(sym, 8u);
            in.consume(L);
            in.refill();
            e = kLut1Null;
          }
          if constexpr (V == 1) {
            chk += e;
            in.consume((e >> 16) & 31u);
          } else {
            out.put(e & 0xffffu, (e >> 26) & 31u);
            in.consume((e >> 16) & 31u);
          }
        }
      }
      in.refill();
      if constexpr (V != 1) out.flush(out_w);
    }
    chk += in.p + out.ow;
  } else if constexpr (V == 3) {
    BitBuf a, b;
    a.init(sm.in_w, p0);
    b.init(sm.in_w, p1);
    for (uint32_t i = 0; i < probes; i += 2) {
#pragma unroll
      for (int u = 0; u < 2; u++) {
        uint32_t ea = sm.lut1[a.top32() >> (32 - kLut1Bits)];
        uint32_t eb = sm.lut1[b.top32() >> (32 - kLut1Bits)];
        if ((int32_t)ea >= 0) {
          a.refill();
          uint32_t sym = 0;
          a.consume(long_code(sm.lut2, a.top32(), sym));
          a.refill();
          ea = kLut1Null | sym;
        }
        if ((int32_t)eb >= 0) {
          b.refill();
          uint32_t sym = 0;
          b.consume(long_code(sm.lut2, b.top32(), sym));
          b.refill();
          eb = kLut1Null | sym;
        }
        chk += ea + eb;
        a.consume((ea >> 16) & 31u);
        b.consume((eb >> 16) & 31u);
      }
      a.refill();
      b.refill();
    }
    chk += a.p + b.p;
  } else if constexpr (V == 5 || V == 6 || V == 7 || V == 9 || V == 10) {
    // lean loop: SDWA-friendly entries (byte0 tot, byte1 nsym, byte2 sym0, byte3 sym1; 0 = long),
    // one long check per 2 probes; V5 writes symbols with ds_write_b16 (unaligned), V6 with two
    // ds_write_b8, V7 through the 64-bit accumulator + ds_or.
    const uint32_t *lutL = sm.lutL;
    uint8_t *ob = (uint8_t *)out_w;
    uint32_t optr = lane * 128u + (p0 & 3u);
    BitBuf in;
    in.init(sm.in_w, p0);
    uint32_t nb = 64u - (p0 & 31u);
    OutAcc out;
    out.init(optr);
    for (uint32_t i = 0; i < probes; i += 2) {
#pragma unroll
      for (int u = 0; u < 2; u++) {
        uint32_t e = lutL[in.top32() >> (32 - kLut1Bits)];
        if (u == 1 && e == 0) {
          in.p = in.kb - nb;
          in.refill();
          nb = in.kb - in.p;
          uint32_t sym = 0;
          const uint32_t L = long_code(sm.lut2, in.top32(), sym);
          e = L | (8u << 8) | (sym << 16);
        }
        in.bb <<= (e & 63u);
        nb -= e & 0xffu;
        if constexpr (V == 5) {
          *(uint16_t *)(ob + (optr & 8191u)) = (uint16_t)(e >> 16);
          optr += ((e >> 8) & 0xffu) >> 3;
        } else if constexpr (V == 6) {
          ob[optr & 8191u] = (uint8_t)(e >> 16);
          ob[(optr & 8191u) + 1] = (uint8_t)(e >> 24);
          optr += ((e >> 8) & 0xffu) >> 3;
        } else {
          out.put(e >> 16, (e >> 8) & 0xffu);
        }
      }
      if constexpr (V == 10) {  // timing bound: no flush store, the accumulator drains in registers
        chk ^= (uint32_t)out.acc;
        out.acc >>= out.ab & 32u;
        out.ab &= 31u;
      }
      {
        const bool need = nb <= 32u;
        in.bb |= (uint64_t)(need ? in.w : 0u) << ((32u - nb) & 63u);
        in.kb += need ? 32u : 0u;
        nb += need ? 32u : 0u;
        if constexpr (V == 9) {
          in.w = in.kb * 0x9e3779b9u;  // timing bound: no refill read (wrong bits)
        } else {
          in.w = in.in_w[in.kb >> 5];
        }
      }
      if constexpr (V == 7 || V == 9) out.flush(out_w);
    }
    chk += nb + optr + out.ow;
  } else if constexpr (V == 11 || V == 12) {
    // lean acc+ds_or loop; refill variants: V11 reads the look-ahead word only
    // when a refill used it; V12 keeps 64 pending bits and reads two words
    // (ds_read_b64) every other refill.
    const uint32_t *lutL = sm.lutL;
    const uint32_t *w = sm.in_w;
    const uint32_t k0 = p0 >> 5;
    uint64_t bb = (((uint64_t)w[k0] << 32) | w[k0 + 1]) << (p0 & 31u);
    uint32_t nb = 64u - (p0 & 31u);
    uint32_t kw = k0 + 2u, lw = w[kw];  // V11
    uint64_t pw = 0;                     // V12
    uint32_t pn = 0;
    if constexpr (V == 12) {
      if (kw & 1u) {
        pw = (uint64_t)w[kw] << 32;
        pn = 32u;
        kw += 1u;
      } else {
        const uint2 v = *(const uint2 *)(w + kw);
        pw = ((uint64_t)v.x << 32) | v.y;
        pn = 64u;
        kw += 2u;
      }
    }
    OutAcc out;
    out.init(lane * 128u + (p0 & 3u));
    auto refill = [&]() {
      const bool need = nb <= 32u;
      if constexpr (V == 11) {
        bb |= (uint64_t)(need ? lw : 0u) << ((32u - nb) & 63u);
        nb += need ? 32u : 0u;
        if (need) {
          kw += 1u;
          lw = w[kw];
        }
      } else {
        bb |= (uint64_t)(need ? (uint32_t)(pw >> 32) : 0u) << ((32u - nb) & 63u);
        nb += need ? 32u : 0u;
        pw = need ? pw << 32 : pw;
        pn -= need ? 32u : 0u;
        if (pn == 0u) {
          const uint2 v = *(const uint2 *)(w + kw);
          pw = ((uint64_t)v.x << 32) | v.y;
          pn = 64u;
          kw += 2u;
        }
      }
    };
    for (uint32_t i = 0; i < probes; i += 2) {
#pragma unroll
      for (int u = 0; u < 2; u++) {
        uint32_t e = lutL[(uint32_t)(bb >> 32) >> (32 - kLut1Bits)];
        if (u == 1 && e == 0) {
          refill();
          uint32_t sym = 0;
          const uint32_t L = long_code(sm.lut2, (uint32_t)(bb >> 32), sym);
          e = L | (8u << 8) | (sym << 16);
        }
        bb <<= (e & 63u);
        nb -= e & 0xffu;
        out.put(e >> 16, (e >> 8) & 0xffu);
      }
      refill();
      out.flush(out_w);
    }
    chk += nb + out.ow + (uint32_t)bb;
  } else if constexpr (V == 8) {
    // two independent lean chains per lane (acc + ds_or), interleaved probe by probe
    const uint32_t *lutL = sm.lutL;
    BitBuf in[2];
    uint32_t nb[2];
    OutAcc out[2];
    const uint32_t ps[2] = {p0, p1};
#pragma unroll
    for (int c = 0; c < 2; c++) {
      in[c].init(sm.in_w, ps[c]);
      nb[c] = 64u - (ps[c] & 31u);
      out[c].init(lane * 128u + c * 64u + (ps[c] & 3u));
    }
    for (uint32_t i = 0; i < probes; i += 2) {
#pragma unroll
      for (int u = 0; u < 2; u++) {
#pragma unroll
        for (int c = 0; c < 2; c++) {
          uint32_t e = lutL[in[c].top32() >> (32 - kLut1Bits)];
          if (u == 1 && e == 0) {
            in[c].p = in[c].kb - nb[c];
            in[c].refill();
            nb[c] = in[c].kb - in[c].p;
            uint32_t sym = 0;
            const uint32_t L = long_code(sm.lut2, in[c].top32(), sym);
            e = L | (8u << 8) | (sym << 16);
          }
          in[c].bb <<= (e & 63u);
          nb[c] -= e & 0xffu;
          out[c].put(e >> 16, (e >> 8) & 0xffu);
        }
      }
#pragma unroll
      for (int c = 0; c < 2; c++) {
        const bool need = nb[c] <= 32u;
        in[c].bb |= (uint64_t)(need ? in[c].w : 0u) << ((32u - nb[c]) & 63u);
        in[c].kb += need ? 32u : 0u;
        nb[c] += need ? 32u : 0u;
        in[c].w = in[c].in_w[in[c].kb >> 5];
        out[c].flush(out_w);
      }
    }
    chk += nb[0] + nb[1] + out[0].ow + out[1].ow;
  } else {
    uint32_t p = p0;
    for (uint32_t i = 0; i < probes; i++) {
      const uint32_t k = p >> 5, sh = p & 31u;
      const uint64_t ww = ((uint64_t)sm.in_w[k] << 32) | sm.in_w[k + 1];
      const uint32_t win = (uint32_t)((ww << sh) >> 32);
      uint32_t e = sm.lut1[win >> (32 - kLut1Bits)];
      uint32_t tot = (e >> 16) & 31u;
      if ((int32_t)e >= 0) {
        uint32_t sym = 0;
        tot = long_code(sm.lut2, win, sym);
        e = sym;
      }
      chk += e;
      p += tot;
    }
    chk += p;
  }
  return chk;
}

template <int V>
__global__ __launch_bounds__(1024) void ubench(const uint32_t *g_lutL, const uint32_t *g_lut1, const uint16_t *g_lut2, const uint32_t *g_words,
                                               const uint32_t *starts, uint32_t nstarts, uint32_t probes,
                                               uint32_t *sink, unsigned long long *cycles) {
  __shared__ Smem sm;
  const uint32_t tid = threadIdx.x, lane = tid & 63u;
  for (uint32_t i = tid; i < kLut1Size; i += blockDim.x) sm.lut1[i] = g_lut1[i];
  for (uint32_t i = tid; i < kLut1Size; i += blockDim.x) sm.lutL[i] = g_lutL[i];
  for (uint32_t i = tid; i < kLut2Size; i += blockDim.x) sm.lut2[i] = g_lut2[i];
  for (uint32_t i = tid; i < kStreamWords + 8; i += blockDim.x) sm.in_w[i] = i < kStreamWords ? g_words[i] : 0u;
  for (uint32_t i = tid; i < 2048; i += blockDim.x) sm.out_w[i] = 0;
  if (blockIdx.x == 0 && tid < 64) sink[(1 << 20) - 64 * 16 - 64 + tid] = starts[((blockIdx.x * blockDim.x + tid) * 7919u) % nstarts];
  __syncthreads();
  const uint32_t g = blockIdx.x * blockDim.x + tid;
  const uint32_t p0 = starts[(g * 7919u) % nstarts], p1 = starts[(g * 104729u + 17u) % nstarts];
  const unsigned long long t0 = clock64();
  const uint32_t chk = run<V>(sm, sm.out_w, p0, p1, probes, tid & 63u);
  const unsigned long long t1 = clock64();
  __syncthreads();
  sink[g] = chk + sm.out_w[tid & 2047u];
  if (blockIdx.x == 0 && tid < 64) {  // lane outputs of block 0 wave 0 for the correctness check
    const uint8_t *ob = (const uint8_t *)sm.out_w + tid * 128u + (p0 & 3u);
    for (int i = 0; i < 64; i++) ((uint8_t *)(sink + (1 << 20) - 64 * 64))[tid * 64 + i] = ob[i];
  }
  if (lane == 0) atomicAdd(cycles, t1 - t0);
}

static uint64_t rng_state = 0x1234567;
static uint64_t rnd() {
  rng_state ^= rng_state << 13;
  rng_state ^= rng_state >> 7;
  rng_state ^= rng_state << 17;
  return rng_state;
}

int main(int argc, char **argv) {
  const uint32_t probes = argc > 1 ? (uint32_t)atoi(argv[1]) : 4000;
  Tables t;
  if (!build_tables(&t)) return 1;
  // hdr-like text: netbsd.qif byte histogram (minhq_amd/workloads.py NETBSD_HIST), add-one smoothed
  static const int hist[95] = {163, 0, 0, 0, 0, 0, 0, 0, 18, 18, 36, 1, 41, 162, 181, 165, 183, 74, 19, 0, 36, 72, 36, 0,
                               37, 1, 107, 75, 0, 22, 0, 0, 0, 0, 2, 1, 1, 18, 19, 36, 0, 0, 0, 0, 0, 19, 19, 0,
                               2, 0, 0, 21, 37, 19, 0, 36, 0, 1, 0, 0, 0, 0, 0, 4, 0, 331, 45, 343, 115, 540, 57, 180,
                               163, 198, 4, 41, 135, 78, 326, 301, 187, 22, 211, 130, 324, 61, 38, 125, 41, 22, 36,
                               0, 0, 0, 0};
  std::vector<double> cdf(95);
  double tot = 0;
  for (int i = 0; i < 95; i++) tot += hist[i] + 1;
  double acc = 0;
  for (int i = 0; i < 95; i++) cdf[i] = (acc += (hist[i] + 1) / tot);
  std::vector<uint32_t> words(kStreamWords, 0);
  std::vector<uint32_t> starts;
  uint64_t bit = 0;
  const uint64_t limit = (uint64_t)kStreamBytes * 8 - 64;
  while (true) {
    const double u = (rnd() >> 11) * (1.0 / 9007199254740992.0);
    int s = 0;
    while (s < 94 && cdf[s] < u) s++;
    const int sym = 0x20 + s;
    const int L = t.len[sym];
    if (bit + L > limit) break;
    if (bit < (uint64_t)kStreamBytes * 8 / 2) starts.push_back((uint32_t)bit);
    for (int b = L - 1; b >= 0; b--, bit++)
      if ((t.code[sym] >> b) & 1u) words[bit >> 5] |= 1u << (31 - (bit & 31));
  }
  printf("stream: %llu bits, %zu start positions, probes/lane %u\n", (unsigned long long)bit, starts.size(), probes);
  std::vector<uint32_t> lutL(kLut1Size);
  for (int i = 0; i < kLut1Size; i++) {
    const uint32_t e = t.lut1[i];
    lutL[i] = e;  // the production layout: tot | 8*nsym << 8 | sym0 << 16 | sym1 << 24, 0 = long
  }
  uint32_t *d_lutL;
  CHECK(hipMalloc(&d_lutL, lutL.size() * 4));
  CHECK(hipMemcpy(d_lutL, lutL.data(), lutL.size() * 4, hipMemcpyHostToDevice));
  uint32_t *d_lut1, *d_words, *d_starts, *d_sink;
  uint16_t *d_lut2;
  unsigned long long *d_cyc;
  CHECK(hipMalloc(&d_lut1, sizeof(t.lut1)));
  CHECK(hipMalloc(&d_lut2, sizeof(t.lut2)));
  CHECK(hipMalloc(&d_words, words.size() * 4));
  CHECK(hipMalloc(&d_starts, starts.size() * 4));
  CHECK(hipMalloc(&d_sink, 1024 * 1024 * 4));
  CHECK(hipMalloc(&d_cyc, 8));
  CHECK(hipMemcpy(d_lut1, t.lut1, sizeof(t.lut1), hipMemcpyHostToDevice));
  CHECK(hipMemcpy(d_lut2, t.lut2, sizeof(t.lut2), hipMemcpyHostToDevice));
  CHECK(hipMemcpy(d_words, words.data(), words.size() * 4, hipMemcpyHostToDevice));
  CHECK(hipMemcpy(d_starts, starts.data(), starts.size() * 4, hipMemcpyHostToDevice));
  int dev = 0, cus = 0;
  CHECK(hipGetDevice(&dev));
  CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  const char *names[] = {"regbuf+ds_or", "regbuf,no-out", "regbuf+ds_or,1chk", "regbuf,2chains,no-out", "window,no-out",
                         "lean,ds_write_b16", "lean,2x ds_write_b8", "lean,acc+ds_or", "lean,acc+ds_or,2chains", "lean,no refill read", "lean,no flush", "lean,refill read when used", "lean,refill b64"};
  // host decode for the correctness check: (len, code) -> symbol
  auto host_decode = [&](uint64_t p, int nsym, std::vector<uint8_t> &outv) {
    outv.clear();
    while ((int)outv.size() < nsym) {
      uint32_t v = 0;
      int L = 0, found = -1;
      while (found < 0 && L < 30) {
        v = (v << 1) | ((words[(p + L) >> 5] >> (31 - ((p + L) & 31))) & 1u);
        L++;
        for (int sidx = 0; sidx < 256; sidx++)
          if (t.len[sidx] == L && t.code[sidx] == v) { found = sidx; break; }
      }
      if (found < 0) break;
      outv.push_back((uint8_t)found);
      p += L;
    }
  };
  auto launch = [&](int v, int waves) {
    dim3 grid(cus), block(waves * 64);
    switch (v) {
      case 0: ubench<0><<<grid, block>>>(d_lutL, d_lut1, d_lut2, d_words, d_starts, starts.size(), probes, d_sink, d_cyc); break;
      case 1: ubench<1><<<grid, block>>>(d_lutL, d_lut1, d_lut2, d_words, d_starts, starts.size(), probes, d_sink, d_cyc); break;
      case 2: ubench<2><<<grid, block>>>(d_lutL, d_lut1, d_lut2, d_words, d_starts, starts.size(), probes, d_sink, d_cyc); break;
      case 3: ubench<3><<<grid, block>>>(d_lutL, d_lut1, d_lut2, d_words, d_starts, starts.size(), probes, d_sink, d_cyc); break;
      case 4: ubench<4><<<grid, block>>>(d_lutL, d_lut1, d_lut2, d_words, d_starts, starts.size(), probes, d_sink, d_cyc); break;
      case 5: ubench<5><<<grid, block>>>(d_lutL, d_lut1, d_lut2, d_words, d_starts, starts.size(), probes, d_sink, d_cyc); break;
      case 6: ubench<6><<<grid, block>>>(d_lutL, d_lut1, d_lut2, d_words, d_starts, starts.size(), probes, d_sink, d_cyc); break;
      case 7: ubench<7><<<grid, block>>>(d_lutL, d_lut1, d_lut2, d_words, d_starts, starts.size(), probes, d_sink, d_cyc); break;
      case 8: ubench<8><<<grid, block>>>(d_lutL, d_lut1, d_lut2, d_words, d_starts, starts.size(), probes, d_sink, d_cyc); break;
      case 9: ubench<9><<<grid, block>>>(d_lutL, d_lut1, d_lut2, d_words, d_starts, starts.size(), probes, d_sink, d_cyc); break;
      case 10: ubench<10><<<grid, block>>>(d_lutL, d_lut1, d_lut2, d_words, d_starts, starts.size(), probes, d_sink, d_cyc); break;
      case 11: ubench<11><<<grid, block>>>(d_lutL, d_lut1, d_lut2, d_words, d_starts, starts.size(), probes, d_sink, d_cyc); break;
      case 12: ubench<12><<<grid, block>>>(d_lutL, d_lut1, d_lut2, d_words, d_starts, starts.size(), probes, d_sink, d_cyc); break;
    }
  };
  // correctness of the lean variants: one wave, 24 probes per lane, compare 40 output bytes
  for (int v = 5; v < 13; v++) {
    if (v > 7 && v < 11) continue;
    const uint32_t save = probes;
    (void)save;
    dim3 grid1(1), block1(64);
    const uint32_t pr = 40;
    switch (v) {
      case 5: ubench<5><<<grid1, block1>>>(d_lutL, d_lut1, d_lut2, d_words, d_starts, starts.size(), pr, d_sink, d_cyc); break;
      case 6: ubench<6><<<grid1, block1>>>(d_lutL, d_lut1, d_lut2, d_words, d_starts, starts.size(), pr, d_sink, d_cyc); break;
      case 7: ubench<7><<<grid1, block1>>>(d_lutL, d_lut1, d_lut2, d_words, d_starts, starts.size(), pr, d_sink, d_cyc); break;
      case 11: ubench<11><<<grid1, block1>>>(d_lutL, d_lut1, d_lut2, d_words, d_starts, starts.size(), pr, d_sink, d_cyc); break;
      case 12: ubench<12><<<grid1, block1>>>(d_lutL, d_lut1, d_lut2, d_words, d_starts, starts.size(), pr, d_sink, d_cyc); break;
    }
    CHECK(hipDeviceSynchronize());
    std::vector<uint32_t> sink(1 << 20);
    CHECK(hipMemcpy(sink.data(), d_sink, sink.size() * 4, hipMemcpyDeviceToHost));
    const uint8_t *got = (const uint8_t *)(sink.data() + (1 << 20) - 64 * 64);
    int bad = 0;
    std::vector<uint8_t> ref;
    for (int l = 0; l < 64; l++) {
      const uint32_t p0 = sink[(1 << 20) - 64 * 16 - 64 + l];
      host_decode(p0, 20, ref);
      for (int i = 0; i < 20; i++) bad += got[l * 64 + i] != ref[i];
    }
    printf("check %-22s: %s (%d byte mismatches in 64 lanes x 20 bytes)\n", names[v], bad ? "MISMATCH" : "ok", bad);
  }
  const int only_v = argc > 2 ? atoi(argv[2]) : -1, only_w = argc > 3 ? atoi(argv[3]) : 0;
  for (int v = 7; v < 13; v++) {
    if (only_v >= 0 && v != only_v) continue;
    for (int waves : {12, 16}) {
      if (only_w && waves != only_w) continue;
      launch(v, waves);
      CHECK(hipDeviceSynchronize());
      CHECK(hipMemset(d_cyc, 0, 8));
      CHECK(hipEventRecord(e0));
      const int reps = 5;
      for (int r = 0; r < reps; r++) launch(v, waves);
      CHECK(hipEventRecord(e1));
      CHECK(hipEventSynchronize(e1));
      float ms = 0;
      CHECK(hipEventElapsedTime(&ms, e0, e1));
      unsigned long long cyc = 0;
      CHECK(hipMemcpy(&cyc, d_cyc, 8, hipMemcpyDeviceToHost));
      const double chains = (v == 3 || v == 8 ? 2.0 : 1.0);
      const double lane_probes = (double)cus * waves * 64 * probes * chains * reps;
      const double wave_cyc = (double)cyc / ((double)cus * waves * reps);
      printf("%-24s waves/CU %2d: %7.3f ms  %8.1f Gprobe/s  wave-cycles/probe-step %6.1f  SIMD-cycles/wave-probe %5.1f\n",
             names[v], waves, ms / reps, lane_probes / (ms * 1e-3) / 1e9, wave_cyc / probes,
             wave_cyc / probes / (waves / 4.0));
    }
  }
  return 0;
}
