// ubench_step.hip -- occupancy sweep of the decode fast step (the loop body of
// huff_decode_wg.hip's decoders), to tell latency-bound from throughput-bound.
//
// Every lane decodes `steps` fast steps (two LUT1 probes each, bit buffer
// refilled from LDS words read byte-swapped, output OR-ed into LDS) of an
// hdr-like Huffman stream staged in LDS, starting at a symbol boundary of its
// own.  Workgroups of W waves, B workgroups per CU: W*B waves per CU.  Prints
// wall time, chip-wide lane-steps per second and cycles per step per wave.
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I minhq_amd/csrc \
//     tools/ubench/ubench_step.hip minhq_amd/csrc/huff_table.cpp -o tools/ubench/ubench_step
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include <vector>

#include "huff_table.h"

#define CHECK(x)                                                                             \
  do {                                                                                       \
    hipError_t e_ = (x);                                                                     \
    if (e_ != hipSuccess) {                                                                  \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_));      \
      exit(1);                                                                               \
    }                                                                                        \
  } while (0)

using namespace mhq;

constexpr int kStreamBytes = 32768;
constexpr int kStreamWords = kStreamBytes / 4;
constexpr int kOutWords = 4096;

struct Smem {
  uint32_t lut1[kLut1Size];
  uint16_t lut2[kLut2Size];
  alignas(16) uint32_t in_w[kStreamWords + 8];  // raw (little-endian) words, as LDS-DMA leaves them
  uint32_t out_w[kOutWords];
};

__device__ __forceinline__ uint32_t sw(const uint32_t *w, uint32_t k) { return __builtin_bswap32(w[k]); }

template <int kVariant>
__device__ uint32_t run(const Smem &sm, uint32_t *out_w, uint32_t p0, uint32_t steps, uint32_t lane) {
  // bit buffer
  uint32_t p = p0;
  const uint32_t k0 = p0 >> 5;
  uint64_t bb = (((uint64_t)sw(sm.in_w, k0) << 32) | sw(sm.in_w, k0 + 1)) << (p0 & 31u);
  uint32_t kb = (k0 + 2u) * 32u, w = sw(sm.in_w, k0 + 2u);
  // output accumulator: lane-private region
  uint64_t acc = 0;
  uint32_t ow = lane * 64u, ab = 0;
  uint32_t chk = 0;
  for (uint32_t i = 0; i < steps; i++) {
    uint32_t e = sm.lut1[(uint32_t)(bb >> 32) >> (32 - kLut1Bits)];
    acc |= (uint64_t)(e >> 16) << ab;
    ab += (e >> 8) & 0xffu;
    bb <<= (e & 63u);
    p += e & 0xffu;
    e = sm.lut1[(uint32_t)(bb >> 32) >> (32 - kLut1Bits)];
    if (e == 0) e = (8u << 8) | 13u;  // a long code: take 13 bits, no symbol (timing only)
    acc |= (uint64_t)(e >> 16) << ab;
    ab += (e >> 8) & 0xffu;
    bb <<= (e & 63u);
    p += e & 0xffu;
    // refill
    const uint32_t nb = kb - p;
    const bool need = nb <= 32u;
    bb |= (uint64_t)(need ? w : 0u) << ((32u - nb) & 63u);
    kb += need ? 32u : 0u;
    w = sw(sm.in_w, (kb >> 5) & (kStreamWords - 1u));
    if (kVariant == 0) atomicOr(&out_w[ow & (kOutWords - 1u)], (uint32_t)acc);
    chk += (uint32_t)acc;
    acc >>= ab & 32u;
    ow += ab >> 5;
    ab &= 31u;
    if (p > (uint32_t)kStreamBytes * 8u - 256u) {  // wrap
      p = p0;
      const uint32_t k = p0 >> 5;
      bb = (((uint64_t)sw(sm.in_w, k) << 32) | sw(sm.in_w, k + 1)) << (p0 & 31u);
      kb = (k + 2u) * 32u;
      w = sw(sm.in_w, k + 2u);
    }
  }
  return chk + p;
}

template <int kVariant, int kMinWavesPerEU>
__global__ __launch_bounds__(1024, kMinWavesPerEU) void ubench(const uint32_t *g_lut1, const uint16_t *g_lut2,
                                                               const uint32_t *g_words, const uint32_t *starts,
                                                               uint32_t nstarts, uint32_t steps, uint32_t *sink,
                                                               unsigned long long *cycles) {
  __shared__ Smem sm;
  const uint32_t tid = threadIdx.x;
  for (uint32_t i = tid; i < kLut1Size; i += blockDim.x) sm.lut1[i] = g_lut1[i];
  for (uint32_t i = tid; i < kLut2Size; i += blockDim.x) sm.lut2[i] = g_lut2[i];
  for (uint32_t i = tid; i < kStreamWords + 8; i += blockDim.x) sm.in_w[i] = i < kStreamWords ? g_words[i] : 0u;
  for (uint32_t i = tid; i < kOutWords; i += blockDim.x) sm.out_w[i] = 0;
  __syncthreads();
  const uint32_t g = blockIdx.x * blockDim.x + tid;
  const uint32_t p0 = starts[(g * 7919u) % nstarts];
  const unsigned long long t0 = clock64();
  const uint32_t chk = run<kVariant>(sm, sm.out_w, p0, steps, tid & 63u);
  const unsigned long long t1 = clock64();
  __syncthreads();
  sink[g & ((1u << 20) - 1u)] = chk + sm.out_w[tid & (kOutWords - 1u)];
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
  const uint32_t steps = argc > 1 ? (uint32_t)atoi(argv[1]) : 2000;
  Tables t;
  if (!build_tables(&t)) return 1;
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
      if ((t.code[sym] >> b) & 1u) bytes[bit >> 3] |= (uint8_t)(0x80u >> (bit & 7));
  }
  std::vector<uint32_t> words(kStreamWords);
  for (int i = 0; i < kStreamWords; i++)
    words[i] = bytes[4 * i] | bytes[4 * i + 1] << 8 | bytes[4 * i + 2] << 16 | (uint32_t)bytes[4 * i + 3] << 24;
  uint32_t *d_lut1, *d_words, *d_starts, *d_sink;
  uint16_t *d_lut2;
  unsigned long long *d_cyc;
  CHECK(hipMalloc(&d_lut1, sizeof(t.lut1)));
  CHECK(hipMalloc(&d_lut2, sizeof(t.lut2)));
  CHECK(hipMalloc(&d_words, words.size() * 4));
  CHECK(hipMalloc(&d_starts, starts.size() * 4));
  CHECK(hipMalloc(&d_sink, (1 << 20) * 4));
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
  struct Cfg {
    int waves, blocks, variant;
  };
  const Cfg cfgs[] = {{4, 1, 0}, {8, 1, 0}, {12, 1, 0}, {16, 1, 0}, {12, 2, 0}, {16, 2, 0},
                      {12, 1, 1}, {16, 1, 1}, {16, 2, 1}};
  for (const Cfg &c : cfgs) {
    auto launch = [&]() {
      dim3 grid(cus * c.blocks), block(c.waves * 64);
      if (c.variant == 0) {
        if (c.blocks == 1)
          ubench<0, 1><<<grid, block>>>(d_lut1, d_lut2, d_words, d_starts, starts.size(), steps, d_sink, d_cyc);
        else
          ubench<0, 2><<<grid, block>>>(d_lut1, d_lut2, d_words, d_starts, starts.size(), steps, d_sink, d_cyc);
      } else {
        if (c.blocks == 1)
          ubench<1, 1><<<grid, block>>>(d_lut1, d_lut2, d_words, d_starts, starts.size(), steps, d_sink, d_cyc);
        else
          ubench<1, 2><<<grid, block>>>(d_lut1, d_lut2, d_words, d_starts, starts.size(), steps, d_sink, d_cyc);
      }
    };
    launch();
    CHECK(hipDeviceSynchronize());
    CHECK(hipMemset(d_cyc, 0, 8));
    const int reps = 5;
    CHECK(hipEventRecord(e0));
    for (int r = 0; r < reps; r++) launch();
    CHECK(hipEventRecord(e1));
    CHECK(hipEventSynchronize(e1));
    float ms = 0;
    CHECK(hipEventElapsedTime(&ms, e0, e1));
    unsigned long long cyc = 0;
    CHECK(hipMemcpy(&cyc, d_cyc, 8, hipMemcpyDeviceToHost));
    const double wpc = c.waves * c.blocks;
    const double lane_steps = (double)cus * wpc * 64 * steps * reps;
    const double wave_cyc = (double)cyc / ((double)cus * wpc * reps);
    printf("%s waves/CU %2.0f (%2d x %d): %7.3f ms  %8.1f G lane-steps/s  cycles/step/wave %6.1f\n",
           c.variant == 0 ? "ds_or " : "no-out", wpc, c.waves, c.blocks, ms / reps, lane_steps / (ms * 1e-3) / 1e9,
           wave_cyc / steps);
  }
  return 0;
}
