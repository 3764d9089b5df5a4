// Host-memory decode rate before and after a device free, without torch
// (tools/hostpath.py's devalloc step restated in C++: is the slowdown the
// HIP runtime's or torch's?).
//
//   hipcc -O2 -o build/hostpath_c tools/hostpath_c.cpp -Iinclude \
//       -Lminhq_amd -lmhq_huff -Wl,-rpath,'$ORIGIN/../minhq_amd'
//   build/hostpath_c [steps...]      steps: free, smallfree, pageable, sleep, hostfree,
//                                    zerocopy, zeroenc
//
// Prints one line per measurement: GiB/s of plaintext (config-2 shape:
// 2^20 literals of 8..64 header-alphabet bytes).
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <unistd.h>

#include <chrono>
#include <random>
#include <vector>

#include "mhq_huff.h"

#define CK(x)                                                              \
  do {                                                                     \
    int rc_ = (x);                                                         \
    if (rc_) {                                                             \
      fprintf(stderr, "%s failed: %d %s\n", #x, rc_, mhq_strerror(rc_)); \
      exit(1);                                                             \
    }                                                                      \
  } while (0)

template <class T>
T *pinned(size_t n) {
  void *p = nullptr;
  if (hipHostMalloc(&p, n * sizeof(T) + 16, hipHostMallocDefault) != hipSuccess) exit(2);
  return (T *)p;
}

int main(int argc, char **argv) {
  const uint64_t n = 1u << 20;
  std::mt19937_64 rng(7);
  const char *alpha = "abcdefghijklmnopqrstuvwxyz0123456789-_/.=:;, ";
  std::vector<uint64_t> off(n + 1);
  off[0] = 0;
  for (uint64_t i = 0; i < n; i++) off[i + 1] = off[i] + 8 + rng() % 57;
  const uint64_t bytes = off[n];
  uint8_t *data = pinned<uint8_t>(bytes);
  for (uint64_t i = 0; i < bytes; i++) data[i] = (uint8_t)alpha[rng() % strlen(alpha)];
  uint64_t *in_off = pinned<uint64_t>(n + 1);
  memcpy(in_off, off.data(), (n + 1) * 8);
  mhq_ctx *ctx = nullptr;
  CK(mhq_open(&ctx, 1));
  uint32_t *enc_len = pinned<uint32_t>(n);
  CK(mhq_huff_encode_len(ctx, data, in_off, n, enc_len));
  uint64_t *eoff = pinned<uint64_t>(n + 1), *cap = pinned<uint64_t>(n + 1);
  eoff[0] = cap[0] = 0;
  for (uint64_t i = 0; i < n; i++) {
    eoff[i + 1] = eoff[i] + enc_len[i];
    cap[i + 1] = cap[i] + (uint64_t)enc_len[i] * 8 / 5;
  }
  uint8_t *enc = pinned<uint8_t>(eoff[n]);
  CK(mhq_huff_encode(ctx, data, in_off, n, enc, eoff));
  uint8_t *out = pinned<uint8_t>(cap[n]), *st = pinned<uint8_t>(n);
  uint32_t *olen = pinned<uint32_t>(n);
  auto dec = [&](uint8_t *o, uint32_t *l, uint8_t *s) {
    const auto t0 = std::chrono::steady_clock::now();
    CK(mhq_huff_decode(ctx, enc, eoff, n, o, cap, l, s));
    const double dt = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    for (uint64_t i = 0; i < n; i += 4097)
      if (l[i] != off[i + 1] - off[i] || s[i]) {
        fprintf(stderr, "decode mismatch at %llu\n", (unsigned long long)i);
        exit(3);
      }
    return bytes / dt / (1 << 30);
  };
  printf("first:");
  for (int k = 0; k < 4; k++) printf(" %.2f", dec(out, olen, st));
  printf("\n");
  for (int a = 1; a < argc; a++) {
    const char *step = argv[a];
    if (!strcmp(step, "free")) {
      void *p = nullptr;
      if (hipMalloc(&p, (size_t)8 << 30) != hipSuccess) exit(4);
      (void)hipMemset(p, 1, (size_t)8 << 30);
      (void)hipDeviceSynchronize();
      (void)hipFree(p);
    } else if (!strcmp(step, "smallfree")) {
      void *p = nullptr;
      if (hipMalloc(&p, (size_t)64 << 20) != hipSuccess) exit(4);
      (void)hipDeviceSynchronize();
      (void)hipFree(p);
    } else if (!strcmp(step, "pageable")) {
      std::vector<uint8_t> o(cap[n] + 16), s(n);
      std::vector<uint32_t> l(n);
      printf("pageable_rate %.2f\n", dec(o.data(), l.data(), s.data()));
    } else if (!strcmp(step, "hostfree")) {  // a pinned buffer allocated and freed
      uint8_t *p = pinned<uint8_t>((size_t)256 << 20);
      memset(p, 1, (size_t)256 << 20);
      (void)hipHostFree(p);
    } else if (!strcmp(step, "zerocopy") || !strcmp(step, "zeroenc")) {
      // the device-resident entry points on the pinned host buffers: the
      // kernels read and write host memory over PCIe, no staging copies
      const bool e = step[4] == 'e';
      uint8_t *enc2 = e ? pinned<uint8_t>(eoff[n]) : nullptr;
      printf("%s:", step);
      for (int k = 0; k < 4; k++) {
        const auto t0 = std::chrono::steady_clock::now();
        if (e)
          CK(mhq_huff_encode_dev(ctx, 0, data, in_off, n, enc2, eoff, nullptr));
        else
          CK(mhq_huff_decode_dev(ctx, 0, enc, eoff, n, out, cap, olen, st, nullptr));
        (void)hipDeviceSynchronize();
        const double dt = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
        printf(" %.2f", bytes / dt / (1 << 30));
      }
      if (e) {
        printf(" same=%d", memcmp(enc, enc2, eoff[n]) == 0);
        (void)hipHostFree(enc2);
      } else {
        bool ok = true;
        for (uint64_t i = 0; i < n; i++) ok = ok && olen[i] == off[i + 1] - off[i] && !st[i];
        for (uint64_t i = 0; i < n && ok; i += 1001) ok = !memcmp(out + cap[i], data + off[i], olen[i]);
        printf(" ok=%d", (int)ok);
      }
      printf("\n");
      continue;
    } else if (!strcmp(step, "sleep")) {
      sleep(2);
    } else {
      fprintf(stderr, "unknown step %s\n", step);
      return 1;
    }
    printf("%s:", step);
    for (int k = 0; k < 3; k++) printf(" %.2f", dec(out, olen, st));
    printf("\n");
    fflush(stdout);
  }
  mhq_close(ctx);
  return 0;
}
