// What the HIP runtime reports for host buffers of each kind (the host
// path's zero-copy test): hipPointerGetAttributes and hipMemGetAddressRange on
// hipHostMalloc'd, hipHostRegister'ed and pageable memory, at the start and
// inside the buffer.
//   hipcc --offload-arch=gfx950 -o build/ptrattr tools/ptrattr.cpp && build/ptrattr
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

static void show(const char *what, void *p) {
  hipPointerAttribute_t a{};
  const hipError_t e = hipPointerGetAttributes(&a, p);
  hipDeviceptr_t base = nullptr;
  size_t size = 0;
  const hipError_t e2 = hipMemGetAddressRange(&base, &size, (hipDeviceptr_t)p);
  printf("%-22s attr=%d type=%d device=%d host=%p dev=%p (p=%p) range=%d base=%p size=%zu\n", what, (int)e, (int)a.type, a.device,
         a.hostPointer, a.devicePointer, p, (int)e2, base, size);
  (void)hipGetLastError();
}

int main() {
  void *h = nullptr;
  if (hipHostMalloc(&h, 1 << 20, hipHostMallocDefault) != hipSuccess) return 1;
  show("hostmalloc", h);
  show("hostmalloc+1000", (char *)h + 1000);
  show("hostmalloc+end-1", (char *)h + (1 << 20) - 1);
  show("hostmalloc+end", (char *)h + (1 << 20));
  void *r = aligned_alloc(4096, 1 << 20);
  if (hipHostRegister(r, 1 << 20, hipHostRegisterDefault) != hipSuccess) return 2;
  show("registered", r);
  show("registered+1000", (char *)r + 1000);
  void *m = malloc(1 << 20);
  show("pageable", m);
  void *d = nullptr;
  if (hipMalloc(&d, 1 << 20) != hipSuccess) return 3;
  show("device", d);
  show("device+1000", (char *)d + 1000);
  return 0;
}
