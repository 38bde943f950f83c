// ptr_probe — what hipPointerGetAttributes reports for each kind of buffer (no kernels launched):
// libmpjx rejects anything a kernel could not dereference before it launches one.
// Build: hipcc --offload-arch=gfx950 -O2 -o tools/ptr_probe tools/ptr_probe.cpp
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

static void show(const char* what, const void* p) {
  hipPointerAttribute_t at{};
  hipError_t e = hipPointerGetAttributes(&at, p);
  printf("%-28s %-22s type=%d device=%d devptr=%p\n", what, hipGetErrorString(e), (int)at.type, at.device,
         at.devicePointer);
  (void)hipGetLastError();
}

int main() {
  (void)hipSetDevice(0);
  int stackv[16];
  void* heap = malloc(1 << 20);
  void *dev = nullptr, *pinned = nullptr, *managed = nullptr;
  (void)hipMalloc(&dev, 1 << 20);
  (void)hipHostMalloc(&pinned, 1 << 20, 0);
  (void)hipMallocManaged(&managed, 1 << 20);
  void* reg = malloc(1 << 20);
  (void)hipHostRegister(reg, 1 << 20, 0);
  show("malloc (pageable)", heap);
  show("stack", stackv);
  show("hipMalloc", dev);
  show("hipMalloc + 4096", (char*)dev + 4096);
  show("hipHostMalloc", pinned);
  show("hipMallocManaged", managed);
  show("malloc + hipHostRegister", reg);
  printf("hipMemoryTypeUnregistered=%d Host=%d Device=%d Managed=%d\n", (int)hipMemoryTypeUnregistered,
         (int)hipMemoryTypeHost, (int)hipMemoryTypeDevice, (int)hipMemoryTypeManaged);
  return 0;
}
