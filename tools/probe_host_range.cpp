// probe_host_range.cpp — what the HIP runtime reports for page-locked host ranges (hipHostMalloc'd
// blocks and hipHostRegister'ed halves of one mapping), and which copies into them it accepts: the
// evidence behind host_copy() / in_one_allocation() in mpjx_collectives.hip.
// Prints one JSON object per case. Build: hipcc -O2 tools/probe_host_range.cpp -o /tmp/probe_host_range
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <string.h>
#include <sys/mman.h>

#include <algorithm>
#include <vector>

static void report(const char* what, void* p, size_t want) {
  hipPointerAttribute_t a{};
  const hipError_t ea = hipPointerGetAttributes(&a, p);
  (void)hipGetLastError();
  hipDeviceptr_t base = nullptr;
  size_t size = 0;
  const hipError_t er = hipMemGetAddressRange(&base, &size, (hipDeviceptr_t)p);
  (void)hipGetLastError();
  void* rs = nullptr;
  size_t rz = 0;
  const hipError_t e1 = hipPointerGetAttribute(&rs, HIP_POINTER_ATTRIBUTE_RANGE_START_ADDR, (hipDeviceptr_t)p);
  (void)hipGetLastError();
  const hipError_t e2 = hipPointerGetAttribute(&rz, HIP_POINTER_ATTRIBUTE_RANGE_SIZE, (hipDeviceptr_t)p);
  (void)hipGetLastError();
  printf("{\"case\": \"%s\", \"attrs\": %d, \"type\": %d, \"dev_eq_host\": %d, \"addr_range\": %d, \"off\": %lld, "
         "\"size\": %zu, \"range_start_rc\": %d, \"range_start_off\": %lld, \"range_size_rc\": %d, \"range_size\": %zu, "
         "\"want\": %zu}\n",
         what, (int)ea, (int)a.type, a.devicePointer == p, (int)er, base ? (long long)((char*)p - (char*)base) : -1LL,
         size, (int)e1, rs ? (long long)((char*)p - (char*)rs) : -1LL, (int)e2, rz, want);
}

static void copy_case(const char* what, void* host, size_t bytes, void* dev) {
  const hipError_t e = hipMemcpy(host, dev, bytes, hipMemcpyDeviceToHost);
  (void)hipGetLastError();
  printf("{\"copy\": \"%s\", \"bytes\": %zu, \"rc\": %d}\n", what, bytes, (int)e);
}

int main() {
  void* dev = nullptr;
  if (hipMalloc(&dev, 8 << 20) != hipSuccess) return 1;
  // hipHostMalloc'd blocks: look for two placed back to back
  std::vector<char*> blocks;
  for (int i = 0; i < 24; i++) {
    void* p = nullptr;
    if (hipHostMalloc(&p, 1 << 20, 0) != hipSuccess) return 2;
    blocks.push_back((char*)p);
  }
  report("hostmalloc_block", blocks[0], 1 << 20);
  report("hostmalloc_mid", blocks[0] + 12345, 1 << 20);
  std::vector<char*> sorted = blocks;
  std::sort(sorted.begin(), sorted.end());
  long long gap_min = -1;
  for (size_t i = 1; i < sorted.size(); i++) {
    const long long g = (long long)(sorted[i] - sorted[i - 1]) - (1 << 20);
    if (gap_min < 0 || g < gap_min) gap_min = g;
  }
  printf("{\"hostmalloc_min_gap_bytes\": %lld}\n", gap_min);
  // two registered halves of one anonymous mapping
  const size_t half = 2 << 20;
  char* m = (char*)mmap(nullptr, 2 * half, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0);
  memset(m, 0, 2 * half);
  const hipError_t r1 = hipHostRegister(m, half, 0), r2 = hipHostRegister(m + half, half, 0);
  printf("{\"register\": [%d, %d]}\n", (int)r1, (int)r2);
  report("registered_first_half", m, half);
  report("registered_second_half_mid", m + half + 4096, half);
  copy_case("registered_within_first_half", m + half - 65536, 65536, dev);
  copy_case("registered_spanning_halves", m + half - 65536, 131072, dev);
  copy_case("registered_second_half", m + half, 65536, dev);
  copy_case("hostmalloc_within", blocks[0], 65536, dev);
  hipHostUnregister(m);
  hipHostUnregister(m + half);
  munmap(m, 2 * half);
  for (char* b : blocks) hipHostFree(b);
  hipFree(dev);
  return 0;
}
