// When does HBM released from VMM chunks (hipMemUnmap + hipMemRelease) come
// back?  Variants after mapping + touching 80 GiB: (a) unmap + release only,
// (b) + hipMemAddressFree of the range, (c) + hipDeviceSynchronize / sleep;
// free reported by hipMemGetInfo and a 200 GiB hipMalloc after each.
#include <hip/hip_runtime.h>
#include <unistd.h>
#include <chrono>
#include <cstdio>
#include <vector>
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %s\n", hipGetErrorString(e), #x); return 1; } } while (0)
static double now() { return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count(); }
static double freegib() { size_t f = 0, t = 0; (void)hipMemGetInfo(&f, &t); return f / 1073741824.0; }
static const size_t CH = 512ULL << 20;
static int map80(void* va, std::vector<hipMemGenericAllocationHandle_t>& hs) {
  hipMemAllocationProp prop = {};
  prop.type = hipMemAllocationTypePinned;
  prop.location.type = hipMemLocationTypeDevice;
  prop.location.id = 0;
  hipMemAccessDesc acc = {};
  acc.location.type = hipMemLocationTypeDevice;
  acc.location.id = 0;
  acc.flags = hipMemAccessFlagsProtReadWrite;
  for (size_t i = 0; i < hs.size(); i++) {
    CK(hipMemCreate(&hs[i], CH, &prop, 0));
    CK(hipMemMap((char*)va + i * CH, CH, 0, hs[i], 0));
    CK(hipMemSetAccess((char*)va + i * CH, CH, &acc, 1));
  }
  CK(hipMemset(va, 0x5A, hs.size() * CH));
  CK(hipDeviceSynchronize());
  return 0;
}
static void unmap(void* va, std::vector<hipMemGenericAllocationHandle_t>& hs) {
  for (size_t i = 0; i < hs.size(); i++) {
    (void)hipMemUnmap((char*)va + i * CH, CH);
    (void)hipMemRelease(hs[i]);
  }
}
static void try_malloc(const char* tag) {
  void* p = nullptr;
  double t = now();
  hipError_t e = hipMalloc(&p, 200ULL << 30);
  printf("  %-34s hipMalloc 200 GiB: %s in %.3fs (free before free() %.1f)\n", tag, hipGetErrorString(e), now() - t,
         freegib());
  if (p) (void)hipFree(p);
  (void)hipGetLastError();
}
int main() {
  CK(hipSetDevice(0));
  CK(hipFree(nullptr));
  size_t total = 0;
  CK(hipDeviceTotalMem(&total, 0));
  const size_t resv = (total + CH - 1) / CH * CH;
  std::vector<hipMemGenericAllocationHandle_t> hs(160);
  printf("free at start %.1f GiB\n", freegib());
  for (int variant = 0; variant < 3; variant++) {
    void* va = nullptr;
    CK(hipMemAddressReserve(&va, resv, CH, nullptr, 0));
    if (map80(va, hs)) return 1;
    printf("variant %d: mapped 80 GiB, free %.1f\n", variant, freegib());
    unmap(va, hs);
    printf("  unmap+release: free %.1f\n", freegib());
    if (variant >= 1) {
      CK(hipMemAddressFree(va, resv));
      va = nullptr;
      printf("  + address free: free %.1f\n", freegib());
    }
    if (variant == 2) {
      CK(hipDeviceSynchronize());
      sleep(2);
      printf("  + sync + 2 s: free %.1f\n", freegib());
    }
    try_malloc("");
    printf("  after: free %.1f\n", freegib());
    if (va) CK(hipMemAddressFree(va, resv));
    sleep(1);
  }
  return 0;
}
