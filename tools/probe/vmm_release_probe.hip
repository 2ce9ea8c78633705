// Does unmapping + releasing VMM chunks return their HBM (hipMemGetInfo,
// a following hipMalloc)?  And does hipMalloc stall once VMM ranges are
// reserved (the engine's GrowBufs reserve 4 x the device size of VA)?
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>
#include <vector>
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %s\n", hipGetErrorString(e), #x); return 1; } } while (0)
static double now() { return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count(); }
static double freegib() { size_t f = 0, t = 0; (void)hipMemGetInfo(&f, &t); return f / 1073741824.0; }
int main() {
  CK(hipSetDevice(0));
  CK(hipFree(nullptr));
  size_t total = 0;
  CK(hipDeviceTotalMem(&total, 0));
  const size_t CH = 512ULL << 20;
  const size_t resv = (total + CH - 1) / CH * CH;
  hipMemAllocationProp prop = {};
  prop.type = hipMemAllocationTypePinned;
  prop.location.type = hipMemLocationTypeDevice;
  prop.location.id = 0;
  hipMemAccessDesc acc = {};
  acc.location.type = hipMemLocationTypeDevice;
  acc.location.id = 0;
  acc.flags = hipMemAccessFlagsProtReadWrite;
  void* va[4];
  for (int k = 0; k < 4; k++) CK(hipMemAddressReserve(&va[k], resv, CH, nullptr, 0));
  printf("free at start %.1f GiB\n", freegib());
  const int n = 160;  // 80 GiB in fa
  std::vector<hipMemGenericAllocationHandle_t> hs(n);
  double t = now();
  for (int i = 0; i < n; i++) {
    CK(hipMemCreate(&hs[i], CH, &prop, 0));
    CK(hipMemMap((char*)va[0] + i * CH, CH, 0, hs[i], 0));
    CK(hipMemSetAccess((char*)va[0] + i * CH, CH, &acc, 1));
  }
  printf("mapped %d chunks in %.3fs; free %.1f GiB\n", n, now() - t, freegib());
  t = now();
  CK(hipMemset(va[0], 0x5A, n * CH));
  CK(hipDeviceSynchronize());
  printf("touched in %.3fs; free %.1f GiB\n", now() - t, freegib());
  t = now();
  for (int i = 0; i < n; i++) {
    hipError_t e1 = hipMemUnmap((char*)va[0] + i * CH, CH);
    hipError_t e2 = hipMemRelease(hs[i]);
    if (e1 != hipSuccess || e2 != hipSuccess) { printf("unmap/release %d: %s / %s\n", i, hipGetErrorString(e1), hipGetErrorString(e2)); break; }
  }
  printf("unmapped+released in %.3fs; free %.1f GiB\n", now() - t, freegib());
  CK(hipDeviceSynchronize());
  printf("after sync free %.1f GiB\n", freegib());
  void* p = nullptr;
  t = now();
  hipError_t e = hipMalloc(&p, 200ULL << 30);
  printf("hipMalloc 200 GiB: %s in %.3fs; free %.1f GiB\n", hipGetErrorString(e), now() - t, freegib());
  if (p) CK(hipFree(p));
  // the engine's table growth sequence with the VA reservations in place
  void* prev = nullptr;
  for (size_t b = 256ULL << 20; b <= (64ULL << 30); b *= 2) {
    void* q = nullptr;
    double t0 = now();
    CK(hipMalloc(&q, b));
    double t1 = now();
    CK(hipMemset(q, 0xFF, b));
    CK(hipDeviceSynchronize());
    double t2 = now();
    if (prev) CK(hipFree(prev));
    printf("hipMalloc %6.2f GiB: malloc %.3fs fill %.3fs free-prev %.3fs\n", b / 1073741824.0, t1 - t0, t2 - t1, now() - t2);
    prev = q;
  }
  CK(hipFree(prev));
  for (int k = 0; k < 4; k++) CK(hipMemAddressFree(va[k], resv));
  return 0;
}
