// Device-memory allocation cost on the GPU box (the cold-check stalls:
// growth of the fingerprint set to 2^30 slots took ~6 s in a fresh process).
// Times hipMalloc + hipMemset of a sequence of sizes, then VMM chunk maps.
//   alloc_probe [max_gib]
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <vector>
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %s\n", hipGetErrorString(e), #x); return 1; } } while (0)
static double now() { return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count(); }
int main(int argc, char** argv) {
  const double max_gib = argc > 1 ? atof(argv[1]) : 64;
  double t = now();
  CK(hipSetDevice(0));
  CK(hipFree(nullptr));
  printf("runtime init %.3fs\n", now() - t);
  std::vector<void*> keep;
  // the fingerprint-set growth sequence: 256 MiB doubling, the older table freed after the next is ready
  void* prev = nullptr;
  for (size_t b = 256ULL << 20; b <= (size_t)(max_gib * 1073741824.0); b *= 2) {
    void* p = nullptr;
    double t0 = now();
    CK(hipMalloc(&p, b));
    double t1 = now();
    CK(hipMemset(p, 0xFF, b));
    CK(hipDeviceSynchronize());
    double t2 = now();
    if (prev) CK(hipFree(prev));
    double t3 = now();
    printf("hipMalloc %7.2f GiB: malloc %.3fs memset %.3fs (%.0f GB/s) free-prev %.3fs\n", b / 1073741824.0, t1 - t0,
           t2 - t1, b / (t2 - t1) / 1e9, t3 - t2);
    prev = p;
  }
  if (prev) CK(hipFree(prev));
  // VMM: 512 MiB chunks mapped one after another (GrowBuf)
  hipMemAllocationProp prop = {};
  prop.type = hipMemAllocationTypePinned;
  prop.location.type = hipMemLocationTypeDevice;
  prop.location.id = 0;
  hipMemAccessDesc acc = {};
  acc.location.type = hipMemLocationTypeDevice;
  acc.location.id = 0;
  acc.flags = hipMemAccessFlagsProtReadWrite;
  const size_t CH = 512ULL << 20;
  const int nch = (int)(max_gib * 2);
  void* base = nullptr;
  CK(hipMemAddressReserve(&base, CH * nch, CH, nullptr, 0));
  std::vector<hipMemGenericAllocationHandle_t> hs;
  double tv = now(), tl = tv;
  for (int i = 0; i < nch; i++) {
    hipMemGenericAllocationHandle_t h;
    CK(hipMemCreate(&h, CH, &prop, 0));
    CK(hipMemMap((char*)base + i * CH, CH, 0, h, 0));
    CK(hipMemSetAccess((char*)base + i * CH, CH, &acc, 1));
    hs.push_back(h);
    if ((i + 1) % 16 == 0) {
      printf("VMM chunks %3d..%3d (%.0f GiB mapped): %.3fs (%.1f ms/chunk)\n", i - 15, i, (i + 1) * 0.5, now() - tl,
             (now() - tl) * 1000 / 16);
      tl = now();
    }
  }
  printf("VMM total %d chunks %.3fs\n", nch, now() - tv);
  for (int i = 0; i < nch; i++) { CK(hipMemUnmap((char*)base + i * CH, CH)); CK(hipMemRelease(hs[i])); }
  CK(hipMemAddressFree(base, CH * nch));
  return 0;
}
