// Probe of the HIP virtual-memory API on this ROCm: reserve a range, map two
// chunks one after the other, set access per chunk / over the whole range.
#include <hip/hip_runtime.h>
#include <cstdio>
int main() {
  int dev = 0;
  hipSetDevice(dev);
  hipMemAllocationProp prop = {};
  prop.type = hipMemAllocationTypePinned;
  prop.location.type = hipMemLocationTypeDevice;
  prop.location.id = dev;
  size_t gran = 0;
  printf("gran %d\n", (int)hipMemGetAllocationGranularity(&gran, &prop, hipMemAllocationGranularityRecommended));
  printf("granularity %zu\n", gran);
  size_t total = 0;
  hipDeviceTotalMem(&total, dev);
  size_t reserved = (total + gran - 1) / gran * gran;
  void* p = nullptr;
  printf("reserve %d (%zu GiB)\n", (int)hipMemAddressReserve(&p, reserved, 0, nullptr, 0), reserved >> 30);
  size_t step = 256ull << 20;
  hipMemAccessDesc acc = {};
  acc.location.type = hipMemLocationTypeDevice;
  acc.location.id = dev;
  acc.flags = hipMemAccessFlagsProtReadWrite;
  for (int mode = 0; mode < 2; mode++) {
    size_t base = mode * 4 * step;
    for (int c = 0; c < 3; c++) {
      hipMemGenericAllocationHandle_t h;
      int e1 = hipMemCreate(&h, step, &prop, 0);
      char* at = (char*)p + base + c * step;
      int e2 = hipMemMap(at, step, 0, h, 0);
      int e3 = mode == 0 ? hipMemSetAccess(at, step, &acc, 1) : hipMemSetAccess((char*)p + base, (c + 1) * step, &acc, 1);
      printf("mode %d chunk %d: create %d map %d access %d\n", mode, c, e1, e2, e3);
      (void)hipGetLastError();
    }
    int e4 = hipMemset((char*)p + base, 1, 3 * step);
    int e5 = hipDeviceSynchronize();
    unsigned char x = 0;
    int e6 = hipMemcpy(&x, (char*)p + base + 3 * step - 1, 1, hipMemcpyDeviceToHost);
    printf("mode %d memset %d sync %d read %d value %d\n", mode, e4, e5, e6, (int)x);
  }
  return 0;
}
