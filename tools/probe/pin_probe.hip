// Pinned host memory costs on the GPU box: hipHostMalloc of 256 MiB pages
// (serial and from 4 threads) against mmap + MAP_POPULATE (4 threads) followed
// by hipHostRegister, and the H2D rate from each kind of page.
#include <hip/hip_runtime.h>
#include <sys/mman.h>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <thread>
#include <vector>
static double now() { return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count(); }
#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s failed: %s\n", #x, hipGetErrorString(e_)); exit(1); } } while (0)
int main(int argc, char** argv) {
  const size_t page = 256ull << 20;
  const int n = argc > 1 ? atoi(argv[1]) : 32;  // pages per experiment
  CK(hipSetDevice(0));
  void* dev = nullptr;
  CK(hipMalloc(&dev, page));
  // (a) hipHostMalloc, serial
  std::vector<void*> a(n);
  double t = now();
  for (int i = 0; i < n; ++i) CK(hipHostMalloc(&a[i], page, hipHostMallocDefault));
  double ta = now() - t;
  printf("hipHostMalloc serial: %.2f GB/s (%d x 256 MiB in %.3f s)\n", n * page / ta / 1e9, n, ta);
  // (b) hipHostMalloc from 4 threads
  std::vector<void*> b(n);
  t = now();
  {
    std::vector<std::thread> th;
    for (int k = 0; k < 4; ++k) th.emplace_back([&, k] { for (int i = k; i < n; i += 4) CK(hipHostMalloc(&b[i], page, hipHostMallocDefault)); });
    for (auto& x : th) x.join();
  }
  double tb = now() - t;
  printf("hipHostMalloc 4 threads: %.2f GB/s\n", n * page / tb / 1e9);
  // (c) mmap + MAP_POPULATE from 4 threads, then hipHostRegister serially
  std::vector<void*> c(n);
  t = now();
  {
    std::vector<std::thread> th;
    for (int k = 0; k < 4; ++k) th.emplace_back([&, k] {
      for (int i = k; i < n; i += 4) {
        c[i] = mmap(nullptr, page, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS | MAP_POPULATE, -1, 0);
        if (c[i] == MAP_FAILED) { printf("mmap failed\n"); exit(1); }
      }
    });
    for (auto& x : th) x.join();
  }
  double tc1 = now() - t;
  t = now();
  for (int i = 0; i < n; ++i) CK(hipHostRegister(c[i], page, hipHostRegisterDefault));
  double tc2 = now() - t;
  printf("mmap+populate 4 threads: %.2f GB/s; hipHostRegister serial: %.2f GB/s; combined %.2f GB/s\n", n * page / tc1 / 1e9,
         n * page / tc2 / 1e9, n * page / (tc1 + tc2) / 1e9);
  // (d) hipHostRegister from 4 threads on fresh populated memory
  std::vector<void*> d(n);
  for (int i = 0; i < n; ++i) {
    d[i] = mmap(nullptr, page, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS | MAP_POPULATE, -1, 0);
    if (d[i] == MAP_FAILED) { printf("mmap failed\n"); exit(1); }
  }
  t = now();
  {
    std::vector<std::thread> th;
    for (int k = 0; k < 4; ++k) th.emplace_back([&, k] { for (int i = k; i < n; i += 4) CK(hipHostRegister(d[i], page, hipHostRegisterDefault)); });
    for (auto& x : th) x.join();
  }
  double td = now() - t;
  printf("hipHostRegister 4 threads: %.2f GB/s\n", n * page / td / 1e9);
  // H2D rates
  hipStream_t s;
  CK(hipStreamCreate(&s));
  for (auto* v : {&a, &c}) {
    CK(hipMemcpyAsync(dev, (*v)[0], page, hipMemcpyHostToDevice, s));
    CK(hipStreamSynchronize(s));
    t = now();
    for (int i = 0; i < n; ++i) CK(hipMemcpyAsync(dev, (*v)[i], page, hipMemcpyHostToDevice, s));
    CK(hipStreamSynchronize(s));
    double th2d = now() - t;
    t = now();
    for (int i = 0; i < n; ++i) CK(hipMemcpyAsync((*v)[i], dev, page, hipMemcpyDeviceToHost, s));
    CK(hipStreamSynchronize(s));
    double td2h = now() - t;
    printf("%s: H2D %.2f GB/s, D2H %.2f GB/s\n", v == &a ? "hipHostMalloc pages" : "registered pages", n * page / th2d / 1e9,
           n * page / td2h / 1e9);
  }
  t = now();
  for (int i = 0; i < n; ++i) CK(hipHostFree(a[i]));
  for (int i = 0; i < n; ++i) CK(hipHostFree(b[i]));
  double tf = now() - t;
  t = now();
  for (int i = 0; i < n; ++i) { CK(hipHostUnregister(c[i])); munmap(c[i], page); CK(hipHostUnregister(d[i])); munmap(d[i], page); }
  printf("free: hipHostFree %.3f s, unregister+munmap %.3f s\n", tf, now() - t);
  CK(hipFree(dev));
  return 0;
}
