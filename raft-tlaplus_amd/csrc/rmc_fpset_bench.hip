// rmc_fpset_bench.hip — fingerprint-set insert microbenchmark.
//
// The BFS's own insert (rmc_fpset.h fpset_insert: a CAS per probe; an
// atomicMin of the TLC-order rank unless the key is an earlier level's) on a
// table of 2^S slots.  Keys are splitmix64(42 + i).  For each target load L
// the table is prefilled (untimed, as an earlier level) to L minus the timed
// batch's new keys, then a batch of B inserts is timed with HIP events: a
// fraction `dup` of them re-insert an already present key (default 1 - D/G
// of the bench workload: 1 - 1/3.58), the rest are new, so the table ends at
// load L.  One line of JSON per load: inserts/s and line-granular bytes/s.
//
//   fpset_bench [-slots_log2 S] [-batch B] [-dup F] [-loads 0.25,0.5,0.75]
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <string>
#include <vector>
#include "rmc_fpset.h"

#define CK(x)                                                                       \
  do {                                                                              \
    hipError_t e_ = (x);                                                            \
    if (e_ != hipSuccess) {                                                         \
      fprintf(stderr, "HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); \
      exit(1);                                                                      \
    }                                                                               \
  } while (0)

namespace rmc {

__device__ __forceinline__ unsigned long long sm64(unsigned long long x) {
  unsigned long long z = x + 0x9E3779B97F4A7C15ULL;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
  return z ^ (z >> 31);
}
__device__ __forceinline__ unsigned long long key_of(unsigned long long i) { return sm64(42 + i); }

// keys [first, first + n) as an earlier level's entries (prefill; floor 0)
__global__ __launch_bounds__(256) void k_fill(unsigned long long* T, unsigned long long mask, unsigned long long first,
                                              unsigned long long n, DevStatus* st) {
  const unsigned long long stride = (unsigned long long)gridDim.x * blockDim.x;
  for (unsigned long long j = (unsigned long long)blockIdx.x * blockDim.x + threadIdx.x; j < n; j += stride)
    (void)fpset_insert(T, mask, key_of(first + j), (first + j) << VAL_RANK_SHIFT, 0ULL, st);
}

// the timed batch (level 2): insert j re-inserts a present key when its hash
// falls below dup_thresh, else inserts the new key present + j.  One slot written per insert,
// as k_expand writes cand_slot.
__global__ __launch_bounds__(256) void k_batch(unsigned long long* T, unsigned long long mask,
                                               unsigned long long present, unsigned long long nb,
                                               unsigned long long dup_thresh, unsigned long long* new_ctr,
                                               unsigned long long* out_slot, DevStatus* st) {
  const unsigned long long stride = (unsigned long long)gridDim.x * blockDim.x;
  for (unsigned long long j = (unsigned long long)blockIdx.x * blockDim.x + threadIdx.x; j < nb; j += stride) {
    const unsigned long long h = sm64(0xABCDEF ^ j);
    const bool fresh = h >= dup_thresh;
    const unsigned long long i = fresh ? present + j : sm64(h) % present;  // new keys: distinct indices
    const unsigned long long m = __ballot(fresh);  // one counter atomic per wave, not per key
    if ((threadIdx.x & 63) == 0 && m) atomicAdd(new_ctr, (unsigned long long)__popcll(m));
    // the batch is the next level: floor above every prefilled rank
    out_slot[j] = fpset_insert(T, mask, key_of(i), (present + 1 + j) << VAL_RANK_SHIFT,
                               present << VAL_RANK_SHIFT, st);
  }
}

// Counter calibration (MI355X_MICROARCH.md: FETCH_SIZE / WRITE_SIZE are
// calibrated only for wide streaming accesses): n random 16 B reads (one
// entry, one 128 B line each) of a table far larger than the 256 MiB
// Infinity Cache, then n random returning atomicMin on 8 B words.  Run under
// rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE: bytes per access = counter * 1024 / n.
__global__ __launch_bounds__(256) void k_calib_read(const unsigned long long* T, unsigned long long mask,
                                                    unsigned long long n, unsigned long long* sink) {
  const unsigned long long stride = (unsigned long long)gridDim.x * blockDim.x;
  unsigned long long acc = 0;
  for (unsigned long long j = (unsigned long long)blockIdx.x * blockDim.x + threadIdx.x; j < n; j += stride) {
    const ulonglong2 e = reinterpret_cast<const ulonglong2*>(T)[sm64(j * 7919) & mask];
    acc ^= e.x + e.y;
  }
  if (acc == 0x1234567ULL) sink[0] = acc;
}
__global__ __launch_bounds__(256) void k_calib_atomic(unsigned long long* T, unsigned long long mask,
                                                      unsigned long long n, unsigned long long* sink) {
  const unsigned long long stride = (unsigned long long)gridDim.x * blockDim.x;
  unsigned long long acc = 0;
  for (unsigned long long j = (unsigned long long)blockIdx.x * blockDim.x + threadIdx.x; j < n; j += stride)
    acc += atomicMin(T + 2 * (sm64(j * 104729) & mask) + 1, j);
  if (acc == 0x1234567ULL) sink[0] = acc;
}

}  // namespace rmc

int main(int argc, char** argv) {
  int slots_log2 = 30;
  unsigned long long batch = 64ULL << 20;
  double dup = 1.0 - 1.0 / 3.58;
  std::vector<double> loads = {0.25, 0.5, 0.75};
  bool calib = false;
  for (int a = 1; a < argc; a++) {
    std::string k = argv[a];
    const char* v = a + 1 < argc ? argv[a + 1] : "";
    if (k == "-calib") calib = true;
    else if (k == "-slots_log2") slots_log2 = atoi(v), a++;
    else if (k == "-batch") batch = strtoull(v, nullptr, 10), a++;
    else if (k == "-dup") dup = atof(v), a++;
    else if (k == "-loads") {
      loads.clear();
      for (char* t = strtok((char*)v, ","); t; t = strtok(nullptr, ",")) loads.push_back(atof(t));
      a++;
    } else {
      fprintf(stderr, "usage: fpset_bench [-slots_log2 S] [-batch B] [-dup F] [-loads L1,L2,...] [-calib]\n");
      return 2;
    }
  }
  if (slots_log2 < 10 || slots_log2 > 34 || dup < 0 || dup >= 1) {
    fprintf(stderr, "fpset_bench: bad arguments\n");
    return 2;
  }
  const unsigned long long slots = 1ULL << slots_log2, mask = slots - 1;
  unsigned long long *T = nullptr, *slot = nullptr, *ctr = nullptr;
  rmc::DevStatus* st = nullptr;
  CK(hipMalloc(&T, slots * 16));
  CK(hipMalloc(&slot, batch * 8));
  CK(hipMalloc(&ctr, 8));
  CK(hipMalloc(&st, sizeof(rmc::DevStatus)));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const unsigned grid = 256 * 64;  // grid-stride: 64 blocks per CU
  if (calib) {
    CK(hipMemset(T, 0x11, slots * 16));
    CK(hipDeviceSynchronize());
    for (int kind = 0; kind < 2; kind++) {
      CK(hipEventRecord(e0, 0));
      if (kind == 0) hipLaunchKernelGGL(rmc::k_calib_read, dim3(grid), dim3(256), 0, 0, T, mask, batch, ctr);
      else hipLaunchKernelGGL(rmc::k_calib_atomic, dim3(grid), dim3(256), 0, 0, T, mask, batch, ctr);
      CK(hipGetLastError());
      CK(hipEventRecord(e1, 0));
      CK(hipEventSynchronize(e1));
      float ms = 0;
      CK(hipEventElapsedTime(&ms, e0, e1));
      printf("{\"calib\": \"%s\", \"accesses\": %llu, \"table_bytes\": %llu, \"ms\": %.3f, \"per_s\": %.4g}\n",
             kind == 0 ? "random_16B_read" : "random_8B_atomicMin", batch, slots * 16, ms, batch / (ms * 1e-3));
      fflush(stdout);
    }
    return 0;
  }
  for (double L : loads) {
    const unsigned long long target = (unsigned long long)(L * (double)slots);
    const unsigned long long nb_new = (unsigned long long)((1.0 - dup) * (double)batch);
    if (target <= nb_new + 1 || L >= 0.95) {
      fprintf(stderr, "fpset_bench: load %.2f too small for the batch (or too close to full)\n", L);
      return 2;
    }
    const unsigned long long present = target - nb_new;
    CK(hipMemset(T, 0xFF, slots * 16));
    CK(hipMemset(ctr, 0, 8));
    CK(hipMemset(st, 0, sizeof(rmc::DevStatus)));
    hipLaunchKernelGGL(rmc::k_fill, dim3(grid), dim3(256), 0, 0, T, mask, 0ULL, present, st);
    CK(hipGetLastError());
    CK(hipDeviceSynchronize());
    const unsigned long long thresh = (unsigned long long)(dup * 18446744073709551615.0);
    CK(hipEventRecord(e0, 0));
    hipLaunchKernelGGL(rmc::k_batch, dim3(grid), dim3(256), 0, 0, T, mask, present, batch, thresh, ctr, slot, st);
    CK(hipGetLastError());
    CK(hipEventRecord(e1, 0));
    CK(hipEventSynchronize(e1));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, e0, e1));
    unsigned long long added = 0;
    rmc::DevStatus hs;
    CK(hipMemcpy(&added, ctr, 8, hipMemcpyDeviceToHost));
    CK(hipMemcpy(&hs, st, sizeof hs, hipMemcpyDeviceToHost));
    const double s = ms * 1e-3;
    // line-granular traffic: every insert reads one 128 B line; a new key
    // also writes it back (duplicates of earlier levels leave it clean)
    printf("{\"slots_log2\": %d, \"load\": %.3f, \"batch\": %llu, \"dup\": %.3f, \"new\": %llu, \"ms\": %.3f, "
           "\"inserts_per_s\": %.4g, \"line_GBps_min\": %.1f, \"table_full\": %d}\n",
           slots_log2, (double)(present + added) / (double)slots, batch, dup, added, ms, batch / s,
           (batch * 128.0 + added * 128.0) / s / 1e9, hs.cap_flags != 0);
    fflush(stdout);
  }
  CK(hipFree(T));
  CK(hipFree(slot));
  CK(hipFree(ctr));
  CK(hipFree(st));
  return 0;
}
