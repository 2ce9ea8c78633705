// rmc_internal.h — librmc internals shared by the single-GPU driver
// (rmc_engine.cpp) and the sharded multi-GPU driver (rmc_sharded.cpp).
#pragma once
#include <hip/hip_runtime.h>
#include <stdexcept>
#include <string>
#include <utility>
#include <vector>
#include <algorithm>
#include "../../include/rmc.h"
#include "rmc_engine.h"

#define HIPCHK(x)                                                                   \
  do {                                                                              \
    hipError_t e_ = (x);                                                            \
    if (e_ != hipSuccess) {                                                         \
      throw std::runtime_error(std::string("HIP error: ") + hipGetErrorString(e_) + \
                               " at " #x);                                          \
    }                                                                               \
  } while (0)

// ---------------------------------------------------------------- model
struct rmc_model {
  std::string module, tla_text;
  rmc::Model M;
  int fp_aux = 0;  // reserved: no VIEW -> aux vars would join the fingerprint
  std::vector<std::string> server_names, value_names, inv_names;
  std::vector<std::string> var_order;
  std::vector<std::pair<std::string, std::string>> cfg_consts;  // cfg CONSTANTS, as written back by the trace module
  // results of the last check
  std::vector<std::pair<unsigned long long, unsigned long long>> levels;
  std::vector<std::vector<uint32_t>> trace_states;
  std::vector<std::string> trace_actions;
  uint32_t kmax_user = 0;
  // sizes the last check ended with (pre-size the next check of this model)
  unsigned long long hint_slots = 0, hint_fcap = 0, hint_trcap = 0;
  // largest |DOMAIN messages| of the last complete check: the next check of
  // this model packs rows to exactly that many message slots (an overflow
  // still re-runs with a larger capacity, so the hint is never unsafe)
  uint32_t hint_kmax = 0;
  // test hook (rmc_selftest_profile_expand): time k_expand's phases on the
  // first chunk of this level; (diag, ms) pairs of the last check
  unsigned profile_level = 0;
  std::vector<std::pair<int, double>> profile_ms;
};


namespace rmcx {

// Device memory ran out: the check ends with status 3 (capacity) and the
// counts reached so far, instead of an API error.
struct OutOfDeviceMemory : std::runtime_error {
  using std::runtime_error::runtime_error;
};

struct DevBuf {
  void* p = nullptr;
  size_t bytes = 0;
  void alloc(size_t b) {
    if (p) HIPCHK(hipFree(p));
    p = nullptr;
    bytes = 0;
    if (b) {
      hipError_t e = hipMalloc(&p, b);
      if (e == hipErrorOutOfMemory) {
        (void)hipGetLastError();
        p = nullptr;
        throw OutOfDeviceMemory("device memory exhausted (" + std::to_string(b >> 20) + " MiB requested)");
      }
      HIPCHK(e);
      bytes = b;
    }
  }
  void grow_copy(size_t b, size_t keep) {
    void* q = nullptr;
    HIPCHK(hipMalloc(&q, b));
    if (p && keep) HIPCHK(hipMemcpy(q, p, keep, hipMemcpyDeviceToDevice));
    if (p) HIPCHK(hipFree(p));
    p = q;
    bytes = b;
  }
  void ensure(size_t b) {  // at least b bytes; contents not kept
    if (p && bytes >= b) return;
    alloc(b);
  }
  void release() {
    if (p) (void)hipFree(p);
    p = nullptr;
    bytes = 0;
  }
  ~DevBuf() { release(); }
  template <class T>
  T* as() const { return (T*)p; }
};

// A device buffer that grows IN PLACE: one virtual address range is reserved
// once (the device's whole memory size), and physical memory is mapped onto
// its end as it grows (hipMemCreate/hipMemMap).  Growing never copies and
// never holds old and new copies at once -- the frontier and trace arrays of a
// large search would otherwise need twice their size during growth.  Falls
// back to allocate + copy + free where the VMM API is unavailable.
struct GrowBuf {
  void* p = nullptr;
  size_t bytes = 0;  // usable (mapped) bytes
  size_t reserved = 0, gran = 0;
  int dev = -1;
  bool vmm = false, tried = false;
  std::vector<std::pair<hipMemGenericAllocationHandle_t, size_t>> chunks;
  void init() {
    tried = true;
    HIPCHK(hipGetDevice(&dev));
    hipMemAllocationProp prop = {};
    prop.type = hipMemAllocationTypePinned;
    prop.location.type = hipMemLocationTypeDevice;
    prop.location.id = dev;
    if (hipMemGetAllocationGranularity(&gran, &prop, hipMemAllocationGranularityRecommended) != hipSuccess || !gran)
      return;
    size_t total = 0;
    if (hipDeviceTotalMem(&total, dev) != hipSuccess) return;
    const size_t CHUNK = (size_t)512 << 20;
    reserved = (total + CHUNK - 1) / CHUNK * CHUNK;
    void* q = nullptr;
    if (hipMemAddressReserve(&q, reserved, CHUNK, nullptr, 0) != hipSuccess) {
      (void)hipGetLastError();
      return;
    }
    p = q;
    vmm = true;
  }
  // at least b bytes; contents kept
  void ensure(size_t b) {
    if (b <= bytes && p) return;
    if (!tried) init();
    if (!vmm) {
      size_t nb = std::max(b, bytes * 2);
      void* q = nullptr;
      if (hipMalloc(&q, nb) != hipSuccess) {
        (void)hipGetLastError();
        throw OutOfDeviceMemory("device memory exhausted growing a frontier/trace buffer");
      }
      if (p && bytes) HIPCHK(hipMemcpy(q, p, bytes, hipMemcpyDeviceToDevice));
      if (p) HIPCHK(hipFree(p));
      p = q;
      bytes = nb;
      return;
    }
    // fixed 512 MiB chunks at chunk-aligned offsets (mapping at offsets that
    // are not multiples of the chunk size failed hipMemSetAccess on ROCm 7.2)
    const size_t CHUNK = (size_t)512 << 20;
    hipMemAllocationProp prop = {};
    prop.type = hipMemAllocationTypePinned;
    prop.location.type = hipMemLocationTypeDevice;
    prop.location.id = dev;
    hipMemAccessDesc acc = {};
    acc.location.type = hipMemLocationTypeDevice;
    acc.location.id = dev;
    acc.flags = hipMemAccessFlagsProtReadWrite;
    while (bytes < b) {
      if (bytes + CHUNK > reserved) throw OutOfDeviceMemory("buffer larger than the device");
      hipMemGenericAllocationHandle_t h;
      if (hipMemCreate(&h, CHUNK, &prop, 0) != hipSuccess) {
        (void)hipGetLastError();
        throw OutOfDeviceMemory("device memory exhausted growing a frontier/trace buffer");
      }
      char* at = (char*)p + bytes;
      HIPCHK(hipMemMap(at, CHUNK, 0, h, 0));
      HIPCHK(hipMemSetAccess(at, CHUNK, &acc, 1));
      chunks.push_back({h, CHUNK});
      bytes += CHUNK;
    }
  }
  void grow_copy(size_t b, size_t /*keep*/) { ensure(b); }  // contents are always kept
  void release() {
    if (vmm) {
      size_t off = 0;
      for (auto& c : chunks) {
        (void)hipMemUnmap((char*)p + off, c.second);
        (void)hipMemRelease(c.first);
        off += c.second;
      }
      chunks.clear();
      bytes = 0;  // the address range stays reserved for reuse
    } else {
      if (p) (void)hipFree(p);
      p = nullptr;
      bytes = 0;
    }
  }
  ~GrowBuf() {
    release();
    if (vmm && p) (void)hipMemAddressFree(p, reserved);
  }
  template <class T>
  T* as() const { return (T*)p; }
};

struct EventTimer {
  hipEvent_t a, b;
  EventTimer() { HIPCHK(hipEventCreate(&a)); HIPCHK(hipEventCreate(&b)); }
  ~EventTimer() { (void)hipEventDestroy(a); (void)hipEventDestroy(b); }
};

const char* act_label(int a);
void finalize_model(rmc_model* m, uint32_t kmax);
uint32_t default_kmax(const rmc::Model& M);
uint32_t model_kmax(const rmc_model* m);
std::vector<uint32_t> init_state(const rmc::Model& M);
std::string binding_label(const rmc_model* m, int b, int act);
void set_last_error(const std::string& s);
void release_shard_buffers();
// Rebuild the behaviour Init -> ... from the binding chain (root first), plus
// the failing binding (last_b >= 0) whose successor violated or erred.
void replay_trace(rmc_model* m, const std::vector<int>& binds, int last_b, int status, std::string& message,
                  rmc_result* res);

}  // namespace rmcx
