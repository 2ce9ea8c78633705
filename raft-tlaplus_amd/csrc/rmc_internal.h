// rmc_internal.h — librmc internals shared by the single-GPU driver
// (rmc_engine.cpp) and the sharded multi-GPU driver (rmc_sharded.cpp).
#pragma once
#include <hip/hip_runtime.h>
#include <stdexcept>
#include <string>
#include <utility>
#include <vector>
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
  // results of the last check
  std::vector<std::pair<unsigned long long, unsigned long long>> levels;
  std::vector<std::vector<uint32_t>> trace_states;
  std::vector<std::string> trace_actions;
  uint32_t kmax_user = 0;
  // sizes the last check ended with (pre-size the next check of this model)
  unsigned long long hint_slots = 0, hint_fcap = 0, hint_trcap = 0;
};


namespace rmcx {

struct DevBuf {
  void* p = nullptr;
  size_t bytes = 0;
  void alloc(size_t b) {
    if (p) HIPCHK(hipFree(p));
    p = nullptr;
    bytes = b;
    if (b) HIPCHK(hipMalloc(&p, b));
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

struct EventTimer {
  hipEvent_t a, b;
  EventTimer() { HIPCHK(hipEventCreate(&a)); HIPCHK(hipEventCreate(&b)); }
  ~EventTimer() { (void)hipEventDestroy(a); (void)hipEventDestroy(b); }
};

const char* act_label(int a);
void finalize_model(rmc_model* m, uint32_t kmax);
uint32_t default_kmax(const rmc::Model& M);
std::vector<uint32_t> init_state(const rmc::Model& M);
std::string binding_label(const rmc_model* m, int b, int act);
void set_last_error(const std::string& s);
void release_shard_buffers();
// Rebuild the behaviour Init -> ... from the binding chain (root first), plus
// the failing binding (last_b >= 0) whose successor violated or erred.
void replay_trace(rmc_model* m, const std::vector<int>& binds, int last_b, int status, std::string& message,
                  rmc_result* res);

}  // namespace rmcx
