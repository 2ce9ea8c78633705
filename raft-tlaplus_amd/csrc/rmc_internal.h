// rmc_internal.h — librmc internals shared by the single-GPU driver
// (rmc_engine.cpp) and the sharded multi-GPU driver (rmc_sharded.cpp).
#pragma once
#include <hip/hip_runtime.h>
#include <stdexcept>
#include <string>
#include <utility>
#include <vector>
#include <algorithm>
#include <sys/mman.h>
#include <chrono>
#include <condition_variable>
#include <mutex>
#include <thread>
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
  // set when the TLA+ front end lowered the module text (rmc_tla.cpp): the
  // action table in the module's Next order, and its own operator names
  std::vector<std::pair<int, int>> lowered_actions;
  std::vector<std::string> lowered_labels;
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

// Host memory ran out (the host-frontier page pool hit its limit).
struct OutOfHostMemory : std::runtime_error {
  using std::runtime_error::runtime_error;
};

// BFS levels in pinned host memory (SURVEY.md §7 hard part 5: "page the
// frontier to pinned host memory when a level exceeds its budget").  A level
// is a sequence of fixed-size pinned pages, each holding `page_rows` packed
// rows; rows stream through HBM in chunk-sized windows (H2D before expansion,
// D2H after materialization) with async copies on a copy stream.  Pages of
// rows already consumed go back to the pool while the level is still being
// read, so the host peak is about one level plus the growth of the next.
struct HostPagePool {
  size_t page_bytes = 0;
  size_t allocated = 0, limit = 0;  // bytes of pinned pages held / allowed (including pages being pinned)
  double alloc_s = 0;               // time the BFS thread spent pinning or waiting for a pinned page
  std::vector<void*> free_pages;
  // Pinning threads: keep up to `ahead` free pages pinned so the BFS thread
  // does not wait for pinning while a level grows (hipHostMalloc pages at
  // 5.5 GB/s dominated host-frontier levels:
  // profiles/r03/ladder_Raft_n3v2e3_auto_pinning.txt).
  std::mutex mu;
  std::condition_variable cv;
  std::vector<std::thread> fillers;
  size_t ahead = 0, inflight = 0;
  bool stop = false, failed = false;
  // One page, outside the lock; nullptr when the host refuses.  Pages are
  // populated by the calling thread (mmap MAP_POPULATE: the kernel zeroes them
  // in parallel across threads) and then registered with HIP, which is cheap
  // on populated memory: 15 GB/s with 4 threads against 5.8 GB/s for
  // hipHostMalloc, which serialises in the driver (profiles/r03/pin_probe.txt).
  void* pin() {
    void* p = mmap(nullptr, page_bytes, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS | MAP_POPULATE, -1, 0);
    if (p == MAP_FAILED) return nullptr;
    if (hipHostRegister(p, page_bytes, hipHostRegisterDefault) != hipSuccess) {
      (void)hipGetLastError();
      munmap(p, page_bytes);
      return nullptr;
    }
    return p;
  }
  void unpin(void* p) {
    (void)hipHostUnregister(p);
    munmap(p, page_bytes);
  }
  void start_fillers(size_t pages, int threads) {
    if (!fillers.empty() || !pages || threads < 1) return;
    ahead = pages;
    stop = failed = false;
    for (int t = 0; t < threads; ++t) fillers.emplace_back([this] {
      std::unique_lock<std::mutex> lk(mu);
      for (;;) {
        cv.wait(lk, [this] { return stop || (!failed && free_pages.size() + inflight < ahead && allocated + page_bytes <= limit); });
        if (stop) return;
        allocated += page_bytes;  // reserved before pinning so get() cannot overshoot the limit
        ++inflight;
        lk.unlock();
        void* p = pin();
        lk.lock();
        --inflight;
        if (!p) {
          allocated -= page_bytes;
          failed = true;
        } else {
          free_pages.push_back(p);
        }
        cv.notify_all();
      }
    });
  }
  void stop_fillers() {
    if (fillers.empty()) return;
    {
      std::lock_guard<std::mutex> lk(mu);
      stop = true;
    }
    cv.notify_all();
    for (auto& t : fillers) t.join();
    fillers.clear();
  }
  void* get() {
    std::unique_lock<std::mutex> lk(mu);
    if (free_pages.empty() && !fillers.empty() && !failed) {
      // the pinning thread is behind: wait for its page rather than pin a second one here
      const auto t0 = std::chrono::steady_clock::now();
      cv.notify_all();
      cv.wait(lk, [this] { return !free_pages.empty() || failed || (!inflight && allocated + page_bytes > limit); });
      alloc_s += std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    }
    if (!free_pages.empty()) {
      void* p = free_pages.back();
      free_pages.pop_back();
      cv.notify_all();
      return p;
    }
    if (allocated + page_bytes > limit)
      throw OutOfHostMemory("host frontier pages exhausted (" + std::to_string(limit >> 30) + " GiB limit)");
    allocated += page_bytes;
    lk.unlock();
    const auto t0 = std::chrono::steady_clock::now();
    void* p = pin();
    lk.lock();
    alloc_s += std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    if (!p) {
      allocated -= page_bytes;
      throw OutOfHostMemory("pinned host memory exhausted (" + std::to_string(allocated >> 30) + " GiB held)");
    }
    return p;
  }
  void put(void* p) {
    if (!p) return;
    std::lock_guard<std::mutex> lk(mu);
    free_pages.push_back(p);
  }
  void release() {
    stop_fillers();
    const size_t nt = std::min<size_t>(4, free_pages.size() / 8);  // unmapping frees in parallel
    if (nt > 1) {
      std::vector<std::thread> th;
      for (size_t t = 0; t < nt; ++t)
        th.emplace_back([this, t, nt] { for (size_t i = t; i < free_pages.size(); i += nt) unpin(free_pages[i]); });
      for (auto& x : th) x.join();
    } else {
      for (void* p : free_pages) unpin(p);
    }
    allocated -= free_pages.size() * page_bytes;
    free_pages.clear();
  }
  ~HostPagePool() { release(); }
};
struct HostLevel {
  std::vector<void*> pages;  // nullptr: recycled (its rows were consumed)
  unsigned long long rows = 0;
  size_t page_rows = 1, row_bytes = 4;
  void init(size_t prow, size_t rb) { pages.clear(); rows = 0; page_rows = prow; row_bytes = rb; }
  // copy rows [r0, r0 + n) to dev (async on stream)
  void h2d(unsigned long long r0, unsigned long long n, void* dev, hipStream_t stream) const {
    char* d = (char*)dev;
    while (n) {
      const size_t pg = r0 / page_rows, off = r0 % page_rows, k = std::min<unsigned long long>(n, page_rows - off);
      if (pg >= pages.size() || !pages[pg]) throw std::runtime_error("host frontier: rows already recycled");
      HIPCHK(hipMemcpyAsync(d, (char*)pages[pg] + off * row_bytes, k * row_bytes, hipMemcpyHostToDevice, stream));
      d += k * row_bytes;
      r0 += k;
      n -= k;
    }
  }
  // reserve pages for n more rows (may allocate: call before enqueuing the copy)
  void reserve(unsigned long long n, HostPagePool& pool) {
    while ((rows + n + page_rows - 1) / page_rows > pages.size()) pages.push_back(pool.get());
  }
  // append n rows from dev (async on stream; pages reserved beforehand)
  void d2h_append(const void* dev, unsigned long long n, hipStream_t stream) {
    const char* s = (const char*)dev;
    while (n) {
      const size_t pg = rows / page_rows, off = rows % page_rows, k = std::min<unsigned long long>(n, page_rows - off);
      HIPCHK(hipMemcpyAsync((char*)pages[pg] + off * row_bytes, s, k * row_bytes, hipMemcpyDeviceToHost, stream));
      s += k * row_bytes;
      rows += k;
      n -= k;
    }
  }
  // give back the pages whose rows all lie below row r
  void recycle_below(unsigned long long r, HostPagePool& pool) {
    for (size_t pg = 0; pg < pages.size() && (pg + 1) * page_rows <= r; pg++) {
      pool.put(pages[pg]);
      pages[pg] = nullptr;
    }
  }
  void clear(HostPagePool& pool) {
    for (void* p : pages) pool.put(p);
    pages.clear();
    rows = 0;
  }
  const uint32_t* row(unsigned long long r) const {
    return (const uint32_t*)((const char*)pages[r / page_rows] + (r % page_rows) * row_bytes);
  }
};
// Host memory the host frontier may pin: RMC_HOST_FRONTIER_GIB, or 80% of
// MemAvailable capped at 200 GiB (a shared host must keep room for others).
size_t host_frontier_limit();

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
void release_single_buffers();
// Rebuild the behaviour Init -> ... from the binding chain (root first), plus
// the failing binding (last_b >= 0) whose successor violated or erred.
void replay_trace(rmc_model* m, const std::vector<int>& binds, int last_b, int status, std::string& message,
                  rmc_result* res);

}  // namespace rmcx
