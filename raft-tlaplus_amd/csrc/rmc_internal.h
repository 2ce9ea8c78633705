// rmc_internal.h — librmc internals shared by the single-GPU driver
// (rmc_engine.cpp) and the sharded multi-GPU driver (rmc_sharded.cpp).
#pragma once
#include <hip/hip_runtime.h>
#include <cstring>
#include <stdexcept>
#include <string>
#include <utility>
#include <vector>
#include <array>
#include <algorithm>
#include <sys/mman.h>
#include <chrono>
#include <condition_variable>
#include <mutex>
#include <thread>
#include "../../include/rmc.h"
#include "rmc_engine.h"
#include "rmc_tla.h"
#include <map>

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
  // the cfg's integer constants (the guard compiler's environment) and the
  // guards compiled onto library effects (rmc_guard.cpp)
  std::map<std::string, long long> int_consts;
  std::vector<rmc::tla::GuardSrc> guard_srcs;
  // actions defined as TLA+ text (rmc_model_define_action), by name: compiled
  // whole when rmc_model_set_next puts them in Next
  std::map<std::string, rmc::tla::GuardSrc> defined_actions;
  // the last check's row widenings (depth, first parent of the redone chunk, new message slots)
  std::vector<std::array<unsigned long long, 3>> widenings;
  // the last check's host-frontier buffer regrowths while its copy streams ran:
  // compact-row pack buffers, output windows (test hook rmc_selftest_hf_stats)
  unsigned long long hf_pack_regrows = 0, hf_out_regrows = 0;
  // the last single-GPU check's wall time by phase, seconds (rmc_check_phases)
  std::vector<std::pair<std::string, double>> phases;
};


namespace rmcx {

// Device memory ran out: the check ends with status 3 (capacity) and the
// counts reached so far, instead of an API error.
struct OutOfDeviceMemory : std::runtime_error {
  using std::runtime_error::runtime_error;
};

// Freeing or unmapping device memory waits for the whole device first: async
// copies and kernels of the check's several streams (the host frontier's
// copy streams among them) may still read a buffer that is being regrown or
// released -- an unmapped range they touch is a GPU page fault ("illegal
// memory access" at the next sync, the r04/r05 host-frontier failure).
inline void drain_device() { (void)hipDeviceSynchronize(); }
// The same on a path that can report: a fault of in-flight work surfaces here,
// named after the buffer being freed, not at some later unrelated call.
inline void drain_device_checked(const char* what) {
  const hipError_t e = hipDeviceSynchronize();
  if (e != hipSuccess)
    throw std::runtime_error(std::string("HIP error: ") + hipGetErrorString(e) + " at the drain before " + what);
}

struct DevBuf {
  void* p = nullptr;
  size_t bytes = 0;
  void alloc(size_t b) {
    if (p) {
      drain_device_checked("a device buffer is regrown");
      HIPCHK(hipFree(p));
    }
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
    if (p) {
      drain_device_checked("a device buffer is regrown (copy)");
      HIPCHK(hipFree(p));
    }
    p = q;
    bytes = b;
  }
  void ensure(size_t b) {  // at least b bytes; contents not kept
    if (p && bytes >= b) return;
    alloc(b);
  }
  void release() {
    if (p) {
      drain_device();
      (void)hipFree(p);
    }
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
      if (p) {
        drain_device_checked("a frontier/trace buffer is regrown");
        HIPCHK(hipFree(p));
      }
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
  // Unmapped and released chunks return their HBM only when the address
  // range is freed too (measured: profiles/r04/vmm_free_probe.txt -- 80 GiB
  // stayed in use after hipMemUnmap + hipMemRelease and came back at
  // hipMemAddressFree), so the range goes as well; the next ensure()
  // reserves a new one.
  void release() {
    if (p) drain_device();
    if (vmm) {
      size_t off = 0;
      for (auto& c : chunks) {
        (void)hipMemUnmap((char*)p + off, c.second);
        (void)hipMemRelease(c.first);
        off += c.second;
      }
      chunks.clear();
      if (p) (void)hipMemAddressFree(p, reserved);
      vmm = false;
      tried = false;
      reserved = 0;
    } else if (p) {
      (void)hipFree(p);
    }
    p = nullptr;
    bytes = 0;
  }
  ~GrowBuf() { release(); }
  template <class T>
  T* as() const { return (T*)p; }
};

// Host memory ran out (the host-frontier page pool hit its limit).
struct OutOfHostMemory : std::runtime_error {
  using std::runtime_error::runtime_error;
};
// A compact row longer than its fixed row (k_row_words' bound): status 3.
struct RowCapacity : std::runtime_error {
  using std::runtime_error::runtime_error;
};

// Registered host pages outlive a check (r05).  Each check used to pin its
// own pages (mmap + hipHostRegister) and unregister + munmap them at its end;
// the next check's mmap then got the same virtual addresses back and
// registered them again.  The driver's GPU run of r04 faulted in a D2H copy
// into host-frontier pages (an illegal address on the copy-out stream) after
// ~30 such checks in one process, a fault no bounded kernel access explains.
// Now (1) a process-wide cache keeps up to RMC_HF_RETAIN_GIB (default 8) of
// registered pages for the next check, so a test process registers them once,
// and (2) a page given up is unregistered and its address range is replaced
// by an inaccessible reservation (PROT_NONE, no backing memory) instead of
// unmapped, so no address that was ever registered is handed to a new
// registration -- whatever the runtime still holds for a retired range can
// never alias a live page.
struct PinnedPageCache {
  std::mutex mu;
  size_t page_bytes = 0;
  std::vector<void*> pages;
  size_t retain = 0;
  unsigned long long retired = 0;  // pages given up (address ranges quarantined)
  static PinnedPageCache& get() {
    static PinnedPageCache* c = [] {  // never destroyed: pages may outlive static destructors' HIP runtime
      auto* k = new PinnedPageCache();
      const char* e = getenv("RMC_HF_RETAIN_GIB");
      k->retain = (size_t)((e ? atof(e) : 8.0) * 1073741824.0);
      return k;
    }();
    return *c;
  }
  static void retire(void* p, size_t bytes) {
    drain_device();  // no copy may still target the page
    (void)hipHostUnregister(p);
    void* q = mmap(p, bytes, PROT_NONE, MAP_FIXED | MAP_PRIVATE | MAP_ANONYMOUS | MAP_NORESERVE, -1, 0);
    if (q == MAP_FAILED) munmap(p, bytes);
  }
  void* take(size_t bytes) {
    std::lock_guard<std::mutex> lk(mu);
    if (page_bytes != bytes || pages.empty()) return nullptr;
    void* p = pages.back();
    pages.pop_back();
    return p;
  }
  // keep p for a later check, or retire it; returns true when kept
  bool give(void* p, size_t bytes) {
    {
      std::lock_guard<std::mutex> lk(mu);
      if (page_bytes != bytes) {  // another page size: the cached ones go
        for (void* q : pages) retire(q, page_bytes);
        retired += pages.size();
        pages.clear();
        page_bytes = bytes;
      }
      if ((pages.size() + 1) * bytes <= retain) {
        pages.push_back(p);
        return true;
      }
      retired++;
    }
    retire(p, bytes);
    return false;
  }
};

// BFS levels in pinned host memory (SURVEY.md §7 hard part 5: "page the
// frontier to pinned host memory when a level exceeds its budget").  A level
// is a sequence of fixed-size pinned pages, each holding `page_rows` packed
// rows; rows stream through HBM in chunk-sized windows (H2D before expansion,
// D2H after materialization) with async copies on a copy stream.  Pages of
// rows already consumed go back to the pool while the level is still being
// read, so the host peak is about one level plus the growth of the next.
struct HostPagePool {
  // every pool pages in these units (compact rows straddle pages; tests set
  // RMC_HOST_PAGE_ROWS for small ones), so cached pages fit every check
  static constexpr size_t PAGE_BYTES = 256ULL << 20;
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
  // One page, outside the lock; nullptr when the host refuses.  A page the
  // process-wide cache holds is reused as it is; otherwise pages are
  // populated by the calling thread (mmap MAP_POPULATE: the kernel zeroes them
  // in parallel across threads) and then registered with HIP, which is cheap
  // on populated memory: 15 GB/s with 4 threads against 5.8 GB/s for
  // hipHostMalloc, which serialises in the driver (profiles/r03/pin_probe.txt).
  void* pin() {
    if (void* c = PinnedPageCache::get().take(page_bytes)) return c;
    void* p = mmap(nullptr, page_bytes, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS | MAP_POPULATE, -1, 0);
    if (p == MAP_FAILED) return nullptr;
    // portable: a cached page may serve another GPU's thread in a later check (rmc_check_multi)
    if (hipHostRegister(p, page_bytes, hipHostRegisterPortable) != hipSuccess) {
      (void)hipGetLastError();
      munmap(p, page_bytes);
      return nullptr;
    }
    return p;
  }
  void unpin(void* p) { PinnedPageCache::get().give(p, page_bytes); }
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
// A level in host memory, COMPACT: each packed row trimmed after its last
// DOMAIN message (1 + 4N + nmsg words), rows back to back in a byte stream
// over pinned pages (a row may straddle two pages).  lens[r] = row r's words;
// cum[k] = byte offset of row k * IDX (a chunk's byte range is found from
// them).  Rows are packed on the device before they cross PCIe and unpacked
// into fixed-stride rows on the way back (rmc_kernels.hip k_pack_rows /
// k_unpack_rows), so the kernels never see this form.
struct HostLevel {
  static constexpr unsigned long long IDX = 4096;
  std::vector<void*> pages;  // nullptr: recycled (its rows were consumed)
  size_t page_bytes = 1, row_bytes = 4;
  unsigned long long rows = 0, bytes = 0;
  std::vector<uint8_t> lens;
  std::vector<unsigned long long> cum;
  void init(size_t pbytes, size_t rb) {
    pages.clear();
    lens.clear();
    cum.clear();
    rows = bytes = 0;
    page_bytes = pbytes;
    row_bytes = rb;
  }
  unsigned long long byte_of(unsigned long long r) const {  // r <= rows
    if (r >= rows) return bytes;
    unsigned long long b = cum[r / IDX];
    for (unsigned long long q = r / IDX * IDX; q < r; q++) b += 4ULL * lens[q];
    return b;
  }
  void reserve_bytes(unsigned long long nb, HostPagePool& pool) {
    while ((bytes + nb + page_bytes - 1) / page_bytes > pages.size()) pages.push_back(pool.get());
  }
  // record n rows of the given word counts; returns their bytes (the caller copies them in)
  unsigned long long add_rows(const uint8_t* l, unsigned long long n) {
    unsigned long long b = bytes, nb = 0;
    lens.reserve(lens.size() + n);
    for (unsigned long long q = 0; q < n; q++) {
      if ((rows + q) % IDX == 0) cum.push_back(b + nb);
      lens.push_back(l[q]);
      nb += 4ULL * l[q];
    }
    return nb;
  }
  // byte stream [b0, b0 + nb) <-> a contiguous buffer (async copies, page by page)
  void copy_out(const void* dev, unsigned long long b0, unsigned long long nb, hipStream_t stream) {
    const char* s = (const char*)dev;
    while (nb) {
      const size_t pg = b0 / page_bytes, off = b0 % page_bytes, k = std::min<unsigned long long>(nb, page_bytes - off);
      if (pg >= pages.size() || !pages[pg]) throw std::runtime_error("host frontier: copy-out past the reserved pages");
      HIPCHK(hipMemcpyAsync((char*)pages[pg] + off, s, k, hipMemcpyDeviceToHost, stream));
      s += k;
      b0 += k;
      nb -= k;
    }
  }
  void copy_in(unsigned long long b0, unsigned long long nb, void* dev, hipStream_t stream) const {
    char* d = (char*)dev;
    while (nb) {
      const size_t pg = b0 / page_bytes, off = b0 % page_bytes, k = std::min<unsigned long long>(nb, page_bytes - off);
      if (pg >= pages.size() || !pages[pg]) throw std::runtime_error("host frontier: rows already recycled");
      HIPCHK(hipMemcpyAsync(d, (char*)pages[pg] + off, k, hipMemcpyHostToDevice, stream));
      d += k;
      b0 += k;
      nb -= k;
    }
  }
  void read_host(unsigned long long b0, unsigned long long nb, void* out) const {
    char* d = (char*)out;
    while (nb) {
      const size_t pg = b0 / page_bytes, off = b0 % page_bytes, k = std::min<unsigned long long>(nb, page_bytes - off);
      memcpy(d, (const char*)pages[pg] + off, k);
      d += k;
      b0 += k;
      nb -= k;
    }
  }
  void write_host(const void* src, unsigned long long nb) {  // at the end of the stream (pages reserved)
    const char* s = (const char*)src;
    unsigned long long b0 = bytes;
    while (nb) {
      const size_t pg = b0 / page_bytes, off = b0 % page_bytes, k = std::min<unsigned long long>(nb, page_bytes - off);
      memcpy((char*)pages[pg] + off, s, k);
      s += k;
      b0 += k;
      nb -= k;
    }
  }
  // append n compact rows (word counts l) whose bytes are in dev (dev_bytes
  // long: the rows' bytes are checked against it), async on stream
  void append_dev(const uint8_t* l, unsigned long long n, const void* dev, size_t dev_bytes, hipStream_t stream,
                  HostPagePool& pool) {
    unsigned long long nb = 0;
    for (unsigned long long q = 0; q < n; q++) nb += 4ULL * l[q];
    if (nb > dev_bytes)
      throw std::runtime_error("host frontier: " + std::to_string(n) + " compact rows of " + std::to_string(nb) +
                               " B exceed their " + std::to_string(dev_bytes) + " B pack buffer");
    reserve_bytes(nb, pool);
    add_rows(l, n);
    copy_out(dev, bytes, nb, stream);
    bytes += nb;
    rows += n;
  }
  // append fixed-stride host rows (hdr_words + nmsg words each), compacting them on the host
  void append_fixed_host(const uint32_t* fixed, unsigned long long n, size_t W, int hdr_words, HostPagePool& pool) {
    std::vector<uint8_t> l(n);
    unsigned long long nb = 0;
    for (unsigned long long q = 0; q < n; q++) {
      l[q] = (uint8_t)(hdr_words + (fixed[q * W] & 0xFFu));
      nb += 4ULL * l[q];
    }
    reserve_bytes(nb, pool);
    add_rows(l.data(), n);
    for (unsigned long long q = 0; q < n; q++) {
      write_host(fixed + q * W, 4ULL * l[q]);
      bytes += 4ULL * l[q];
    }
    rows += n;
  }
  // rows [r0, r0 + n) as fixed-stride rows (host side; checkpoints)
  void read_fixed_host(unsigned long long r0, unsigned long long n, uint32_t* out) const {
    const size_t W = row_bytes / 4;
    unsigned long long b = byte_of(r0);
    for (unsigned long long q = 0; q < n; q++) {
      const unsigned L = lens[r0 + q];
      memset(out + q * W, 0, row_bytes);
      read_host(b, 4ULL * L, out + q * W);
      b += 4ULL * L;
    }
  }
  // give back the pages whose bytes all lie below row r
  void recycle_below(unsigned long long r, HostPagePool& pool) {
    const unsigned long long b = byte_of(std::min(r, rows));
    for (size_t pg = 0; pg < pages.size() && (pg + 1) * page_bytes <= b; pg++) {
      pool.put(pages[pg]);
      pages[pg] = nullptr;
    }
  }
  void clear(HostPagePool& pool) {
    for (void* p : pages) pool.put(p);
    pages.clear();
    lens.clear();
    cum.clear();
    rows = bytes = 0;
  }
};
// Synchronous compact-row transfers between a host level and fixed-stride
// device rows (the sharded search's per-shard host frontier; the single-GPU
// search pipelines the same kernels over its copy streams).
struct HostRowsIO {
  DevBuf pack, l32, l8, off, scan, stage, il32, il8, ioff, iscan, flag;
  static size_t atleast(size_t b) { return b < 16 ? 16 : b; }
  // rows [r0, r0 + n) of h -> fixed rows at dev, in stream order on st
  void load(const HostLevel& h, unsigned long long r0, unsigned long long n, uint32_t* dev, size_t W, hipStream_t st) {
    if (!n) return;
    stage.ensure(atleast(n * W * 4));
    il32.ensure(atleast(n * 4));
    il8.ensure(atleast(n));
    ioff.ensure(atleast(n * 4));
    iscan.ensure(atleast(rmc::scan_temp_bytes(n)));
    const unsigned long long b0 = h.byte_of(r0), b1 = h.byte_of(r0 + n);
    h.copy_in(b0, b1 - b0, stage.p, st);
    HIPCHK(hipMemcpyAsync(il8.p, h.lens.data() + r0, n, hipMemcpyHostToDevice, st));
    rmc::launch_widen_lens(il8.as<uint8_t>(), n, il32.as<uint32_t>(), st);
    rmc::launch_scan(iscan.p, iscan.bytes, il32.as<uint32_t>(), ioff.as<uint32_t>(), n, st);
    rmc::launch_unpack_rows(stage.as<uint32_t>(), n, (int)W, ioff.as<uint32_t>(), il32.as<uint32_t>(), dev, st);
    HIPCHK(hipGetLastError());
  }
  // n fixed rows at dev -> appended to h; returns once they are in the pages.
  // In slices of at most 2^24 rows and 256 MiB of pack buffer (the pack
  // offsets are 32-bit words, and a whole level would need a second copy of
  // itself in HBM just when HBM is short: ADVICE r04).  A row whose header
  // claims more words than W (never written) ends the check with status 3.
  static unsigned long long slice_rows(size_t W) {
    return std::max<unsigned long long>(1, std::min<unsigned long long>(1ULL << 24, (256ULL << 20) / (W * 4)));
  }
  void store(HostLevel& h, const uint32_t* dev, unsigned long long n, size_t W, int hdr_words, hipStream_t st,
             HostPagePool& pool) {
    if (!n) return;
    const unsigned long long S = std::min<unsigned long long>(n, slice_rows(W));
    pack.ensure(atleast(S * W * 4));
    l32.ensure(atleast(S * 4));
    l8.ensure(atleast(S));
    off.ensure(atleast(S * 4));
    scan.ensure(atleast(rmc::scan_temp_bytes(S)));
    flag.ensure(16);
    HIPCHK(hipMemsetAsync(flag.p, 0, 4, st));
    std::vector<uint8_t> lens;
    for (unsigned long long r = 0; r < n; r += S) {
      const unsigned long long k = std::min(S, n - r);
      const uint32_t* rows = dev + r * W;
      rmc::launch_row_words(rows, k, (int)W, hdr_words, max_words(W), l32.as<uint32_t>(), l8.as<uint8_t>(),
                            flag.as<unsigned>(), st);
      rmc::launch_scan(scan.p, scan.bytes, l32.as<uint32_t>(), off.as<uint32_t>(), k, st);
      rmc::launch_pack_rows(rows, k, (int)W, off.as<uint32_t>(), l32.as<uint32_t>(), pack.as<uint32_t>(), st);
      HIPCHK(hipGetLastError());
      lens.resize(k);
      unsigned f = 0;
      HIPCHK(hipMemcpyAsync(lens.data(), l8.p, k, hipMemcpyDeviceToHost, st));
      HIPCHK(hipMemcpyAsync(&f, flag.p, 4, hipMemcpyDeviceToHost, st));
      HIPCHK(hipStreamSynchronize(st));
      if (f) throw RowCapacity("capacity overflow: a row's message count exceeds the row width (a row never written)");
      h.append_dev(lens.data(), k, pack.p, pack.bytes, st, pool);
      HIPCHK(hipStreamSynchronize(st));
    }
  }
  // the pack bound (test hook RMC_HF_ROW_MAX_WORDS lowers it to exercise the
  // capacity report)
  static int max_words(size_t W) {
    if (const char* e = getenv("RMC_HF_ROW_MAX_WORDS")) return std::min<int>((int)W, atoi(e));
    return (int)W;
  }
  void release() {
    for (DevBuf* b : {&pack, &l32, &l8, &off, &scan, &stage, &il32, &il8, &ioff, &iscan, &flag}) b->release();
  }
};

// Host memory the host frontier may pin: RMC_HOST_FRONTIER_GIB, or 80% of
// MemAvailable capped at 200 GiB (a shared host must keep room for others).
size_t host_frontier_limit();
double hf_hbm_fraction();

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
