// rmc_sharded.cpp — the fingerprint-sharded BFS over W shards:
// one shard per GPU, one process per GPU, RCCL over xGMI; or W logical shards
// driven by one process on one GPU (the same protocol with device copies as
// the transport — SURVEY §4 item 5, "multi-GPU without a cluster").
//
// Exactness.  TLC keeps, per fingerprint, the successor first in its BFS
// exploration order (parent position in the level, then the action's ordinal
// in Next).  A level's states are distributed BLOCK-CYCLICALLY by their global
// TLC position g: shard (g / CH) mod W holds g at local index
// (g / (W·CH))·CH + g mod CH.  Round c of a level has every shard expand its
// c-th local block, which together are the contiguous global range
// [c·W·CH, (c+1)·W·CH): rounds are increasing in TLC order, so a fingerprint
// won in an earlier round can never be displaced by a later one, and within a
// round the owner's atomicMin on (parent gid, ordinal) picks TLC's winner.
// The winners of a round are, in TLC order, the generators' winners in shard
// order; they are written to their global positions (next level's block-
// cyclic layout) by an all-to-all of state rows.
//
// Per round: expand (fp + key per candidate; the candidates whose fp this
// shard owns are inserted right there, as the single-GPU search does) ->
// bucket the others by owner -> all-to-all (fp, key) 16 B -> owners insert,
// then mark -> reverse all-to-all of 1-byte win flags -> per-parent winner
// ranks (local-owner outcomes read from the shard's own table), scan ->
// materialize (straight into the next frontier when every winner stays with
// its generator, else into staging) -> all-to-all of rows + trace records.
// At W = 1 that is the single-GPU search plus the protocol's host round trips.
#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstring>
#include <map>
#include <set>
#include <memory>
#include <mutex>
#include <string>
#include <vector>
#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <signal.h>
#include <cerrno>
#include <unistd.h>
#include <rccl/rccl.h>
#include "rmc_internal.h"
#include "rmc_fpset.h"

using namespace rmc;

namespace rmcx {

// -------------------------------------------------------------- transports
struct Xfer {
  int src, dst;        // global shard ids
  const void* sbuf;    // valid on the sender
  void* rbuf;          // valid on the receiver
  size_t bytes;
};

struct Comm {
  int world = 1;
  std::vector<int> local;  // global ids of the shards this process drives
  // in-process multi-GPU (rmc_check_multi): the threads that share this
  // process's host memory, and those that share this thread's device
  int host_share = 1, dev_share = 1;
  virtual ~Comm() {}
  // in[i] = the k values of local shard local[i]; out = world*k values by shard id
  virtual void allgather(const std::vector<std::vector<uint64_t>>& in, std::vector<uint64_t>& out, int k) = 0;
  // every transfer this process takes part in, in one global order
  virtual void alltoallv(const std::vector<Xfer>& x) = 0;
  hipStream_t stream = nullptr;
};

// All W shards in this process, on one GPU: transfers are device copies on the
// shared stream (stream order is the synchronisation).
struct LocalComm : Comm {
  LocalComm(int W, hipStream_t s) {
    world = W;
    for (int i = 0; i < W; i++) local.push_back(i);
    stream = s;
  }
  void allgather(const std::vector<std::vector<uint64_t>>& in, std::vector<uint64_t>& out, int k) override {
    out.assign((size_t)world * k, 0);
    for (int i = 0; i < world; i++)
      for (int j = 0; j < k; j++) out[(size_t)i * k + j] = in[i][j];
  }
  // the step's transfers in one batched copy kernel (k_multi_copy): a
  // hipMemcpyAsync each cost ~15,000 launches per check at W = 8
  std::vector<CopyDesc> desc;
  DevBuf ddesc;
  CopyDesc* hdesc = nullptr;  // pinned staging of the descriptors
  size_t hcap = 0;
  hipEvent_t hdone = nullptr;  // the last descriptor upload has been read
  ~LocalComm() override {
    if (hdone) (void)hipEventSynchronize(hdone), (void)hipEventDestroy(hdone);
    if (hdesc) (void)hipHostFree(hdesc);
  }
  void alltoallv(const std::vector<Xfer>& x) override {
    desc.clear();
    unsigned long long mx = 0;
    for (auto& t : x)
      if (t.bytes) {
        desc.push_back({t.sbuf, t.rbuf, (unsigned long long)t.bytes});
        mx = std::max<unsigned long long>(mx, t.bytes);
      }
    if (desc.empty()) return;
    if (desc.size() == 1) {
      HIPCHK(hipMemcpyAsync(desc[0].dst, desc[0].src, desc[0].bytes, hipMemcpyDeviceToDevice, stream));
      return;
    }
    if (!hdone) HIPCHK(hipEventCreateWithFlags(&hdone, hipEventDisableTiming));
    else HIPCHK(hipEventSynchronize(hdone));  // the staging is free again
    if (hcap < desc.size()) {
      if (hdesc) HIPCHK(hipHostFree(hdesc));
      hcap = std::max<size_t>(desc.size(), 1024);
      HIPCHK(hipHostMalloc((void**)&hdesc, hcap * sizeof(CopyDesc), hipHostMallocDefault));
    }
    memcpy(hdesc, desc.data(), desc.size() * sizeof(CopyDesc));
    ddesc.ensure(hcap * sizeof(CopyDesc));
    HIPCHK(hipMemcpyAsync(ddesc.p, hdesc, desc.size() * sizeof(CopyDesc), hipMemcpyHostToDevice, stream));
    HIPCHK(hipEventRecord(hdone, stream));
    launch_multi_copy(ddesc.as<CopyDesc>(), (int)desc.size(), mx, stream);
    HIPCHK(hipGetLastError());
  }
};

#define NCCLCHK(x)                                                                                   \
  do {                                                                                               \
    ncclResult_t r_ = (x);                                                                           \
    if (r_ != ncclSuccess) throw std::runtime_error(std::string("RCCL error: ") + ncclGetErrorString(r_) + " at " #x); \
  } while (0)

// One shard per process (one process per GPU); RCCL point-to-point over xGMI.
struct RcclComm : Comm {
  ncclComm_t comm = nullptr;
  int rank = 0;
  bool owns = true;  // false: a communicator of an in-process group (rmc_check_multi owns it)
  // in-process group: set when another shard's thread failed -- no collective
  // is started after that, and one blocked in a stream sync is released by
  // rmc_check_multi aborting the communicators
  const std::atomic<bool>* aborted = nullptr;
  void live() const {
    if (aborted && aborted->load()) throw std::runtime_error("in-process multi-GPU check: another shard's thread failed");
  }
  DevBuf gbuf;
  RcclComm(int r, int W, const ncclUniqueId& id, hipStream_t s) {
    rank = r;
    world = W;
    local = {r};
    stream = s;
    NCCLCHK(ncclCommInitRank(&comm, W, id, r));
  }
  RcclComm(int r, int W, ncclComm_t c, hipStream_t s) : comm(c), rank(r), owns(false) {
    world = W;
    local = {r};
    stream = s;
  }
  ~RcclComm() override {
    if (comm && owns) (void)ncclCommDestroy(comm);
  }
  void allgather(const std::vector<std::vector<uint64_t>>& in, std::vector<uint64_t>& out, int k) override {
    live();
    gbuf.ensure((size_t)world * k * 8 + (size_t)k * 8);
    uint64_t* d = gbuf.as<uint64_t>();
    uint64_t* mine = d + (size_t)world * k;
    HIPCHK(hipMemcpyAsync(mine, in[0].data(), (size_t)k * 8, hipMemcpyHostToDevice, stream));
    NCCLCHK(ncclAllGather(mine, d, (size_t)k, ncclUint64, comm, stream));
    out.assign((size_t)world * k, 0);
    HIPCHK(hipMemcpyAsync(out.data(), d, (size_t)world * k * 8, hipMemcpyDeviceToHost, stream));
    const hipError_t e = hipStreamSynchronize(stream);
    live();
    HIPCHK(e);
  }
  void alltoallv(const std::vector<Xfer>& x) override {
    live();
    NCCLCHK(ncclGroupStart());
    for (auto& t : x) {
      if (!t.bytes) continue;
      if (t.src == rank && t.dst == rank) {
        HIPCHK(hipMemcpyAsync(t.rbuf, t.sbuf, t.bytes, hipMemcpyDeviceToDevice, stream));
      } else if (t.src == rank) {
        NCCLCHK(ncclSend(t.sbuf, t.bytes, ncclChar, t.dst, comm, stream));
      } else if (t.dst == rank) {
        NCCLCHK(ncclRecv(t.rbuf, t.bytes, ncclChar, t.src, comm, stream));
      }
    }
    NCCLCHK(ncclGroupEnd());
  }
};

// One shard per process, host shared memory as the transport: the same
// multi-process protocol as RcclComm (rank-local shards, allgathered counts,
// point-to-point transfers) where RCCL cannot run, e.g. several processes on
// one GPU (RCCL refuses two ranks per device).  Transfers are staged through
// per-(source, destination) slots of a POSIX shared-memory segment, in rounds
// of the slot size, with a process-shared barrier between the write and read
// halves of every round.
struct ShmComm : Comm {
  struct Hdr {
    int ready;
    int count;  // arrivals at the current barrier
    int sense;  // flips when the last rank arrives
    int owner;  // rank 0's pid (a segment left by a dead run has a dead owner)
  };
  static constexpr size_t SLOT = 8u << 20;   // bytes per (src, dst) slot and round
  static constexpr int GATHER_MAX = 64;      // values per rank in one allgather
  std::string name;
  int rank = 0;
  size_t bytes = 0;
  unsigned char* base = nullptr;
  Hdr* hdr() { return reinterpret_cast<Hdr*>(base); }
  uint64_t* gather() { return reinterpret_cast<uint64_t*>(base + 256); }
  unsigned char* slot(int src, int dst) {
    return base + 256 + (size_t)world * GATHER_MAX * 8 + ((size_t)src * world + dst) * SLOT;
  }
  ShmComm(int r, int W, const std::string& nm, hipStream_t s) : name(nm), rank(r) {
    world = W;
    local = {r};
    stream = s;
    bytes = 256 + (size_t)W * GATHER_MAX * 8 + (size_t)W * W * SLOT;
    if (rank == 0) {
      // a fresh segment: a stale one of the same name (a crashed run) is
      // unlinked first; its space is allocated now, so a small /dev/shm is a
      // clean error here rather than a SIGBUS on first write
      (void)shm_unlink(name.c_str());
      int fd = shm_open(name.c_str(), O_CREAT | O_EXCL | O_RDWR, 0600);
      if (fd < 0) throw std::runtime_error("shm_open " + name + " failed: " + strerror(errno));
      int e = posix_fallocate(fd, 0, (off_t)bytes);
      if (e != 0) {
        close(fd);
        shm_unlink(name.c_str());
        throw std::runtime_error("shm transport: cannot allocate " + std::to_string(bytes >> 20) + " MiB in /dev/shm: " +
                                 strerror(e));
      }
      void* p = mmap(nullptr, bytes, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
      close(fd);
      if (p == MAP_FAILED) throw std::runtime_error("mmap of the shm segment failed");
      base = (unsigned char*)p;
      __atomic_store_n(&hdr()->count, 0, __ATOMIC_RELAXED);
      __atomic_store_n(&hdr()->sense, 0, __ATOMIC_RELAXED);
      __atomic_store_n(&hdr()->owner, (int)getpid(), __ATOMIC_RELAXED);
      __atomic_store_n(&hdr()->ready, 1, __ATOMIC_RELEASE);
    } else {
      // attach to rank 0's segment: wait until it exists, is initialised and
      // is owned by a live process (a dead run's leftover is not joined)
      for (int t = 0;; t++) {
        if (t > 600000) throw std::runtime_error("shm transport: rank 0 never initialised " + name);
        int fd = shm_open(name.c_str(), O_RDWR, 0600);
        if (fd >= 0) {
          struct stat st;
          if (fstat(fd, &st) == 0 && (size_t)st.st_size >= bytes) {
            void* p = mmap(nullptr, bytes, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
            if (p != MAP_FAILED) {
              Hdr* h = reinterpret_cast<Hdr*>(p);
              const int own = __atomic_load_n(&h->ready, __ATOMIC_ACQUIRE) ? __atomic_load_n(&h->owner, __ATOMIC_RELAXED) : 0;
              if (own > 0 && (kill(own, 0) == 0 || errno == EPERM)) {
                close(fd);
                base = (unsigned char*)p;
                break;
              }
              munmap(p, bytes);
            }
          }
          close(fd);
        }
        usleep(100);
      }
    }
    barrier();
    // every rank has mapped the segment: its name can go now (the mappings
    // stay valid), so a later check under the same name can never attach to
    // this one while rank 0 is still tearing it down
    if (rank == 0) shm_unlink(name.c_str());
  }
  ~ShmComm() override {
    if (!base) return;
    try { barrier(); } catch (...) {}
    munmap(base, bytes);
  }
  // sense-reversing barrier in the segment; a rank that waits 120 s (a peer
  // failed or died) throws instead of hanging
  int my_sense = 0;
  bool dead = false;
  void barrier() {
    if (dead) return;
    my_sense ^= 1;
    if (__atomic_add_fetch(&hdr()->count, 1, __ATOMIC_ACQ_REL) == world) {
      __atomic_store_n(&hdr()->count, 0, __ATOMIC_RELAXED);
      __atomic_store_n(&hdr()->sense, my_sense, __ATOMIC_RELEASE);
      return;
    }
    auto t0 = std::chrono::steady_clock::now();
    for (long k = 0; __atomic_load_n(&hdr()->sense, __ATOMIC_ACQUIRE) != my_sense; k++) {
      if (k > 1000) usleep(50);
      if ((k & 1023) == 0 && std::chrono::steady_clock::now() - t0 > std::chrono::seconds(120)) {
        dead = true;
        throw std::runtime_error("shm transport: a peer rank did not arrive within 120 s");
      }
    }
  }
  void allgather(const std::vector<std::vector<uint64_t>>& in, std::vector<uint64_t>& out, int k) override {
    if (k > GATHER_MAX) throw std::runtime_error("shm transport: allgather too wide");
    memcpy(gather() + (size_t)rank * k, in[0].data(), (size_t)k * 8);
    barrier();
    out.assign(gather(), gather() + (size_t)world * k);
    barrier();
  }
  // x is the round's global transfer list, identical on every rank (the
  // protocol builds it from allgathered counts), so every rank walks the same
  // transfers and rounds: each transfer goes through its pair's slot in
  // SLOT-sized pieces.  Copies go on the check's stream and are waited for
  // before each barrier (a pageable host-to-device copy may return before its
  // DMA lands, and the stream does not order with the null stream).
  void alltoallv(const std::vector<Xfer>& x) override {
    HIPCHK(hipStreamSynchronize(stream));  // the send buffers are ready
    for (auto& t : x) {
      if (!t.bytes || (t.src == t.dst)) {
        if (t.bytes && t.src == rank)
          HIPCHK(hipMemcpyAsync(t.rbuf, t.sbuf, t.bytes, hipMemcpyDeviceToDevice, stream));
        continue;
      }
      for (size_t off = 0; off < t.bytes; off += SLOT) {
        const size_t n = std::min(SLOT, t.bytes - off);
        if (t.src == rank) {
          HIPCHK(hipMemcpyAsync(slot(t.src, t.dst), (const char*)t.sbuf + off, n, hipMemcpyDeviceToHost, stream));
          HIPCHK(hipStreamSynchronize(stream));
        }
        barrier();
        if (t.dst == rank) {
          HIPCHK(hipMemcpyAsync((char*)t.rbuf + off, slot(t.src, t.dst), n, hipMemcpyHostToDevice, stream));
          HIPCHK(hipStreamSynchronize(stream));
        }
        barrier();
      }
    }
    HIPCHK(hipStreamSynchronize(stream));
  }
};

// The W host threads of one in-process multi-GPU check (rmc_check_multi):
// a generation barrier that a failing thread can break (abort), the allgather
// area, and each exchange step's buffer pointers by transfer index.
struct ThreadGroup {
  int W = 1;
  std::vector<int> dev;  // device of each shard
  std::mutex mu;
  std::condition_variable cv;
  int count = 0;
  unsigned long long gen = 0;
  std::atomic<bool> aborted{false};
  std::vector<uint64_t> gather;
  std::vector<const void*> sp;  // transfer k's source (set by its sender)
  std::vector<void*> rp;        // transfer k's destination (set by its receiver)
  void barrier() {
    std::unique_lock<std::mutex> lk(mu);
    if (aborted) throw std::runtime_error("in-process multi-GPU check: another shard's thread failed");
    const unsigned long long g = gen;
    if (++count == W) {
      count = 0;
      gen++;
      cv.notify_all();
      return;
    }
    cv.wait(lk, [&] { return gen != g || aborted; });
    if (gen == g) throw std::runtime_error("in-process multi-GPU check: another shard's thread failed");
  }
  void abort() {
    std::lock_guard<std::mutex> lk(mu);
    aborted = true;
    cv.notify_all();
  }
};

// One shard per host thread of this process, peer device copies as the
// transport (RMC_XPORT_P2P): a receiver pulls each transfer from its sender's
// buffer on its own stream (hipMemcpyPeerAsync over xGMI across devices, a
// device copy when both shards share one -- which is how the one-GPU box
// runs the in-process driver with several threads).  Like ShmComm, every rank
// builds the same global transfer list, so the k-th entry is the same
// transfer everywhere; the pointers are published through the group.
struct ThreadComm : Comm {
  ThreadGroup* g;
  int rank;
  ThreadComm(ThreadGroup* grp, int r, hipStream_t s) : g(grp), rank(r) {
    world = grp->W;
    local = {r};
    stream = s;
  }
  void allgather(const std::vector<std::vector<uint64_t>>& in, std::vector<uint64_t>& out, int k) override {
    {
      std::lock_guard<std::mutex> lk(g->mu);
      if (g->gather.size() < (size_t)world * k) g->gather.resize((size_t)world * k);
      for (int j = 0; j < k; j++) g->gather[(size_t)rank * k + j] = in[0][j];
    }
    g->barrier();
    out.assign(g->gather.begin(), g->gather.begin() + (size_t)world * k);
    g->barrier();  // nobody writes the next gather before every rank has read this one
  }
  void alltoallv(const std::vector<Xfer>& x) override {
    HIPCHK(hipStreamSynchronize(stream));  // this rank's send buffers are complete
    {
      std::lock_guard<std::mutex> lk(g->mu);
      if (g->sp.size() < x.size()) {
        g->sp.resize(x.size());
        g->rp.resize(x.size());
      }
      for (size_t k = 0; k < x.size(); k++) {
        if (x[k].src == rank) g->sp[k] = x[k].sbuf;
        if (x[k].dst == rank) g->rp[k] = x[k].rbuf;
      }
    }
    g->barrier();
    for (size_t k = 0; k < x.size(); k++) {
      const Xfer& t = x[k];
      if (t.dst != rank || !t.bytes) continue;
      if (g->dev[t.src] == g->dev[t.dst])
        HIPCHK(hipMemcpyAsync(g->rp[k], g->sp[k], t.bytes, hipMemcpyDeviceToDevice, stream));
      else
        HIPCHK(hipMemcpyPeerAsync(g->rp[k], g->dev[t.dst], g->sp[k], g->dev[t.src], t.bytes, stream));
    }
    HIPCHK(hipStreamSynchronize(stream));
    g->barrier();  // every pull has landed: senders may reuse their buffers
  }
};

// ---------------------------------------------------------- shard buffers
struct ShardBufs {
  DevBuf table, table2, cfp, cval, cob, cwin, poff, pn, pwin, ppos, counters, stbuf, scantmp;
  DevBuf send, perm, recv, rslot, rflag, sflag, stage, stp, stb, small, bcnt, boff, btmp;
  DevBuf mpc;   // k_materialize's piece map (logical shards)
  DevBuf xmap;  // logical shards: record destinations (k_bucket), flag destinations + recv segments (k_mark_recv)
  GrowBuf fa, fb, trp, trb;  // frontiers and trace records grow in place
  void release() {
    for (DevBuf* b : {&table, &table2, &cfp, &cval, &cob, &cwin, &poff, &pn, &pwin, &ppos, &counters, &stbuf,
                      &scantmp, &send, &perm, &recv, &rslot, &rflag, &sflag, &stage, &stp, &stb, &small, &bcnt,
                      &boff, &btmp, &mpc, &xmap})
      b->release();
    for (GrowBuf* b : {&fa, &fb, &trp, &trb}) b->release();
  }
};
static std::mutex g_shard_mu;
static std::map<std::pair<int, int>, ShardBufs*> g_shard_bufs;
static ShardBufs& shard_bufs(int slot) {
  int dev = 0;
  HIPCHK(hipGetDevice(&dev));
  std::lock_guard<std::mutex> lk(g_shard_mu);
  ShardBufs*& b = g_shard_bufs[{dev, slot}];
  if (!b) b = new ShardBufs();
  return *b;
}
void release_shard_buffers() {
  std::lock_guard<std::mutex> lk(g_shard_mu);
  int cur = 0;
  (void)hipGetDevice(&cur);
  for (auto& kv : g_shard_bufs)
    if (hipSetDevice(kv.first.first) == hipSuccess) kv.second->release();
  (void)hipSetDevice(cur);
}
// Cached shard buffers are sized for the partition that grew them: a check
// with another shard count on this device starts from nothing (a W = 2
// check's shard 0 holds half of every level, twice what a W = 4 shard needs).
// The in-process multi-GPU driver settles this for every device before its
// threads start, so no thread releases buffers another one is using.
static std::mutex g_world_mu;
static std::map<int, int> g_last_world;
static void settle_shard_world(int W) {
  int dev = 0;
  HIPCHK(hipGetDevice(&dev));
  bool rel = false;
  {
    std::lock_guard<std::mutex> lk(g_world_mu);
    int& lw = g_last_world[dev];
    rel = lw && lw != W;
    lw = W;
  }
  if (rel) release_shard_buffers();
}

struct Shard {
  int id = 0;
  ShardBufs* B = nullptr;
  unsigned long long slots = 0, entries = 0;  // fingerprint set of this owner: slots, entries
  unsigned long long expand_slots = 0;        // its size when this round's k_expand inserted
  uint32_t *cur = nullptr, *nxt = nullptr;
  unsigned long long fcap = 0;       // states per frontier buffer
  unsigned long long ncur = 0;       // local states of the current level
  unsigned long long next_fill = 0;  // local states of the next level written so far
  unsigned long long trcap = 0;      // trace records
  std::vector<unsigned long long> tr_base;  // local trace index of each level's first local state (by depth)
  unsigned long long ncand = 0, nrecv = 0, nwin = 0, n = 0;
  std::vector<uint64_t> seg_off, rseg_off;  // send segments by owner / recv segments by source
  DevStatus hst;
  // per-shard host frontier (rmc_options.host_frontier): the shard's current
  // and next level live in compact host pages; each round's block of parents
  // is unpacked into win_in, the round's new local rows (a contiguous local
  // range [fill0, next_fill)) land in win_out and are packed out after it
  bool hf = false;
  HostLevel hcur, hnxt;
  HostRowsIO io;
  DevBuf win_in, win_out;
  unsigned long long fill0 = 0;
};

static unsigned long long local_count(unsigned long long P, int W, unsigned long long CH, int r) {
  unsigned long long full = P / (W * CH), rem = P - full * W * CH;
  long long part = (long long)rem - (long long)r * (long long)CH;
  part = part < 0 ? 0 : (part > (long long)CH ? (long long)CH : part);
  return full * CH + (unsigned long long)part;
}

// Room for need_entries (OutOfDeviceMemory ends the check with status 3): at
// <= 0.5 load while the shard's set is at most 1/W of 32 GiB, <= 0.75 beyond --
// the single-GPU search's thresholds (rmc_engine.cpp over_load) for the W
// shards' sets together, so a shard's set is 1/W of the single search's and
// not twice that (the needs are upper bounds: every candidate counted new).
static void table_grow(Shard& s, unsigned long long need_entries, hipStream_t stream, int W) {
  const unsigned long long small = (32ULL << 30) / (unsigned long long)W;
  auto fits = [&](unsigned long long sl) {
    return sl * 16 <= small ? need_entries * 2 <= sl : need_entries * 4 <= sl * 3;
  };
  if (fits(s.slots)) return;
  unsigned long long nslots = s.slots;
  while (!fits(nslots)) nslots <<= 1;
  DevBuf& nt = s.B->table2;
  nt.ensure(nslots * 16);
  HIPCHK(hipMemsetAsync(nt.p, 0xFF, nslots * 16, stream));
  launch_rehash(s.B->table.as<unsigned long long>(), s.slots, nt.as<unsigned long long>(), nslots - 1,
                s.B->stbuf.as<DevStatus>(), stream);
  HIPCHK(hipGetLastError());
  HIPCHK(hipStreamSynchronize(stream));
  std::swap(s.B->table.p, nt.p);
  std::swap(s.B->table.bytes, nt.bytes);
  s.slots = nslots;
  if (nt.bytes >= (1ULL << 30)) nt.release();
}

// grow a frontier / trace buffer keeping its contents (stream-ordered)
static void grow_keep(GrowBuf& b, size_t need, size_t /*keep*/, hipStream_t stream) {
  if (b.p && b.bytes >= need) return;
  HIPCHK(hipStreamSynchronize(stream));
  b.ensure(need);
}

// Returns 1 when the check must be re-run with a larger message capacity.
static int check_sharded_impl(rmc_model* m, const rmc_options* opt, Comm& comm, rmc_result* res) {
  auto t0 = std::chrono::steady_clock::now();
  Model& M = m->M;
  if (opt->deadlock_check) throw std::runtime_error("deadlock checking is not supported; run with -deadlock (README.md:6)");
  if (opt->fp_bits && opt->fp_bits != 64) throw std::runtime_error("fp_bits 128 is offered by the single-GPU search (rmc_check) only");
  if ((opt->checkpoint_dir && *opt->checkpoint_dir) || (opt->recover_dir && *opt->recover_dir))
    throw std::runtime_error("checkpoint / recover are offered by the single-GPU search (rmc_check) only");
  uint32_t kmax = opt->msg_cap_K ? opt->msg_cap_K : (m->kmax_user ? m->kmax_user : model_kmax(m));
  if (kmax > 120) kmax = 120;
  finalize_model(m, kmax);
  HIPCHK(upload_model(M));
  hipStream_t stream = comm.stream;
  const int W = comm.world;
  const size_t WD = (size_t)M.words;
  res->state_bytes = (uint32_t)(WD * 4);
  const int maxsucc = max_successors(M);
  const unsigned long long CH = opt->chunk_parents ? opt->chunk_parents : (1ULL << 22);
  const unsigned long long cand_cap = CH * (unsigned long long)std::min(maxsucc, 256);
  const int NL = (int)comm.local.size();
  if (W > 64) throw std::runtime_error("at most 64 shards");
  settle_shard_world(W);

  std::vector<Shard> sh(NL);
  // every shard on this device, driven by this process (logical shards)
  const bool same_device = dynamic_cast<LocalComm*>(&comm) != nullptr;
  // the per-shard host frontier: one pinned-page pool for this process's shards
  HostPagePool pool;
  pool.page_bytes = std::max<size_t>(WD * 4, 256ULL << 20);
  if (const char* e = getenv("RMC_HOST_PAGE_ROWS")) pool.page_bytes = std::max<long long>(1, atoll(e)) * WD * 4;
  pool.limit = host_frontier_limit() / (size_t)std::max(1, comm.host_share);  // threads of one process split it
  struct PagesGuard {
    std::vector<Shard>& sh;
    HostPagePool& pool;
    ~PagesGuard() {
      for (Shard& s : sh) { s.hcur.clear(pool); s.hnxt.clear(pool); }
    }
  } pages_guard{sh, pool};
  const int hdr_words = 1 + 4 * M.N;
  size_t hbm_total = 0;
  {
    int dev = 0;
    if (hipGetDevice(&dev) == hipSuccess) (void)hipDeviceTotalMem(&hbm_total, dev);
  }
  // the model's size hints are whole-search totals (the single-GPU search
  // keeps them so too): a shard starts at its 1/W share
  auto share = [&](unsigned long long total) { return total / (unsigned long long)W; };
  unsigned long long hint_slots_1 = 1;
  while (hint_slots_1 < share(m->hint_slots)) hint_slots_1 <<= 1;
  for (int i = 0; i < NL; i++) {
    Shard& s = sh[i];
    s.id = comm.local[i];
    s.B = &shard_bufs(s.id);  // by shard id: threads sharing one device keep apart
    ShardBufs& B = *s.B;
    s.slots = opt->hash_slots ? opt->hash_slots : std::max(1ULL << 22, hint_slots_1);
    if (s.slots & (s.slots - 1)) throw std::runtime_error("hash_slots must be a power of two");
    B.table.ensure(s.slots * 16);
    HIPCHK(hipMemsetAsync(B.table.p, 0xFF, s.slots * 16, stream));
    s.fcap = opt->frontier_cap ? opt->frontier_cap : std::max(1ULL << 20, share(m->hint_fcap));
    B.fa.ensure(s.fcap * WD * 4);
    B.fb.ensure(s.fcap * WD * 4);
    s.cur = B.fa.as<uint32_t>();
    s.nxt = B.fb.as<uint32_t>();
    B.cfp.ensure(cand_cap * 8);
    B.cval.ensure(cand_cap * 8);
    B.cob.ensure(cand_cap * 4);
    B.cwin.ensure(cand_cap * 2);
    B.perm.ensure(cand_cap * 4);
    B.poff.ensure(CH * 4);
    B.pn.ensure(CH * 4);
    B.pwin.ensure(CH * 4);
    B.ppos.ensure(CH * 4);
    B.counters.ensure(64);
    B.stbuf.ensure(sizeof(DevStatus));
    size_t stb = scan_temp_bytes(CH);
    B.scantmp.ensure(stb ? stb : 16);
    B.small.ensure(4096);
    s.trcap = std::max(s.fcap * 4, share(m->hint_trcap));
    B.trp.ensure(s.trcap * 8);
    B.trb.ensure(s.trcap * 2);
    s.hst.err_key = s.hst.inv_err_key = s.hst.viol_key = ~0ULL;
    s.hst.cap_flags = 0;
    s.hst.max_msgs = 0;
    s.hst.hidden_coll = 0;
    s.hst.row_words = 0;
    HIPCHK(hipMemcpyAsync(B.stbuf.p, &s.hst, sizeof s.hst, hipMemcpyHostToDevice, stream));
  }

  // ---- level 1: Init on shard 0 (global position 0); its fp on its owner
  std::vector<uint32_t> init = init_state(M);
  unsigned long long fp0 = host_fingerprint(M, init.data());
  if (fp0 == ~0ULL) fp0--;
  const int owner0 = host_fp_owner(fp0, W);
  for (Shard& s : sh) {
    s.tr_base.assign(2, 0);  // index by depth (1-based)
    s.ncur = s.id == 0 ? 1 : 0;
    s.tr_base.push_back(s.ncur);  // tr_base[2] = first record of level 2
    if (s.id == 0) {
      HIPCHK(hipMemcpyAsync(s.cur, init.data(), WD * 4, hipMemcpyHostToDevice, stream));
      unsigned long long root = ~0ULL;
      uint16_t zero = 0;
      HIPCHK(hipMemcpyAsync(s.B->trp.p, &root, 8, hipMemcpyHostToDevice, stream));
      HIPCHK(hipMemcpyAsync(s.B->trb.p, &zero, 2, hipMemcpyHostToDevice, stream));
    }
    if (s.id == owner0) {
      const unsigned long long ent[2] = {fp0, 0ULL};  // val 0: older than every successor
      HIPCHK(hipMemcpyAsync(s.B->table.as<unsigned long long>() + 2 * fp_slot(fp0, s.slots - 1), ent, 16,
                            hipMemcpyHostToDevice, stream));
      s.entries = 1;
    }
  }
  HIPCHK(hipStreamSynchronize(stream));
  m->levels.clear();
  m->trace_states.clear();
  m->trace_actions.clear();
  std::vector<unsigned long long> level_base = {0, 0}, level_size = {0, 1};  // by depth
  unsigned long long generated = 1, distinct = 1, P = 1;
  unsigned depth = 1;
  m->levels.push_back({1, 1});
  int status = 0;
  std::string message;
  unsigned long long bad_key = ~0ULL, bad_state = ~0ULL;
  {
    int err = 0;
    int bad = host_check_invariants(M, init.data(), &err);
    if (err) { status = 2; message = "evaluation error in an invariant on the initial state"; bad_state = 0; }
    else if (bad >= 0) { status = 1; snprintf(res->violated, sizeof res->violated, "%s", m->inv_names[bad].c_str()); bad_state = 0; }
  }
  // a shard's current level (device rows) -> its host pages; the device frontiers are released
  auto shard_to_host = [&](Shard& s) {
    if (s.hf) return;
    s.hcur.init(pool.page_bytes, WD * 4);
    s.hnxt.init(pool.page_bytes, WD * 4);
    HIPCHK(hipStreamSynchronize(stream));
    s.io.store(s.hcur, s.cur, s.ncur, WD, hdr_words, stream, pool);
    s.B->fa.release();
    s.B->fb.release();
    s.cur = s.nxt = nullptr;
    s.hf = true;
  };
  if (opt->host_frontier == 1)
    for (Shard& s : sh) shard_to_host(s);
  // per-shard kernel timers, read after the round's next stream sync (no sync of their own)
  std::vector<EventTimer> te(NL), tz(NL);
  std::vector<char> te_on(NL, 0), tz_on(NL, 0);
  double expand_ms = 0, mat_ms = 0;
  auto read_timers = [&]() {
    for (int i = 0; i < NL; i++) {
      float ms = 0;
      if (te_on[i]) { HIPCHK(hipEventElapsedTime(&ms, te[i].a, te[i].b)); expand_ms += ms; te_on[i] = 0; }
      if (tz_on[i]) { HIPCHK(hipEventElapsedTime(&ms, tz[i].a, tz[i].b)); mat_ms += ms; tz_on[i] = 0; }
    }
  };
  unsigned long long expand_launches = 0;
  std::vector<std::vector<uint64_t>> rows(NL);
  std::vector<uint64_t> all;
  auto read_status = [&](Shard& s) {
    HIPCHK(hipMemcpyAsync(&s.hst, s.B->stbuf.p, sizeof s.hst, hipMemcpyDeviceToHost, stream));
  };
  bool stop = false;
  // generator-side dedup of each tile's remote candidates (RMC_SHARD_DEDUP=0 turns it off for an A/B)
  const bool tile_dedup = !getenv("RMC_SHARD_DEDUP") || atoi(getenv("RMC_SHARD_DEDUP")) != 0;
  unsigned gmax_msgs = 0;  // largest |DOMAIN messages| materialized on any shard
  double rate = 4.0;       // new states per parent of the previous level (pre-sizes the tables per round)
  unsigned long long lbase = 0, floor = 0;
  // the round's arguments for shard s's c-th local block of parents
  auto round_args = [&](LevelArgs& a, Shard& s, unsigned long long c) {
    memset(&a, 0, sizeof a);
    a.model = &M;
    a.frontier = s.hf ? s.win_in.as<uint32_t>() : s.cur + c * CH * WD;
    a.nparents = s.n;
    a.pbase = lbase + c * W * CH + (unsigned long long)s.id * CH;
    a.level = depth + 1;
    a.floor = floor;
    a.sharded = W;
    a.shard_self = s.id;
    a.table = s.B->table.as<unsigned long long>();
    a.mask = s.slots - 1;
    a.cand_slot = s.B->cfp.as<unsigned long long>();
    a.cand_val = s.B->cval.as<unsigned long long>();
    a.cand_ob = s.B->cob.as<uint32_t>();
    a.cand_win = s.B->cwin.as<uint16_t>();
    a.par_off = s.B->poff.as<uint32_t>();
    a.par_n = s.B->pn.as<uint32_t>();
    a.par_win = s.B->pwin.as<uint32_t>();
    a.par_pos = s.B->ppos.as<uint32_t>();
    a.counters = s.B->counters.as<unsigned long long>();
    a.cand_cap = cand_cap;
    a.st = s.B->stbuf.as<DevStatus>();
  };
  // Capacity exhausted mid-level (host pages, HBM, a row longer than its
  // width): the level in progress is abandoned and the check ends with
  // status 3 and the completed levels' counts, as the single-GPU search does.
  // Host pages and HBM are per process, so with RCCL or shm one rank usually
  // runs out first; it must not leave the level loop while its peers wait in
  // the next collective.  Every step that allocates runs under
  // `guard`, which turns the exception into a local flag and skips the
  // process's remaining guarded work; the flag travels with the next
  // allgather (a column of the existing ones, or `agree` before a
  // point-to-point exchange), and all ranks leave together.
  std::string cap_local;  // this process's capacity failure, this round
  bool abandon = false;   // the level in progress is not counted
  auto guard = [&](auto&& f) {
    if (!cap_local.empty()) return;
    try {
      f();
    } catch (OutOfHostMemory& e) {
      cap_local = std::string("capacity overflow: ") + e.what();
    } catch (OutOfDeviceMemory& e) {
      cap_local = std::string("capacity overflow: ") + e.what();
    } catch (RowCapacity& e) {
      cap_local = e.what();
    }
  };
  // the ranks' flags, allgathered (column `col` of `all`, `ncol` per rank): true when any rank failed
  auto any_failed = [&](int col, int ncol) {
    bool any = false;
    for (int r = 0; r < W; r++) any |= all[(size_t)r * ncol + col] != 0;
    if (any) {
      status = 3;
      message = cap_local.empty() ? "capacity overflow on another rank (host pages or HBM)" : cap_local;
      stop = true;
      abandon = true;
    }
    return any;
  };
  auto agree = [&]() {
    for (int i = 0; i < NL; i++) rows[i] = {(uint64_t)!cap_local.empty()};
    comm.allgather(rows, all, 1);
    return any_failed(0, 1);
  };
  try {
  while (status == 0 && P > 0 && !stop) {
    if (opt->max_depth && (int)depth >= opt->max_depth) { status = 4; break; }
    if (opt->time_limit > 0) {
      // every rank must stop at the same level boundary: the slowest clock decides
      const double el = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
      for (int i = 0; i < NL; i++) rows[i] = {(uint64_t)(el * 1e6)};
      comm.allgather(rows, all, 1);
      if ((double)*std::max_element(all.begin(), all.end()) >= opt->time_limit * 1e6) {
        status = 4;
        message = "time limit";
        break;
      }
    }
    if (opt->host_frontier == 0 && hbm_total) {
      // auto: a next level projected past a quarter of this GPU's HBM (per
      // local shard) moves every shard's levels to host pages at this
      // boundary -- decided on the allgathered projections, so all agree
      for (int i = 0; i < NL; i++)
        rows[i] = {(uint64_t)((double)sh[i].ncur * std::max(rate, 1.0) * 1.25 * (double)(WD * 4) >
                              hf_hbm_fraction() * (double)hbm_total / (NL * std::max(1, comm.dev_share)))};
      comm.allgather(rows, all, 1);
      bool any = false;
      for (int r = 0; r < W; r++) any |= all[r] != 0;
      if (any) {
        guard([&] {
          for (Shard& s : sh) shard_to_host(s);
        });
        if (agree()) break;
      }
    }
    const unsigned level = depth + 1;
    if (level >= 0xFFFF) throw std::runtime_error("too many levels");
    const unsigned long long rounds = (P + W * CH - 1) / (W * CH);
    lbase = level_base[depth];
    unsigned long long GW = 0, gen_lvl = 0;
    if (lbase + P + 1 >= (1ULL << 38)) throw std::runtime_error("more than 2^38 states (the TLC-order rank field)");
    for (Shard& s : sh) s.next_fill = 0;
    floor = (lbase + 1) << VAL_FLOOR_SHIFT;  // entries below: earlier levels
    for (unsigned long long c = 0; c < rounds && !stop;) {
      const unsigned long long gen_round0 = gen_lvl, gw_round0 = GW;  // the level's counts before this round
      // ---- room in each owner's table for the local inserts of k_expand (at
      //      the highest rate of new states per parent seen; a full table is
      //      grown and the round redone below)
      {
        const unsigned long long done = std::min(P, c * W * CH);
        const double r = std::max(rate, done ? (double)GW / (double)done : 0.0);
        for (Shard& s : sh) {
          s.n = s.ncur > c * CH ? std::min(CH, s.ncur - c * CH) : 0;
          if (!opt->grow_on_overflow)
            guard([&] { table_grow(s, s.entries + (unsigned long long)((double)s.n * r * 1.25) + 1024, stream, W); });
        }
      }
      // ---- expand: fp + key per candidate; the fps this shard owns are inserted here
      for (int si = 0; si < NL; si++) {
        Shard& s = sh[si];
        HIPCHK(hipMemsetAsync(s.B->counters.p, 0, 64, stream));
        if (s.n && s.hf) {  // the round's block of this shard's parents, unpacked from host pages
          guard([&] {
            s.win_in.ensure(CH * WD * 4);
            s.io.load(s.hcur, c * CH, s.n, s.win_in.as<uint32_t>(), WD, stream);
          });
        }
        if (s.n && cap_local.empty()) {
          LevelArgs a;
          round_args(a, s, c);
          s.expand_slots = s.slots;
          HIPCHK(hipEventRecord(te[si].a, stream));
          launch_expand(M.spec, M.N, a, stream);
          HIPCHK(hipGetLastError());
          HIPCHK(hipEventRecord(te[si].b, stream));
          te_on[si] = 1;
          expand_launches++;
        }
        HIPCHK(hipMemcpyAsync(&s.ncand, s.B->counters.p, 8, hipMemcpyDeviceToHost, stream));
        read_status(s);
      }
      HIPCHK(hipStreamSynchronize(stream));
      read_timers();
      for (int i = 0; i < NL; i++) rows[i] = {sh[i].ncand, sh[i].hst.cap_flags, (uint64_t)!cap_local.empty()};
      comm.allgather(rows, all, 3);
      if (any_failed(2, 3)) break;
      unsigned capf = 0;
      for (int r = 0; r < W; r++) capf |= (unsigned)all[3 * r + 1];
      if (capf == (1u << E_CAP_TABLE)) {
        // a local insert found its owner's table full: grow the full tables and
        // redo the round on every shard (inserts are idempotent; nothing else
        // of the round has happened yet)
        for (Shard& s : sh) {
          if (s.hst.cap_flags) guard([&] { table_grow(s, s.slots, stream, W); });  // doubles
          s.hst.cap_flags = 0;
          HIPCHK(hipMemcpyAsync((char*)s.B->stbuf.p + offsetof(DevStatus, cap_flags), &s.hst.cap_flags, 4,
                                hipMemcpyHostToDevice, stream));
        }
        HIPCHK(hipStreamSynchronize(stream));
        if (agree()) break;
        continue;
      }
      for (int r = 0; r < W; r++) gen_lvl += all[3 * r];
      if (capf) {
        int e = 0;
        while (!((capf >> e) & 1)) e++;
        if (e == E_CAP_MSG && !opt->msg_cap_K && M.kmax < 120) {
          m->kmax_user = std::min(120u, (uint32_t)M.kmax * 2);
          return 1;
        }
        status = 3;
        message = "capacity overflow (sharded search, code " + std::to_string(e) + ")";
        break;
      }
      std::vector<std::vector<unsigned long long>> xmaps(NL);  // (host side of xmap, alive until the round's sync)
      if (W > 1) {
        // ---- remote-owner candidates: bucket by owner (per-block histograms,
        //      owner-major scan), exchange counts
        std::vector<std::vector<unsigned int>> cnts(NL, std::vector<unsigned int>(W + 1));
        for (int i = 0; i < NL; i++) {
          Shard& s = sh[i];
          const unsigned long long nb = bucket_blocks(s.ncand), nbw = nb * (unsigned long long)W;
          guard([&] {
            s.B->bcnt.ensure((nbw + 1) * 4);
            s.B->boff.ensure((nbw + 1) * 4);
            size_t tb = scan_temp_bytes(nbw + 1);
            s.B->btmp.ensure(tb ? tb : 16);
          });
          if (!cap_local.empty()) {
            cnts[i].assign(W + 1, 0);
            continue;
          }
          unsigned int* bc = s.B->bcnt.as<unsigned int>();
          if (s.n && tile_dedup) {  // a tile's repeats of one fp stay home (OB_TDUP): fewer records to bucket and send
            LevelArgs a;
            round_args(a, s, c);
            launch_tile_dedup(a, s.B->cfp.as<unsigned long long>(), s.B->cval.as<unsigned long long>(),
                              s.B->cob.as<uint32_t>(), stream);
            HIPCHK(hipGetLastError());
          }
          HIPCHK(hipMemsetAsync(bc + nbw, 0, 4, stream));
          launch_owner_count(s.B->cfp.as<unsigned long long>(), s.B->cob.as<uint32_t>(), s.ncand, W, bc, stream);
          HIPCHK(hipGetLastError());
          launch_scan(s.B->btmp.p, s.B->btmp.bytes, bc, s.B->boff.as<unsigned int>(), nbw + 1, stream);
          HIPCHK(hipGetLastError());
          // owner segment starts (boff[o*nb]) and the total (boff[nbw])
          HIPCHK(hipMemcpy2DAsync(cnts[i].data(), 4, s.B->boff.as<unsigned int>(), nb * 4, 4, W, hipMemcpyDeviceToHost,
                                  stream));
          HIPCHK(hipMemcpyAsync(&cnts[i][W], s.B->boff.as<unsigned int>() + nbw, 4, hipMemcpyDeviceToHost, stream));
        }
        HIPCHK(hipStreamSynchronize(stream));
        for (int i = 0; i < NL; i++) {
          rows[i].assign(W + 1, 0);
          for (int d = 0; d < W; d++) rows[i][d] = cnts[i][d + 1] - cnts[i][d];
          rows[i][W] = !cap_local.empty();
        }
        comm.allgather(rows, all, W + 1);
        if (any_failed(W, W + 1)) break;
        {  // all[src*W + dst] = records src sends to dst (the flag column dropped)
          std::vector<uint64_t> a2((size_t)W * W);
          for (int q = 0; q < W; q++)
            for (int d = 0; d < W; d++) a2[(size_t)q * W + d] = all[(size_t)q * (W + 1) + d];
          all.swap(a2);
        }
        for (int i = 0; i < NL; i++) {
          Shard& s = sh[i];
          s.seg_off.assign(W + 1, 0);
          for (int d = 0; d < W; d++) s.seg_off[d + 1] = s.seg_off[d] + all[(size_t)s.id * W + d];
          s.rseg_off.assign(W + 1, 0);
          for (int q = 0; q < W; q++) s.rseg_off[q + 1] = s.rseg_off[q] + all[(size_t)q * W + s.id];
          s.nrecv = s.rseg_off[W];
          guard([&] {
            s.B->send.ensure(std::max<size_t>(16, s.seg_off[W] * 16));
            s.B->sflag.ensure(std::max<size_t>(1, s.seg_off[W]));
            s.B->recv.ensure(std::max<size_t>(16, s.nrecv * 16));
            s.B->rslot.ensure(std::max<size_t>(8, s.nrecv * 8));
            s.B->rflag.ensure(std::max<size_t>(1, s.nrecv));
            // exact bound for the owners' inserts below: the local candidates (inserted) and every received record new
            table_grow(s, s.entries + s.ncand + s.nrecv, stream, W);
          });
        }
        {  // the counts matrix outlives the agreement's allgather
          std::vector<uint64_t> keep = all;
          const bool failed = agree();
          all.swap(keep);
          if (failed) break;
        }
        // Shards sharing the device (logical shards): k_bucket writes each
        // record straight into its owner's receive segment and k_mark_recv
        // each flag straight back into its generator's flag buffer, so neither
        // exchange step copies (the byte-address maps per shard: [0, W)
        // record destinations by owner, [W, 2W) flag destinations by source,
        // [2W, 3W] the receive segments).
        if (same_device) {
          for (int i = 0; i < NL; i++) {
            Shard& s = sh[i];
            std::vector<unsigned long long>& xm = xmaps[i];
            xm.assign(3 * W + 1, 0);
            for (int o = 0; o < W; o++) {
              const Shard& d = sh[o];  // LocalComm: shard ids are 0..W-1 in order
              xm[o] = (unsigned long long)d.B->recv.p + 16ULL * (d.rseg_off[s.id] - s.seg_off[o]);
              xm[W + o] = (unsigned long long)d.B->sflag.p + (d.seg_off[s.id] - s.rseg_off[o]);
            }
            for (int q = 0; q <= W; q++) xm[2 * W + q] = s.rseg_off[q];
            s.B->xmap.ensure(xm.size() * 8);
            HIPCHK(hipMemcpyAsync(s.B->xmap.p, xm.data(), xm.size() * 8, hipMemcpyHostToDevice, stream));
          }
        }
        for (int i = 0; i < NL; i++) {
          Shard& s = sh[i];
          launch_bucket(s.B->cfp.as<unsigned long long>(), s.B->cval.as<unsigned long long>(), s.B->cob.as<uint32_t>(),
                        s.ncand, W, s.B->boff.as<unsigned int>(), s.B->send.as<unsigned long long>(),
                        s.B->perm.as<uint32_t>(), stream,
                        same_device ? s.B->xmap.as<unsigned long long>() : nullptr);
          HIPCHK(hipGetLastError());
        }
        // ---- (fp, key) records to their owners
        if (!same_device) {
          std::vector<Xfer> x;
          for (int q = 0; q < W; q++)
            for (int d = 0; d < W; d++) {
              size_t cntqd = all[(size_t)q * W + d];
              if (!cntqd) continue;
              Xfer t{q, d, nullptr, nullptr, cntqd * 16};
              for (Shard& s : sh) {
                if (s.id == q) t.sbuf = s.B->send.as<unsigned long long>() + 2 * s.seg_off[d];
                if (s.id == d) t.rbuf = s.B->recv.as<unsigned long long>() + 2 * s.rseg_off[q];
              }
              x.push_back(t);
            }
          comm.alltoallv(x);
        }
        // ---- owners insert, then mark
        for (Shard& s : sh) {
          launch_insert_recv(s.B->recv.as<unsigned long long>(), s.nrecv, s.B->table.as<unsigned long long>(),
                             s.slots - 1, floor, s.B->rslot.as<unsigned long long>(), s.B->stbuf.as<DevStatus>(), stream);
          HIPCHK(hipGetLastError());
        }
        for (Shard& s : sh) {
          unsigned long long* nc = s.B->counters.as<unsigned long long>() + 1;
          const unsigned long long* xm = same_device ? s.B->xmap.as<unsigned long long>() : nullptr;
          launch_mark_recv(s.B->recv.as<unsigned long long>(), s.B->rslot.as<unsigned long long>(), s.nrecv,
                           s.B->table.as<unsigned long long>(), floor, s.B->rflag.as<uint8_t>(), nc,
                           s.B->stbuf.as<DevStatus>(), stream, xm ? xm + W : nullptr, xm ? xm + 2 * W : nullptr, W);
          HIPCHK(hipGetLastError());
        }
        // ---- win flags back to the generators (reverse of the record exchange)
        if (!same_device) {
          std::vector<Xfer> x;
          for (int q = 0; q < W; q++)
            for (int d = 0; d < W; d++) {
              size_t cntqd = all[(size_t)q * W + d];
              if (!cntqd) continue;
              Xfer t{d, q, nullptr, nullptr, cntqd};
              for (Shard& s : sh) {
                if (s.id == d) t.sbuf = s.B->rflag.as<uint8_t>() + s.rseg_off[q];
                if (s.id == q) t.rbuf = s.B->sflag.as<uint8_t>() + s.seg_off[d];
              }
              x.push_back(t);
            }
          comm.alltoallv(x);
        }
      }
      // ---- generators: winner ranks per parent (local-owner outcomes from
      //      their own table, remote ones from the flags), positions
      std::vector<unsigned long long> newc(NL, 0);
      for (int i = 0; i < NL; i++) {
        Shard& s = sh[i];
        s.nwin = 0;
        if (s.n) {
          LevelArgs a;
          round_args(a, s, c);
          s.B->sflag.ensure(1);
          s.B->perm.ensure(4);
          launch_mark_gen(a, s.slots != s.expand_slots, s.B->perm.as<uint32_t>(), s.B->sflag.as<uint8_t>(),
                          s.B->counters.as<unsigned long long>() + 1, stream);
          HIPCHK(hipGetLastError());
          launch_scan(s.B->scantmp.p, s.B->scantmp.bytes, s.B->pwin.as<uint32_t>(), s.B->ppos.as<uint32_t>(), s.n,
                      stream);
          HIPCHK(hipGetLastError());
        }
        HIPCHK(hipMemcpyAsync(&newc[i], s.B->counters.as<unsigned long long>() + 1, 8, hipMemcpyDeviceToHost, stream));
      }
      std::vector<uint32_t> lastpos(NL, 0), lastwin(NL, 0);
      for (int i = 0; i < NL; i++)
        if (sh[i].n) {
          HIPCHK(hipMemcpyAsync(&lastpos[i], sh[i].B->ppos.as<uint32_t>() + sh[i].n - 1, 4, hipMemcpyDeviceToHost, stream));
          HIPCHK(hipMemcpyAsync(&lastwin[i], sh[i].B->pwin.as<uint32_t>() + sh[i].n - 1, 4, hipMemcpyDeviceToHost, stream));
        }
      HIPCHK(hipStreamSynchronize(stream));
      for (int i = 0; i < NL; i++) {
        sh[i].nwin = (unsigned long long)lastpos[i] + lastwin[i];
        sh[i].entries += newc[i];
        rows[i] = {sh[i].nwin};
      }
      comm.allgather(rows, all, 1);  // all[r] = winners generated by shard r this round
      std::vector<unsigned long long> go(W + 1, 0);
      for (int r = 0; r < W; r++) go[r + 1] = go[r] + all[r];
      // ---- where the winners go: generator q's winners take the global
      //      positions [GW + go[q], GW + go[q+1]), cut into pieces by
      //      next-level owner (block-cyclic)
      struct Piece { int q, d; unsigned long long a, b, dl; };
      std::vector<Piece> pcs;
      for (int q = 0; q < W; q++) {
        unsigned long long a = GW + go[q], end = GW + go[q + 1];
        while (a < end) {
          unsigned long long blk = a / CH, b = std::min(end, (blk + 1) * CH);
          pcs.push_back({q, (int)(blk % W), a, b, (blk / W) * CH + a % CH});
          a = b;
        }
      }
      for (Shard& s : sh) guard([&] {  // capacity of the receiving side
        unsigned long long need = s.next_fill;
        for (auto& pc : pcs)
          if (pc.d == s.id) need = std::max(need, pc.dl + (pc.b - pc.a));
        if (s.hf) {  // this round's rows: the local range [next_fill, need) into win_out
          s.fill0 = s.next_fill;
          s.win_out.ensure(std::max<unsigned long long>(1, need - s.fill0) * WD * 4);
        } else {  // the next-level buffer grows in place to exactly what it receives
          bool cur_is_a = s.cur == s.B->fa.as<uint32_t>();
          GrowBuf& nb = cur_is_a ? s.B->fb : s.B->fa;
          grow_keep(nb, need * WD * 4, s.next_fill * WD * 4, stream);
          s.cur = (cur_is_a ? s.B->fa : s.B->fb).as<uint32_t>();
          s.nxt = nb.as<uint32_t>();
          s.fcap = std::max(s.fcap, need);
        }
        unsigned long long trneed = s.tr_base[depth + 1] + need;
        if (trneed > s.trcap) {
          unsigned long long nt = trneed + trneed / 4;
          grow_keep(s.B->trp, nt * 8, s.tr_base[depth + 1] * 8 + s.next_fill * 8, stream);
          grow_keep(s.B->trb, nt * 2, s.tr_base[depth + 1] * 2 + s.next_fill * 2, stream);
          s.trcap = nt;
        }
        s.next_fill = need;
      });
      // A generator whose winners all stay with it, in one local run (always
      // at W = 1), writes them straight into its next frontier; the others
      // materialize into staging and send -- unless every shard is on this
      // device (logical shards): then each generator's k_materialize writes
      // its winners straight into their owners' rows and trace records
      // through a piece map, and no row crosses the transport.
      std::vector<std::vector<MatPiece>> hpieces(W);  // alive until the round's stream sync
      if (same_device) {
        for (auto& pc : pcs) {
          Shard* dsh = nullptr;
          for (Shard& t : sh)
            if (t.id == pc.d) dsh = &t;
          const unsigned long long tr = dsh->tr_base[depth + 1] + pc.dl;
          hpieces[pc.q].push_back({pc.a - (GW + go[pc.q]),
                                   dsh->hf ? dsh->win_out.as<uint32_t>() + (pc.dl - dsh->fill0) * WD
                                           : dsh->nxt + pc.dl * WD,
                                   dsh->B->trp.as<unsigned long long>() + tr, dsh->B->trb.as<uint16_t>() + tr});
        }
      }
      std::vector<char> direct(W, 0);
      std::vector<unsigned long long> direct_dl(W, 0);
      for (int q = 0; q < W; q++) {
        bool ok = true, first = true;
        unsigned long long expect = 0;
        for (auto& pc : pcs) {
          if (pc.q != q) continue;
          if (pc.d != q || (!first && pc.dl != expect)) ok = false;
          if (first) direct_dl[q] = pc.dl;
          first = false;
          expect = pc.dl + (pc.b - pc.a);
        }
        direct[q] = same_device || (ok && !first);
      }
      for (Shard& s : sh)  // the staged generators' buffers
        if (s.n && s.nwin && !same_device && !direct[s.id])
          guard([&] {
            s.B->stage.ensure(s.nwin * WD * 4);
            s.B->stp.ensure(s.nwin * 8);
            s.B->stb.ensure(s.nwin * 2);
          });
      {  // every rank has room for the round's rows before any is written or sent
        std::vector<uint64_t> keep = all;
        const bool failed = agree();
        all.swap(keep);
        if (failed) break;
      }
      // ---- materialize winners (TLC order within the generator)
      for (int si = 0; si < NL; si++) {
        Shard& s = sh[si];
        if (!s.n || !s.nwin) continue;
        LevelArgs a;
        round_args(a, s, c);
        if (same_device) {
          const std::vector<MatPiece>& hp = hpieces[s.id];
          s.B->mpc.ensure(std::max<size_t>(64, hp.size() * sizeof(MatPiece)));
          HIPCHK(hipMemcpyAsync(s.B->mpc.p, hp.data(), hp.size() * sizeof(MatPiece), hipMemcpyHostToDevice, stream));
          a.pieces = s.B->mpc.as<MatPiece>();
          a.npieces = (int)hp.size();
        } else if (direct[s.id]) {
          a.out = s.hf ? s.win_out.as<uint32_t>() + (direct_dl[s.id] - s.fill0) * WD : s.nxt + direct_dl[s.id] * WD;
          a.out_base_global = s.tr_base[depth + 1] + direct_dl[s.id];
          a.tr_parent = s.B->trp.as<unsigned long long>();
          a.tr_bind = s.B->trb.as<uint16_t>();
        } else {
          a.out = s.B->stage.as<uint32_t>();
          a.out_base_global = 0;
          a.tr_parent = s.B->stp.as<unsigned long long>();
          a.tr_bind = s.B->stb.as<uint16_t>();
        }
        HIPCHK(hipEventRecord(tz[si].a, stream));
        launch_materialize(M.spec, M.N, a, stream);
        HIPCHK(hipGetLastError());
        HIPCHK(hipEventRecord(tz[si].b, stream));
        tz_on[si] = 1;
      }
      // ---- rows + trace records of the staged generators to their next-level owners
      {
        std::vector<Xfer> x;
        for (auto& pc : pcs) {
          if (direct[pc.q]) continue;
          unsigned long long cnt = pc.b - pc.a, so = pc.a - (GW + go[pc.q]);
          Xfer rowsx{pc.q, pc.d, nullptr, nullptr, cnt * WD * 4};
          Xfer parx{pc.q, pc.d, nullptr, nullptr, cnt * 8};
          Xfer bndx{pc.q, pc.d, nullptr, nullptr, cnt * 2};
          for (Shard& s : sh) {
            if (s.id == pc.q) {
              rowsx.sbuf = s.B->stage.as<uint32_t>() + so * WD;
              parx.sbuf = s.B->stp.as<unsigned long long>() + so;
              bndx.sbuf = s.B->stb.as<uint16_t>() + so;
            }
            if (s.id == pc.d) {
              unsigned long long tr = s.tr_base[depth + 1] + pc.dl;
              rowsx.rbuf = s.hf ? s.win_out.as<uint32_t>() + (pc.dl - s.fill0) * WD : s.nxt + pc.dl * WD;
              parx.rbuf = s.B->trp.as<unsigned long long>() + tr;
              bndx.rbuf = s.B->trb.as<uint16_t>() + tr;
            }
          }
          x.push_back(rowsx);
          x.push_back(parx);
          x.push_back(bndx);
        }
        comm.alltoallv(x);
      }
      GW += go[W];
      // ---- first problem in TLC order stops the search (as TLC does)
      for (Shard& s : sh) read_status(s);
      HIPCHK(hipStreamSynchronize(stream));
      read_timers();
      for (Shard& s : sh)
        if (s.hf)  // the round's new rows to host pages; the round's parents are consumed
          guard([&] {
            s.io.store(s.hnxt, s.win_out.as<uint32_t>(), s.next_fill - s.fill0, WD, hdr_words, stream, pool);
            s.hcur.recycle_below((c + 1) * CH, pool);
          });
      for (int i = 0; i < NL; i++)
        rows[i] = {sh[i].hst.err_key, sh[i].hst.inv_err_key, sh[i].hst.viol_key,
                   sh[i].hst.cap_flags | ((unsigned long long)sh[i].hst.max_msgs << 32), (uint64_t)!cap_local.empty()};
      comm.allgather(rows, all, 5);
      if (any_failed(4, 5)) break;
      unsigned long long ek = ~0ULL, iek = ~0ULL, vk = ~0ULL;
      unsigned capm = 0;
      for (int r = 0; r < W; r++) {
        ek = std::min(ek, (unsigned long long)all[5 * r]);
        iek = std::min(iek, (unsigned long long)all[5 * r + 1]);
        vk = std::min(vk, (unsigned long long)all[5 * r + 2]);
        capm |= (unsigned)all[5 * r + 3];
        gmax_msgs = std::max(gmax_msgs, (unsigned)(all[5 * r + 3] >> 32));
      }
      if (capm) {
        status = 3;
        message = "capacity overflow while materializing";
        stop = true;
      } else if (ek != ~0ULL || iek != ~0ULL || vk != ~0ULL) {
        unsigned long long k_err = std::min(ek, iek);
        if (k_err < vk) {
          status = 2;
          bad_key = k_err;
          message = ek <= iek ? "evaluation error in the next-state relation (a sequence applied outside its domain)"
                              : "evaluation error while checking an invariant";
        } else {
          status = 1;
          bad_key = vk;
        }
        stop = true;
        // TLC's counts at the failing state (as rmc_check): this round's
        // successors of the parents before the failing one, plus the failing
        // parent's up to the failing successor (none for an evaluation error
        // in Next); distinct = the winners among them.  Each shard counts its
        // own block of the round's parents; the sums are allgathered.
        const bool parent_key = status == 2 && ek <= iek;
        const unsigned long long fpg = bad_key >> 20;
        const int ordv = (int)((bad_key >> 10) & 0x3FF);
        for (int i = 0; i < NL; i++) {
          Shard& s = sh[i];
          unsigned long long gi = 0, di = 0;
          if (s.n) {
            const unsigned long long start = lbase + c * W * CH + (unsigned long long)s.id * CH;
            const unsigned long long k = fpg <= start ? 0 : std::min(s.n, fpg - start);
            if (k) {
              std::vector<uint32_t> hn(k), hw(k);
              HIPCHK(hipMemcpy(hn.data(), s.B->pn.p, k * 4, hipMemcpyDeviceToHost));
              HIPCHK(hipMemcpy(hw.data(), s.B->pwin.p, k * 4, hipMemcpyDeviceToHost));
              for (unsigned long long p = 0; p < k; p++) { gi += hn[p]; di += hw[p]; }
            }
            if (!parent_key && fpg >= start && fpg < start + s.n) {
              const unsigned long long pl = fpg - start;
              uint32_t off = 0, nn = 0;
              HIPCHK(hipMemcpy(&off, s.B->poff.as<uint32_t>() + pl, 4, hipMemcpyDeviceToHost));
              HIPCHK(hipMemcpy(&nn, s.B->pn.as<uint32_t>() + pl, 4, hipMemcpyDeviceToHost));
              std::vector<uint32_t> ob(nn);
              std::vector<uint16_t> win(nn);
              if (nn) {
                HIPCHK(hipMemcpy(ob.data(), s.B->cob.as<uint32_t>() + off, nn * 4, hipMemcpyDeviceToHost));
                HIPCHK(hipMemcpy(win.data(), s.B->cwin.as<uint16_t>() + off, nn * 2, hipMemcpyDeviceToHost));
              }
              for (uint32_t q = 0; q < nn; q++)
                if ((int)(ob[q] >> 16) == ordv) { gi += q + 1; di += win[q]; break; }
            }
          }
          rows[i] = {gi, di};
        }
        comm.allgather(rows, all, 2);
        unsigned long long gsum = 0, dsum = 0;
        for (int r = 0; r < W; r++) { gsum += all[2 * r]; dsum += all[2 * r + 1]; }
        gen_lvl = gen_round0 + gsum;
        GW = gw_round0 + dsum;
      }
      c++;
    }
    if (abandon) break;  // a capacity failure agreed mid-level: only completed levels count
    generated += gen_lvl;
    distinct += GW;
    if (GW || gen_lvl) m->levels.push_back({gen_lvl, GW});

    level_base.push_back(lbase + P);
    level_size.push_back(GW);
    if (GW) depth++;
    for (Shard& s : sh) {
      s.tr_base.push_back(s.tr_base[depth] + local_count(GW, W, CH, s.id));
      s.ncur = local_count(GW, W, CH, s.id);
      std::swap(s.cur, s.nxt);
      if (s.hf) {
        s.hcur.clear(pool);
        std::swap(s.hcur, s.hnxt);
      }
    }
    if (P) rate = (double)GW / (double)P;
    P = GW;
    if (opt->verbose && comm.local[0] == 0)
      fprintf(stderr, "[rmc] depth %u: %llu new, %llu distinct, %llu generated (%d shards)\n", depth,
              (unsigned long long)GW, (unsigned long long)distinct, (unsigned long long)generated, W);
  }
  } catch (OutOfHostMemory& oom) {
    status = 3;
    message = std::string("capacity overflow: ") + oom.what();
    HIPCHK(hipDeviceSynchronize());
  } catch (OutOfDeviceMemory& oom) {
    status = 3;
    message = std::string("capacity overflow: ") + oom.what();
    HIPCHK(hipDeviceSynchronize());
  } catch (RowCapacity& e) {
    status = 3;
    message = e.what();
    HIPCHK(hipDeviceSynchronize());
  }
  HIPCHK(hipStreamSynchronize(stream));
  // ---- trace: walk the distributed parent records from the failing state to Init
  if (status == 1 || status == 2) {
    unsigned long long g = ~0ULL;
    int last_b = -1;
    if (bad_key != ~0ULL) {
      g = bad_key >> 20;
      last_b = (int)(bad_key & 0x3FF);
    } else if (bad_state != ~0ULL) {
      g = bad_state;
    }
    std::vector<int> binds;
    while (g != ~0ULL && g != 0) {
      int L = 1;
      while (L + 1 < (int)level_base.size() && level_base[L + 1] <= g) L++;
      unsigned long long pos = g - level_base[L];
      int owner = (int)((pos / CH) % W);
      unsigned long long li = (pos / (W * CH)) * CH + pos % CH;
      for (int i = 0; i < NL; i++) {
        Shard& s = sh[i];
        unsigned long long pp = 0;
        uint16_t bb = 0;
        if (s.id == owner) {
          HIPCHK(hipMemcpy(&pp, s.B->trp.as<unsigned long long>() + s.tr_base[L] + li, 8, hipMemcpyDeviceToHost));
          HIPCHK(hipMemcpy(&bb, s.B->trb.as<uint16_t>() + s.tr_base[L] + li, 2, hipMemcpyDeviceToHost));
        }
        rows[i] = {pp, bb};
      }
      comm.allgather(rows, all, 2);
      binds.push_back((int)all[2 * owner + 1]);
      g = all[2 * owner];
    }
    std::reverse(binds.begin(), binds.end());
    replay_trace(m, binds, last_b, status, message, res);
  }
  if (status == 0 && !opt->max_depth && !opt->msg_cap_K) m->hint_kmax = std::max(1u, gmax_msgs);
  res->max_msgs = gmax_msgs;
  if (!opt->hash_slots) m->hint_slots = sh[0].slots * (unsigned long long)W;
  if (!opt->frontier_cap) m->hint_fcap = sh[0].fcap * (unsigned long long)W;
  m->hint_trcap = sh[0].trcap * (unsigned long long)W;
  res->generated = generated;
  res->distinct = distinct;
  res->left_on_queue = status == 0 ? 0 : P;
  res->depth = depth;
  res->status = status;
  snprintf(res->message, sizeof res->message, "%s", message.c_str());
  res->seconds = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
  res->expand_ms = expand_ms;
  res->materialize_ms = mat_ms;
  res->expand_launches = expand_launches;
  res->hash_capacity = sh[0].slots;
  res->device_bytes = 0;
  for (Shard& s : sh) {
    size_t b = 0;
    ShardBufs& B = *s.B;
    for (DevBuf* x : {&B.table, &B.table2, &B.cfp, &B.cval, &B.cob, &B.cwin, &B.poff, &B.pn, &B.pwin, &B.ppos,
                      &B.counters, &B.stbuf, &B.scantmp, &B.send, &B.perm, &B.recv, &B.rslot, &B.rflag, &B.sflag,
                      &B.stage, &B.stp, &B.stb, &B.small, &B.bcnt, &B.boff, &B.btmp, &s.win_in, &s.win_out, &s.io.pack,
                      &s.io.l32, &s.io.l8, &s.io.off, &s.io.scan, &s.io.stage, &s.io.il32, &s.io.il8, &s.io.ioff,
                      &s.io.iscan})
      b += x->bytes;
    for (GrowBuf* x : {&B.fa, &B.fb, &B.trp, &B.trb}) b += x->bytes;
    res->device_bytes = std::max<uint64_t>(res->device_bytes, b);
    if (opt->verbose || (getenv("RMC_VERBOSE") && atoi(getenv("RMC_VERBOSE")) > 0)) {
      auto g = [](std::initializer_list<size_t> l) {
        size_t t = 0;
        for (size_t v : l) t += v;
        return t / 1073741824.0;
      };
      fprintf(stderr,
              "[rmc] shard %d HBM GiB: set %.1f+%.1f candidates %.1f exchange %.1f staging %.1f frontiers %.1f "
              "trace %.1f host windows %.1f other %.1f (total %.1f)\n",
              s.id, B.table.bytes / 1073741824.0, B.table2.bytes / 1073741824.0,
              g({B.cfp.bytes, B.cval.bytes, B.cob.bytes, B.cwin.bytes, B.perm.bytes}),
              g({B.send.bytes, B.recv.bytes, B.rslot.bytes, B.rflag.bytes, B.sflag.bytes}),
              g({B.stage.bytes, B.stp.bytes, B.stb.bytes}), g({B.fa.bytes, B.fb.bytes}), g({B.trp.bytes, B.trb.bytes}),
              g({s.win_in.bytes, s.win_out.bytes, s.io.pack.bytes, s.io.stage.bytes}),
              g({B.poff.bytes, B.pn.bytes, B.pwin.bytes, B.ppos.bytes, B.scantmp.bytes, B.bcnt.bytes, B.boff.bytes,
                 B.btmp.bytes}),
              b / 1073741824.0);
    }
  }
  {  // same-level hidden-variable collisions, summed over the shards
    for (int i = 0; i < NL; i++) {
      DevStatus fin;
      HIPCHK(hipMemcpy(&fin, sh[i].B->stbuf.p, sizeof fin, hipMemcpyDeviceToHost));
      rows[i] = {fin.hidden_coll};
    }
    comm.allgather(rows, all, 1);
    unsigned long long hc = 0;
    for (int r = 0; r < W; r++) hc += all[r];
    res->hidden_var_collisions = hc;
  }
  return 0;
}

static int run_with_regrow(rmc_model* m, const rmc_options* o, Comm& comm, rmc_result* out) {
  m->kmax_user = 0;
  int rc;
  while ((rc = check_sharded_impl(m, o, comm, out)) == 1) memset(out, 0, sizeof *out);
  return rc;
}

// ------------------------------------------- in-process multi-GPU (n_gpus)
// rmc_options.n_gpus > 1 runs the fingerprint-sharded search
// with one host thread per GPU of this process, each on its own stream --
// the same protocol as rmc_check_sharded's one process per GPU, with the
// communicators created in-process.  The streams and RCCL communicators of a
// device list are kept for the next check (a bench step must not pay
// ncclCommInitAll again).
struct MultiGroup {
  std::vector<int> dev;
  std::vector<hipStream_t> streams;
  std::vector<ncclComm_t> comms;  // RMC_XPORT_RCCL only
};
static std::mutex g_multi_mu;
static std::map<std::string, MultiGroup*> g_multi;
static MultiGroup& multi_group(const std::vector<int>& dev, int transport) {
  std::string key = std::to_string(transport);
  for (int d : dev) key += "," + std::to_string(d);
  std::lock_guard<std::mutex> lk(g_multi_mu);
  MultiGroup*& g = g_multi[key];
  if (g) return *g;
  std::unique_ptr<MultiGroup> ng(new MultiGroup());
  ng->dev = dev;
  for (int d : dev) {
    HIPCHK(hipSetDevice(d));
    hipStream_t s;
    HIPCHK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    ng->streams.push_back(s);
  }
  if (transport == RMC_XPORT_RCCL) {
    ng->comms.assign(dev.size(), nullptr);
    NCCLCHK(ncclCommInitAll(ng->comms.data(), (int)dev.size(), dev.data()));
  }
  g = ng.release();
  return *g;
}
// a group whose communicators were aborted is not reused
static void drop_multi_group(MultiGroup* g) {
  std::lock_guard<std::mutex> lk(g_multi_mu);
  for (auto it = g_multi.begin(); it != g_multi.end(); ++it)
    if (it->second == g) {
      g_multi.erase(it);
      break;
    }
}

static int check_multi(rmc_model* m, const rmc_options* o, const std::vector<int>& dev, int transport,
                       rmc_result* out) {
  const int n = (int)dev.size();
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev < 1) {
    set_last_error("no HIP device available: the raftmc GPU path requires an MI355X (gfx950)");
    return -4;
  }
  for (int d : dev)
    if (d < 0 || d >= ndev) {
      set_last_error("GPU " + std::to_string(d) + " requested for a " + std::to_string(n) + "-GPU check, but " +
                     std::to_string(ndev) + " GPU(s) are visible to this process");
      return -4;
    }
  const std::set<int> uniq(dev.begin(), dev.end());
  if (transport == RMC_XPORT_RCCL && (int)uniq.size() != n) {
    set_last_error("the RCCL transport needs a distinct GPU per shard (RCCL refuses two ranks on one device); "
                   "use RMC_XPORT_P2P to run several shards on one GPU");
    return -1;
  }
  int cur = 0;
  HIPCHK(hipGetDevice(&cur));
  for (int d : uniq) {  // this process's single-GPU caches go; every device's shard world is settled now
    HIPCHK(hipSetDevice(d));
    release_single_buffers();
    settle_shard_world(n);
  }
  if (transport == RMC_XPORT_P2P)  // receivers pull straight from their peers' HBM
    for (int a : uniq)
      for (int b : uniq) {
        int can = 0;
        if (a == b || hipDeviceCanAccessPeer(&can, a, b) != hipSuccess || !can) continue;
        HIPCHK(hipSetDevice(a));
        const hipError_t e = hipDeviceEnablePeerAccess(b, 0);
        if (e != hipSuccess && e != hipErrorPeerAccessAlreadyEnabled) HIPCHK(e);
        (void)hipGetLastError();
      }
  MultiGroup& G = multi_group(dev, transport);
  ThreadGroup grp;
  grp.W = n;
  grp.dev = dev;
  std::vector<std::unique_ptr<rmc_model>> cl;
  for (int r = 0; r < n; r++) cl.emplace_back(new rmc_model(*m));  // each thread finalizes its own copy
  std::vector<rmc_result> res(n);
  std::vector<std::string> err(n);
  std::vector<int> rc(n, 0);
  std::atomic<int> first_failed{-1};
  std::mutex dmu;
  std::condition_variable dcv;
  int done = 0;
  auto work = [&](int r) {
    try {
      HIPCHK(hipSetDevice(dev[r]));
      std::unique_ptr<Comm> c;
      if (transport == RMC_XPORT_RCCL) {
        RcclComm* rc_ = new RcclComm(r, n, G.comms[r], G.streams[r]);
        rc_->aborted = &grp.aborted;
        c.reset(rc_);
      } else {
        c.reset(new ThreadComm(&grp, r, G.streams[r]));
      }
      c->host_share = n;
      c->dev_share = (int)std::count(dev.begin(), dev.end(), dev[r]);
      memset(&res[r], 0, sizeof res[r]);
      rc[r] = run_with_regrow(cl[r].get(), o, *c, &res[r]);
    } catch (std::exception& e) {
      err[r] = e.what();
      rc[r] = -5;
      int none = -1;
      first_failed.compare_exchange_strong(none, r);
      grp.abort();
    }
    std::lock_guard<std::mutex> lk(dmu);
    done++;
    dcv.notify_all();
  };
  std::vector<std::thread> th;
  for (int r = 0; r < n; r++) th.emplace_back(work, r);
  bool aborted_comms = false;
  {
    std::unique_lock<std::mutex> lk(dmu);
    for (;;) {
      if (dcv.wait_for(lk, std::chrono::seconds(30), [&] { return done == n; })) break;
      if (first_failed.load() >= 0 && transport == RMC_XPORT_RCCL && !aborted_comms) {
        // a shard failed 30 s ago and its peers are still blocked inside a
        // collective it will never join: abort the communicators (their
        // kernels stop; the threads see `aborted` and leave without another call)
        fprintf(stderr, "[rmc] shard %d failed; aborting the in-process RCCL communicators\n", first_failed.load());
        for (ncclComm_t c : G.comms) (void)ncclCommAbort(c);
        aborted_comms = true;
      }
    }
  }
  for (auto& t : th) t.join();
  (void)hipSetDevice(cur);
  if (first_failed.load() >= 0) {
    if (transport == RMC_XPORT_RCCL) {
      if (!aborted_comms)
        for (ncclComm_t c : G.comms) (void)ncclCommAbort(c);
      drop_multi_group(&G);  // its communicators are gone (its streams are leaked with it)
    }
    const int f = first_failed.load();
    set_last_error("shard " + std::to_string(f) + " (GPU " + std::to_string(dev[f]) + ") of " + std::to_string(n) +
                   ": " + err[f]);
    return -5;
  }
  for (int r = 0; r < n; r++)
    if (rc[r] != 0) {
      set_last_error("shard " + std::to_string(r) + " returned " + std::to_string(rc[r]));
      return rc[r];
    }
  // every rank holds the global result; shard 0's model (finalized, levels,
  // trace, size hints for the next check) becomes the caller's
  *out = res[0];
  for (int r = 1; r < n; r++) out->device_bytes = std::max(out->device_bytes, res[r].device_bytes);
  *m = std::move(*cl[0]);
  return 0;
}

}  // namespace rmcx

using namespace rmcx;

extern "C" {

int rmc_comm_unique_id(unsigned char* id) {
  if (!id) return -1;
  ncclUniqueId u;
  if (ncclGetUniqueId(&u) != ncclSuccess) {
    set_last_error("ncclGetUniqueId failed");
    return -6;
  }
  memcpy(id, u.internal, NCCL_UNIQUE_ID_BYTES);
  return 0;
}

int rmc_check_sharded(rmc_model* m, const rmc_options* o, int rank, int world, int device, const unsigned char* id,
                      rmc_result* out) {
  if (!m || !out || !id || world < 1 || rank < 0 || rank >= world) { set_last_error("bad argument"); return -1; }
  rmc_options def;
  rmc_options_default(&def);
  if (!o) o = &def;
  memset(out, 0, sizeof *out);
  try {
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev < 1) {
      set_last_error("no HIP device available: the raftmc GPU path requires an MI355X (gfx950)");
      return -4;
    }
    HIPCHK(hipSetDevice(device));
    release_single_buffers();
    // The communicator (and its stream) is kept for later checks with the same
    // id, rank and world: repeated checks do not pay ncclCommInitRank again.
    static std::mutex mu;
    static std::map<std::string, RcclComm*> cache;
    std::string key(reinterpret_cast<const char*>(id), NCCL_UNIQUE_ID_BYTES);
    key += ":" + std::to_string(rank) + ":" + std::to_string(world) + ":" + std::to_string(device);
    RcclComm* comm = nullptr;
    {
      std::lock_guard<std::mutex> lk(mu);
      RcclComm*& c = cache[key];
      if (!c) {
        hipStream_t s;
        HIPCHK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
        ncclUniqueId u;
        memcpy(u.internal, id, NCCL_UNIQUE_ID_BYTES);
        c = new RcclComm(rank, world, u, s);
      }
      comm = c;
    }
    return run_with_regrow(m, o, *comm, out);
  } catch (std::exception& e) {
    set_last_error(e.what());
    return -5;
  }
}

int rmc_check_sharded_shm(rmc_model* m, const rmc_options* o, int rank, int world, int device, const char* shm_name,
                          rmc_result* out) {
  if (!m || !out || !shm_name || world < 1 || world > 16 || rank < 0 || rank >= world) {
    set_last_error("bad argument");
    return -1;
  }
  rmc_options def;
  rmc_options_default(&def);
  if (!o) o = &def;
  memset(out, 0, sizeof *out);
  try {
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev < 1) {
      set_last_error("no HIP device available: the raftmc GPU path requires an MI355X (gfx950)");
      return -4;
    }
    HIPCHK(hipSetDevice(device));
    release_single_buffers();
    hipStream_t s;
    HIPCHK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    int rc;
    {
      ShmComm comm(rank, world, std::string("/") + shm_name, s);
      rc = run_with_regrow(m, o, comm, out);
    }
    HIPCHK(hipStreamDestroy(s));
    return rc;
  } catch (std::exception& e) {
    set_last_error(e.what());
    return -5;
  }
}

int rmc_check_multi(rmc_model* m, const rmc_options* o, const int* devices, int n, int transport, rmc_result* out) {
  if (!m || !out || !devices || n < 1 || n > 64 || (transport != RMC_XPORT_RCCL && transport != RMC_XPORT_P2P)) {
    set_last_error("bad argument");
    return -1;
  }
  rmc_options def;
  rmc_options_default(&def);
  if (!o) o = &def;
  memset(out, 0, sizeof *out);
  try {
    return check_multi(m, o, std::vector<int>(devices, devices + n), transport, out);
  } catch (std::exception& e) {
    set_last_error(e.what());
    return -5;
  }
}

int rmc_check_logical(rmc_model* m, const rmc_options* o, int shards, rmc_result* out) {
  if (!m || !out || shards < 1 || shards > 64) { set_last_error("bad argument"); return -1; }
  rmc_options def;
  rmc_options_default(&def);
  if (!o) o = &def;
  memset(out, 0, sizeof *out);
  try {
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev < 1) {
      set_last_error("no HIP device available: the raftmc GPU path requires an MI355X (gfx950)");
      return -4;
    }
    release_single_buffers();
    hipStream_t s;
    HIPCHK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    int rc;
    {
      LocalComm comm(shards, s);
      rc = run_with_regrow(m, o, comm, out);
    }
    HIPCHK(hipStreamDestroy(s));
    return rc;
  } catch (std::exception& e) {
    set_last_error(e.what());
    return -5;
  }
}

}  // extern "C"
