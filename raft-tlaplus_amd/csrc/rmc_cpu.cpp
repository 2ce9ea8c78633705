// rmc_cpu.cpp — the CPU engine: TLC's `-workers N` breadth-first search on
// host threads, over the SAME packed layout, lowered Next actions and
// invariants (rmc_spec.h), canonical fingerprint and fingerprint-set rule
// (first successor in TLC order wins, earlier levels' entries never written;
// rmc_fpset.h) as the GPU path.  BASELINE.md's CPU baseline ("the build's own
// multi-threaded C++ BFS ... same semantics and the same packed layout, so the
// comparison measures only the accelerator"), and `raftmc -cpu -workers N`.
// It is an explicitly requested engine (rmc_check_cpu), never a fallback of
// rmc_check.
//
// Per level, per chunk of parents (one level = one or more chunks, in TLC
// order): A) each worker expands a contiguous range of parents -- every Next
// binding, the successor's fingerprint from the parent's message sums, the
// insert -- recording each parent's successors in TLC ordinal order; B) the
// workers mark the winners (and count same-level hidden-variable
// collisions); C) a prefix over the parents' winner counts places every new
// state at its TLC position, and the workers materialize them, write the
// trace records and check the cfg's invariants.
#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstring>
#include <string>
#include <thread>
#include <vector>
#include "rmc_internal.h"

using namespace rmc;

#ifdef RMC_TILESTATS
#include <cstdio>
#include <unordered_set>
static std::atomic<uint64_t> g_tile_intra{0}, g_tile_early{0};
#endif
namespace rmcx {
namespace {

constexpr uint64_t EMPTY64 = ~0ULL;
constexpr int RANK_SHIFT = 16, FLOOR_SHIFT = 26;  // as rmc_fpset.h

uint64_t slot_of(uint64_t fp, uint64_t mask) { return ((fp * 0x9E3779B97F4A7C15ULL) >> __builtin_clzll(mask)) & mask; }

// rmc_fpset.h's table on host atomics (the same insert rule).
struct HostSet {
  std::vector<uint64_t> T;  // 2 words per slot
  uint64_t mask = 0, entries = 0;
  void init(uint64_t slots) {
    T.assign(2 * slots, EMPTY64);
    mask = slots - 1;
  }
  static void amin(uint64_t* p, uint64_t v) {
    uint64_t cur = __atomic_load_n(p, __ATOMIC_RELAXED);
    while (v < cur && !__atomic_compare_exchange_n(p, &cur, v, true, __ATOMIC_RELAXED, __ATOMIC_RELAXED)) {
    }
  }
  uint64_t insert(uint64_t fp, uint64_t val, uint64_t floor) {
    uint64_t slot = slot_of(fp, mask);
    for (uint64_t probe = 0; probe <= mask; probe++) {
      uint64_t* e = T.data() + 2 * slot;
      uint64_t prev = EMPTY64;
      if (__atomic_compare_exchange_n(e, &prev, fp, false, __ATOMIC_RELAXED, __ATOMIC_RELAXED)) {
        amin(e + 1, val);
        return slot;
      }
      if (prev == fp) {
        if (__atomic_load_n(e + 1, __ATOMIC_RELAXED) >= floor) amin(e + 1, val);
        return slot;
      }
      slot = (slot + 1) & mask;
    }
    return EMPTY64;
  }
  void grow(uint64_t nslots) {  // single-threaded rehash (values kept)
    std::vector<uint64_t> old;
    old.swap(T);
    init(nslots);
    for (size_t e = 0; e < old.size(); e += 2) {
      if (old[e] == EMPTY64) continue;
      uint64_t slot = slot_of(old[e], mask);
      while (T[2 * slot] != EMPTY64) slot = (slot + 1) & mask;
      T[2 * slot] = old[e];
      T[2 * slot + 1] = old[e + 1];
    }
  }
};

struct Cand {
  uint64_t slot;  // table slot, or EMPTY64 for an erroring binding
  uint32_t ob;    // ordinal << 16 | binding, 0x8000 = evaluation error
  uint16_t hidden;
  uint16_t win;   // 1 + winner rank among the parent's successors, 0 = lost
};

template <class F>
void parallel_for(int T, uint64_t n, F f) {  // f(worker, lo, hi): contiguous ranges in TLC order
  if (T <= 1 || n < 64) {
    f(0, 0, n);
    return;
  }
  std::vector<std::thread> th;
  for (int w = 0; w < T; w++) {
    uint64_t lo = n * w / T, hi = n * (w + 1) / T;
    th.emplace_back([=, &f]() { f(w, lo, hi); });
  }
  for (auto& t : th) t.join();
}

uint64_t order_key(uint64_t pg, int ordinal, int b) { return (pg << 20) | ((uint64_t)ordinal << 10) | (uint64_t)b; }

template <int SPEC, int N>
int check_cpu_t(rmc_model* m, const rmc_options* opt, int T, rmc_result* res) {
  auto t0 = std::chrono::steady_clock::now();
  auto elapsed = [&]() { return std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count(); };
  const Model& M = m->M;
  const size_t W = (size_t)M.words;
  res->state_bytes = (uint32_t)(W * 4);
  HostSet set;
  set.init(opt->hash_slots ? opt->hash_slots : (1ULL << 20));
  std::vector<uint32_t> cur = init_state(M), nxt;
  std::vector<uint64_t> tr_parent = {~0ULL};
  std::vector<uint16_t> tr_bind = {0};
  {
    uint64_t fp = host_fingerprint(M, cur.data());
    if (fp == EMPTY64) fp--;
    set.insert(fp, 0, 0);
    set.entries = 1;
  }
  m->levels.clear();
  m->trace_states.clear();
  m->trace_actions.clear();
  m->levels.push_back({1, 1});
  uint64_t generated = 1, distinct = 1, cur_n = 1, cur_base = 0, hidden_coll = 0;
  unsigned depth = 1;
  int status = 0;
  std::string message;
  uint64_t bad_key = ~0ULL, bad_state = ~0ULL;
  bool bad_is_parent_key = false;
  unsigned max_msgs = 0;
  {
    int err = 0;
    int bad = host_check_invariants(M, cur.data(), &err);
    if (err) { status = 2; message = "evaluation error in an invariant on the initial state"; bad_state = 0; }
    else if (bad >= 0) { status = 1; snprintf(res->violated, sizeof res->violated, "%s", m->inv_names[bad].c_str()); bad_state = 0; }
  }
  const uint64_t CH = opt->chunk_parents ? opt->chunk_parents : (1ULL << 20);
  double rate = 4.0;  // new states per parent of the previous level (pre-sizes the table)
  std::vector<std::vector<Cand>> cands(T);
  std::vector<uint64_t> par_off, par_n, par_win, par_pos;
  while (status == 0 && cur_n > 0) {
    if (opt->max_depth && (int)depth >= opt->max_depth) { status = 4; break; }
    if (opt->time_limit > 0 && elapsed() > opt->time_limit) { status = 4; message = "time limit"; break; }
    nxt.clear();
    uint64_t gen_lvl = 0, next_n = 0;
    const uint64_t floor = (cur_base + 1) << FLOOR_SHIFT;
    std::atomic<uint64_t> err_key{~0ULL}, viol_key{~0ULL}, inv_err_key{~0ULL};
    std::atomic<unsigned> capf{0}, mx{0};
    std::atomic<uint64_t> coll{0};
    for (uint64_t c0 = 0; c0 < cur_n && status == 0; c0 += CH) {
      const uint64_t n = std::min(CH, cur_n - c0);
      // room at <= 0.75 load for this chunk's new states at the highest rate seen
      const double r = std::max(rate, c0 ? (double)next_n / (double)c0 : 0.0);
      const uint64_t need = set.entries + (uint64_t)((double)n * r * 1.5) + 1024;
      if (need * 4 > (set.mask + 1) * 3) {
        uint64_t ns = set.mask + 1;
        while (need * 2 > ns) ns <<= 1;
        set.grow(ns);
      }
      par_off.assign(n + 1, 0);
      par_n.assign(n, 0);
      par_win.assign(n, 0);
      par_pos.assign(n, 0);
      for (auto& cv : cands) cv.clear();  // workers that get no parents (small chunks) must not keep stale ones
      // ---- A: expand
      parallel_for(T, n, [&](int w, uint64_t lo, uint64_t hi) {
        std::vector<Cand>& out = cands[w];
        std::vector<std::pair<int, Cand>> succ;
#ifdef RMC_TILESTATS
        // diagnostic: successors whose fingerprint another successor of the same
        // 64-parent tile (k_expand's tile) produced first; earlier-level duplicates
        std::unordered_set<uint64_t> tile_fps;
        uint64_t t_intra = 0, t_early = 0;
#endif
        for (uint64_t q = lo; q < hi; q++) {
#ifdef RMC_TILESTATS
          if (q == lo || q % 64 == 0) tile_fps.clear();
#endif
          const uint64_t pg = cur_base + c0 + q;
          PState<SPEC, N> s{cur.data() + (c0 + q) * W};
          MsgSums<N> ms{};
          const int nm = s.nmsg();
          for (int k = 0; k < nm; k++) {
            int src, dst;
            const uint64_t u = msg_u<SPEC>(s.msg(k), src, dst);
            ms.sig[src] += (uint32_t)u;
            ms.sig[dst] += (uint32_t)(u >> 32);
            if (src != dst) ms.S[MsgSums<N>::pair(src, dst)] += u;
          }
          succ.clear();
          const int B = nbindings(M, nm);
          for (int x = 0; x < B; x++) {
            const int b = binding_at(M, x, nm);
            Delta d;
            if (!eval_binding<SPEC, N>(s, M, b, d)) continue;
            Cand c;
            c.ob = ((uint32_t)d.ordinal << 16) | (uint32_t)b;
            c.win = 0;
            c.hidden = (uint16_t)hidden_of<SPEC>(d.hdr);
            c.slot = EMPTY64;
            if (d.err) {
              c.ob |= 0x8000u;
              if (d.err == E_DOMAIN) {
                uint64_t k = order_key(pg, d.ordinal, b), e = err_key.load();
                while (k < e && !err_key.compare_exchange_weak(e, k)) {}
              } else {
                capf |= 1u << d.err;
              }
            } else {
              int adds = 0;
              for (int x = 0; x < d.nops; x++) adds += d.opk[x] < 0;
              if (nm + adds > M.kmax) capf |= 1u << E_CAP_MSG;
              uint64_t fp = delta_fp_sums<SPEC, N>(s, M, d, ms);
              uint64_t val = ((((pg + 1) << 10) | (uint64_t)d.ordinal) << RANK_SHIFT) | c.hidden;
              c.slot = set.insert(fp, val, floor);
              if (c.slot == EMPTY64) capf |= 1u << E_CAP_TABLE;
#ifdef RMC_TILESTATS
              if (!tile_fps.insert(fp).second) t_intra++;
              else if (c.slot != EMPTY64 && __atomic_load_n(&set.T[2 * c.slot + 1], __ATOMIC_RELAXED) < floor) t_early++;
#endif
            }
            succ.push_back({d.ordinal, c});
          }
          std::sort(succ.begin(), succ.end(), [](const auto& x, const auto& y) { return x.first < y.first; });
          par_n[q] = succ.size();
          par_off[q] = out.size();  // worker-local; rebased below
          for (auto& sc : succ) out.push_back(sc.second);
        }
#ifdef RMC_TILESTATS
        g_tile_intra += t_intra;
        g_tile_early += t_early;
#endif
      });
      if (capf.load()) {
        int e = 0;
        while (!((capf.load() >> e) & 1)) e++;
        if (e == E_CAP_MSG && !opt->msg_cap_K && M.kmax < 120) {
          m->kmax_user = std::min(120u, (uint32_t)M.kmax * 2);
          return 1;
        }
        status = 3;
        message = "capacity overflow (code " + std::to_string(e) + ")";
        break;
      }
      // worker-local offsets -> (worker, offset)
      std::vector<int> owner(n);
      for (int w = 0; w < T; w++) {
        uint64_t lo = (T <= 1 || n < 64) ? (w == 0 ? 0 : n) : n * w / T;
        uint64_t hi = (T <= 1 || n < 64) ? (w == 0 ? n : n) : n * (w + 1) / T;
        for (uint64_t q = lo; q < hi; q++) owner[q] = w;
      }
      // ---- B: winners (after every insert of the chunk)
      parallel_for(T, n, [&](int, uint64_t lo, uint64_t hi) {
        uint64_t cc = 0;
        for (uint64_t q = lo; q < hi; q++) {
          Cand* c = cands[owner[q]].data() + par_off[q];
          const uint64_t base = (cur_base + c0 + q + 1) << 10;
          uint64_t won = 0;
          for (uint64_t k = 0; k < par_n[q]; k++) {
            if (c[k].slot == EMPTY64) continue;
            const uint64_t v = __atomic_load_n(&set.T[2 * c[k].slot + 1], __ATOMIC_RELAXED);
            const bool win = (v >> RANK_SHIFT) == (base | (c[k].ob >> 16));
            if (win) c[k].win = (uint16_t)(++won);
            else if (v >= floor && ((v ^ c[k].hidden) & 0xFFFFULL)) cc++;
          }
          par_win[q] = won;
        }
        coll += cc;
      });
      uint64_t wsum = 0;
      for (uint64_t q = 0; q < n; q++) {
        par_pos[q] = wsum;
        wsum += par_win[q];
      }
      const uint64_t out0 = next_n;
      nxt.resize((next_n + wsum) * W);
      tr_parent.resize(distinct + next_n + wsum);
      tr_bind.resize(distinct + next_n + wsum);
      // ---- C: materialize, trace records, invariants
      parallel_for(T, n, [&](int, uint64_t lo, uint64_t hi) {
        unsigned mloc = 0;
        for (uint64_t q = lo; q < hi; q++) {
          const uint64_t pg = cur_base + c0 + q;
          PState<SPEC, N> s{cur.data() + (c0 + q) * W};
          const Cand* c = cands[owner[q]].data() + par_off[q];
          for (uint64_t k = 0; k < par_n[q]; k++) {
            if (!c[k].win) continue;
            const int b = (int)(c[k].ob & 0x3FF);
            Delta d;
            eval_binding<SPEC, N>(s, M, b, d);
            const uint64_t dst = out0 + par_pos[q] + c[k].win - 1;
            uint32_t* o = nxt.data() + dst * W;
            int nn = 0;
            int e = apply_delta<SPEC, N>(s, M, d, o, &nn);
            if (e) capf |= 1u << e;
            mloc = std::max(mloc, (unsigned)nn);
            tr_parent[distinct + dst] = pg;
            tr_bind[distinct + dst] = (uint16_t)b;
            int ierr = 0;
            PState<SPEC, N> ns{o};
            int bad = check_invariants<SPEC, N>(ns, M, ierr);
            std::atomic<uint64_t>& key = ierr ? inv_err_key : viol_key;
            if (ierr || bad >= 0) {
              uint64_t kk = order_key(pg, (int)(c[k].ob >> 16), b), ev = key.load();
              while (kk < ev && !key.compare_exchange_weak(ev, kk)) {}
            }
          }
        }
        unsigned cm = mx.load();
        while (mloc > cm && !mx.compare_exchange_weak(cm, mloc)) {}
      });
      for (int w = 0; w < T; w++) gen_lvl += cands[w].size();
      next_n += wsum;
      set.entries += wsum;
      if (capf.load()) {
        status = 3;
        message = "capacity overflow while materializing";
        break;
      }
      // TLC stops at the first problem in its exploration order: exact counts up to it
      const uint64_t ek = std::min(err_key.load(), inv_err_key.load()), vk = viol_key.load();
      if (ek != ~0ULL || vk != ~0ULL) {
        const bool is_err = ek < vk;
        bad_key = is_err ? ek : vk;
        bad_is_parent_key = is_err && err_key.load() <= inv_err_key.load();
        status = is_err ? 2 : 1;
        message = !is_err ? "" : bad_is_parent_key ? "evaluation error in the next-state relation (a sequence applied outside its domain)"
                                                   : "evaluation error while checking an invariant";
        const uint64_t pl = (bad_key >> 20) - cur_base - c0;
        const int ordv = (int)((bad_key >> 10) & 0x3FF);
        uint64_t g = gen_lvl, dn = next_n;
        for (int w = 0; w < T; w++) g -= cands[w].size();
        dn -= wsum;
        for (uint64_t q = 0; q < pl; q++) { g += par_n[q]; dn += par_win[q]; }
        if (!bad_is_parent_key) {
          const Cand* c = cands[owner[pl]].data() + par_off[pl];
          for (uint64_t k = 0; k < par_n[pl]; k++)
            if ((int)(c[k].ob >> 16) == ordv) { g += k + 1; dn += c[k].win; break; }
        }
        gen_lvl = g;
        next_n = dn;
      }
    }
    generated += gen_lvl;
    distinct += next_n;
    if (next_n || gen_lvl) m->levels.push_back({gen_lvl, next_n});
    if (next_n) depth++;
    hidden_coll += coll.load();
    max_msgs = std::max(max_msgs, mx.load());
    rate = (double)next_n / (double)cur_n;
    if (opt->verbose)
      fprintf(stderr, "[rmc-cpu] depth %u: %llu new, %llu distinct, %llu generated, t=%.3fs (%d workers)\n", depth,
              (unsigned long long)next_n, (unsigned long long)distinct, (unsigned long long)generated, elapsed(), T);
    cur_base += cur_n;
    cur_n = next_n;
    cur.swap(nxt);
    if (status) break;
  }
  if (status == 1 || status == 2) {
    uint64_t g = ~0ULL;
    int last_b = -1;
    if (bad_key != ~0ULL) {
      g = bad_key >> 20;
      last_b = (int)(bad_key & 0x3FF);
    } else if (bad_state != ~0ULL) {
      g = bad_state;
    }
    std::vector<int> binds;
    while (g != ~0ULL && g != 0) {
      binds.push_back(tr_bind[g]);
      g = tr_parent[g];
    }
    std::reverse(binds.begin(), binds.end());
    replay_trace(m, binds, last_b, status, message, res);
  }
  res->generated = generated;
  res->distinct = distinct;
  res->left_on_queue = status == 0 ? 0 : cur_n;
  res->depth = depth;
  res->status = status;
  snprintf(res->message, sizeof res->message, "%s", message.c_str());
  res->seconds = elapsed();
#ifdef RMC_TILESTATS
  fprintf(stderr, "[rmc-cpu] successors %llu: new %llu, same-tile duplicates %llu, earlier-level duplicates %llu\n",
          (unsigned long long)generated, (unsigned long long)distinct, (unsigned long long)g_tile_intra.load(),
          (unsigned long long)g_tile_early.load());
#endif
  res->hash_capacity = set.mask + 1;
  res->max_msgs = max_msgs;
  res->hidden_var_collisions = hidden_coll;
  if (status == 0 && !opt->max_depth && !opt->msg_cap_K && opt->time_limit <= 0) m->hint_kmax = std::max(1u, max_msgs);
  return 0;
}

}  // namespace

int check_cpu(rmc_model* m, const rmc_options* opt, rmc_result* res) {
  Model& M = m->M;
  uint32_t kmax = opt->msg_cap_K ? opt->msg_cap_K : (m->kmax_user ? m->kmax_user : model_kmax(m));
  if (kmax > 120) kmax = 120;
  finalize_model(m, kmax);
  int T = opt->cpu_workers > 0 ? opt->cpu_workers : (int)std::max(1u, std::thread::hardware_concurrency());
#define RMC_CPU(SP, NN) \
  if (M.spec == SP && M.N == NN) return check_cpu_t<SP, NN>(m, opt, T, res);
  RMC_CPU(RAFT, 2) RMC_CPU(RAFT, 3) RMC_CPU(RAFT, 4) RMC_CPU(RAFT, 5)
  RMC_CPU(FLEX, 2) RMC_CPU(FLEX, 3) RMC_CPU(FLEX, 4) RMC_CPU(FLEX, 5)
  RMC_CPU(FSYNC, 2) RMC_CPU(FSYNC, 3) RMC_CPU(FSYNC, 4) RMC_CPU(FSYNC, 5)
  RMC_CPU(PULL, 2) RMC_CPU(PULL, 3) RMC_CPU(PULL, 4) RMC_CPU(PULL, 5)
  RMC_CPU(PULL2, 2) RMC_CPU(PULL2, 3) RMC_CPU(PULL2, 4) RMC_CPU(PULL2, 5)
  RMC_CPU(KRAFT, 2) RMC_CPU(KRAFT, 3)
#undef RMC_CPU
  throw std::runtime_error("unsupported model shape");
}

}  // namespace rmcx

extern "C" int rmc_check_cpu(rmc_model* m, const rmc_options* o, rmc_result* out) {
  if (!m || !out) { rmcx::set_last_error("null argument"); return -1; }
  rmc_options def;
  rmc_options_default(&def);
  if (!o) o = &def;
  memset(out, 0, sizeof *out);
  try {
    if (o->deadlock_check) throw std::runtime_error("deadlock checking is not supported; run with -deadlock (README.md:6)");
    if (o->fp_bits && o->fp_bits != 64) throw std::runtime_error("fp_bits 128 is offered by the single-GPU search (rmc_check) only");
    if ((o->checkpoint_dir && *o->checkpoint_dir) || (o->recover_dir && *o->recover_dir))
      throw std::runtime_error("checkpoint / recover are offered by the single-GPU search (rmc_check) only");
    if (o->host_frontier == 1) throw std::runtime_error("host_frontier = 1 is offered by the single-GPU search (rmc_check) only");
    m->kmax_user = 0;
    int rc;
    while ((rc = rmcx::check_cpu(m, o, out)) == 1) memset(out, 0, sizeof *out);
    return rc;
  } catch (std::exception& e) {
    rmcx::set_last_error(e.what());
    return -5;
  }
}
