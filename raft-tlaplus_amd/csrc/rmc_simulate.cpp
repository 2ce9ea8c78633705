// rmc_simulate.cpp — TLC's random simulation mode (`-simulate`) on the GPU:
// SURVEY.md §8f rank 2, "the author's recommended mode for the specs too big
// to exhaust" (flexible-raft/FlexibleRaft.cfg:5, pull-raft/KRaftWithReconfig.cfg:5).
//
// Rounds of `walkers` random behaviours run in parallel (k_simulate, one lane
// per behaviour), each from Init for at most `depth` steps, choosing every
// step uniformly among the enabled successors; invariants are checked on every
// state.  The run stops at the first violation / evaluation error (its
// behaviour is replayed on the host into a TLC-format trace), when `behaviors`
// behaviours have been generated, or after `seconds`.
#include <chrono>
#include <cstring>
#include <string>
#include <vector>
#include "rmc_internal.h"

using namespace rmc;

namespace rmcx {

static int simulate_impl(rmc_model* m, const rmc_options* opt, unsigned long long walkers, unsigned depth,
                         unsigned long long seed, unsigned long long behaviors, double seconds, rmc_result* res) {
  auto t0 = std::chrono::steady_clock::now();
  Model& M = m->M;
  uint32_t kmax = opt->msg_cap_K ? opt->msg_cap_K : (m->kmax_user ? m->kmax_user : default_kmax(M));
  if (kmax > 120) kmax = 120;
  finalize_model(m, kmax);
  HIPCHK(upload_model(M));
  const size_t W = (size_t)M.words;
  res->state_bytes = (uint32_t)(W * 4);
  m->levels.clear();
  m->trace_states.clear();
  m->trace_actions.clear();
  std::vector<uint32_t> init = init_state(M);
  std::string message;
  {
    int err = 0;
    int bad = host_check_invariants(M, init.data(), &err);
    if (err || bad >= 0) {
      res->status = err ? 2 : 1;
      if (!err) snprintf(res->violated, sizeof res->violated, "%s", m->inv_names[bad].c_str());
      replay_trace(m, {}, -1, res->status, message, res);
      res->generated = 1;
      res->distinct = 1;
      res->depth = 1;
      return 0;
    }
  }
  hipStream_t stream;
  HIPCHK(hipStreamCreateWithFlags(&stream, hipStreamNonBlocking));
  DevBuf dinit, binds, counters, ssb, stb;
  dinit.ensure(W * 4);
  binds.ensure(walkers * depth * 2);
  counters.ensure(16);
  ssb.ensure(sizeof(SimStatus));
  stb.ensure(sizeof(DevStatus));
  HIPCHK(hipMemcpyAsync(dinit.p, init.data(), W * 4, hipMemcpyHostToDevice, stream));
  HIPCHK(hipMemsetAsync(counters.p, 0, 16, stream));
  {
    SimStatus s0;
    memset(&s0, 0, sizeof s0);
    s0.key = ~0ULL;
    HIPCHK(hipMemcpyAsync(ssb.p, &s0, sizeof s0, hipMemcpyHostToDevice, stream));
  }
  DevStatus hst;
  memset(&hst, 0, sizeof hst);
  hst.err_key = hst.inv_err_key = hst.viol_key = ~0ULL;
  hst.cap_flags = 0;
  hst.max_msgs = 0;
  HIPCHK(hipMemcpyAsync(stb.p, &hst, sizeof hst, hipMemcpyHostToDevice, stream));
  unsigned long long done = 0, generated = 0;
  unsigned long long round = 0;
  SimStatus ss;
  memset(&ss, 0, sizeof ss);
  ss.key = ~0ULL;
  int status = 0;
  unsigned long long cnt[2] = {0, 0};
  while (done < behaviors) {
    unsigned long long n = std::min(walkers, behaviors - done);
    unsigned long long rseed = seed + 0x9E3779B97F4A7C15ULL * (round + 1);
    launch_simulate(M.spec, M.N, dinit.as<uint32_t>(), n, depth, rseed, binds.as<uint16_t>(),
                    counters.as<unsigned long long>(), ssb.as<SimStatus>(), stb.as<DevStatus>(), (int)W, stream);
    HIPCHK(hipGetLastError());
    HIPCHK(hipMemcpyAsync(&ss, ssb.p, sizeof ss, hipMemcpyDeviceToHost, stream));
    HIPCHK(hipMemcpyAsync(&hst, stb.p, sizeof hst, hipMemcpyDeviceToHost, stream));
    HIPCHK(hipMemcpyAsync(cnt, counters.p, 16, hipMemcpyDeviceToHost, stream));
    HIPCHK(hipStreamSynchronize(stream));
    if (ss.key != ~0ULL) {
      ss.stop = (unsigned)(ss.key & 3u);
      ss.steps = (unsigned)((ss.key >> 2) & 0x3FFFFu);
      ss.walker = ss.key >> 20;
    }
    done += n;
    round++;
    if (hst.cap_flags) {
      int e = 0;
      while (!((hst.cap_flags >> e) & 1)) e++;
      if (e == E_CAP_MSG && !opt->msg_cap_K && M.kmax < 120) {
        m->kmax_user = std::min(120u, (uint32_t)M.kmax * 2);
        HIPCHK(hipStreamDestroy(stream));
        return 1;
      }
      status = 3;
      message = "capacity overflow in simulation (code " + std::to_string(e) + ")";
      break;
    }
    if (ss.stop) break;
    if (seconds > 0 && std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() >= seconds) break;
  }
  generated = done + cnt[0];  // initial states + steps
  if (ss.stop) {
    std::vector<uint16_t> b(ss.steps);
    HIPCHK(hipMemcpy(b.data(), binds.as<uint16_t>() + ss.walker * depth, ss.steps * 2, hipMemcpyDeviceToHost));
    std::vector<int> chain(b.begin(), b.end());
    int last_b = -1;
    if (ss.stop == 1) {
      status = 1;
    } else if (ss.stop == 2) {
      status = 2;
      last_b = chain.back();
      chain.pop_back();
      message = "evaluation error in the next-state relation (a sequence applied outside its domain)";
    } else {
      status = 2;
      message = "evaluation error while checking an invariant";
    }
    replay_trace(m, chain, last_b, status, message, res);
  }
  HIPCHK(hipStreamDestroy(stream));
  res->generated = generated;
  res->distinct = done;  // simulation: behaviours generated (TLC reports states generated and traces)
  res->depth = (uint32_t)(cnt[1] + 1);
  res->left_on_queue = 0;
  res->status = status;
  snprintf(res->message, sizeof res->message, "%s", message.c_str());
  res->seconds = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
  return 0;
}

}  // namespace rmcx

using namespace rmcx;

extern "C" int rmc_simulate(rmc_model* m, const rmc_options* o, uint64_t walkers, uint32_t depth, uint64_t seed,
                            uint64_t behaviors, double seconds, rmc_result* out) {
  if (!m || !out || !walkers || !depth || depth > 65535 || !behaviors) {
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
    m->kmax_user = 0;
    int rc;
    while ((rc = simulate_impl(m, o, walkers, depth, seed, behaviors, seconds, out)) == 1) memset(out, 0, sizeof *out);
    return rc;
  } catch (std::exception& e) {
    set_last_error(e.what());
    return -5;
  }
}
