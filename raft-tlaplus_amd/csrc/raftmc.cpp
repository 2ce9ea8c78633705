// raftmc — TLC-compatible command line over librmc:
//   raftmc [-deadlock] [-workers N] [-config M.cfg] [-json] [-v] M.tla
// mirrors `java tlc2.TLC -deadlock [-workers N] [-config M.cfg] M.tla`
// (reference README.md:6) and prints TLC's result lines.
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>
#include "../../include/rmc.h"

int main(int argc, char** argv) {
  rmc_options o;
  rmc_options_default(&o);
  o.deadlock_check = 1;  // TLC default; the reference always passes -deadlock
  std::string tla, cfg;
  bool json = false;
  for (int a = 1; a < argc; a++) {
    std::string k = argv[a];
    auto val = [&]() -> std::string {
      if (a + 1 >= argc) { fprintf(stderr, "missing value for %s\n", k.c_str()); exit(2); }
      return argv[++a];
    };
    if (k == "-deadlock") o.deadlock_check = 0;
    else if (k == "-workers") o.cpu_workers = atoi(val().c_str());
    else if (k == "-config") cfg = val();
    else if (k == "-gpus") o.n_gpus = atoi(val().c_str());
    else if (k == "-msgcap") o.msg_cap_K = (uint32_t)atoi(val().c_str());
    else if (k == "-hashslots") o.hash_slots = strtoull(val().c_str(), nullptr, 10);
    else if (k == "-maxdepth") o.max_depth = atoi(val().c_str());
    else if (k == "-chunk") o.chunk_parents = (uint32_t)atoi(val().c_str());
    else if (k == "-json") json = true;
    else if (k == "-v") o.verbose = 1;
    else if (!k.empty() && k[0] == '-') { fprintf(stderr, "raftmc: unknown option %s\n", k.c_str()); return 2; }
    else tla = k;
  }
  if (tla.empty()) {
    fprintf(stderr, "usage: raftmc [-deadlock] [-workers N] [-config M.cfg] [-json] [-v] M.tla\n");
    return 2;
  }
  char err[512];
  rmc_model* m = nullptr;
  if (rmc_model_load(tla.c_str(), cfg.empty() ? nullptr : cfg.c_str(), &m, err, sizeof err) != 0) {
    fprintf(stderr, "raftmc: %s\n", err);
    return 1;
  }
  printf("raftmc %s: model checking %s\n", rmc_version(), tla.c_str());
  rmc_result r;
  int rc = rmc_check(m, &o, &r);
  if (rc != 0) {
    fprintf(stderr, "raftmc: %s\n", rmc_last_error());
    rmc_model_free(m);
    return 1;
  }
  printf("Finished computing initial states: 1 distinct state generated.\n");
  std::vector<char> buf(1 << 22);
  rmc_format_report(m, &r, buf.data(), buf.size());
  fputs(buf.data(), stdout);
  printf("Finished in %.3fs\n", r.seconds);
  if (json)
    printf("{\"generated\":%llu,\"distinct\":%llu,\"depth\":%u,\"left\":%llu,\"status\":%d,\"violated\":\"%s\","
           "\"seconds\":%.6f,\"expand_ms\":%.3f,\"mark_ms\":%.3f,\"materialize_ms\":%.3f}\n",
           (unsigned long long)r.generated, (unsigned long long)r.distinct, r.depth,
           (unsigned long long)r.left_on_queue, r.status, r.violated, r.seconds, r.expand_ms, r.mark_ms,
           r.materialize_ms);
  rmc_model_free(m);
  return r.status == 0 ? 0 : (r.status == 1 ? 12 : 13);
}
