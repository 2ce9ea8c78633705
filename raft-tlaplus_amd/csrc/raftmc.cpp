// raftmc — TLC-compatible command line over librmc:
//   raftmc [-deadlock] [-workers N] [-config M.cfg] [-json] [-v] M.tla
// mirrors `java tlc2.TLC -deadlock [-workers N] [-config M.cfg] M.tla`
// (reference README.md:6) and prints TLC's result lines.  As TLC, it reads
// M.tla (which must be the reference's text of a supported module);
//   raftmc -module M -config X.cfg ...
// checks the built-in lowering of module M against X.cfg without the .tla.
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>
#include "../../include/rmc.h"

// -dumpTrace tla FILE: FILE (module named after its basename) + the companion
// cfg beside it; -dumpTrace json FILE: the behaviour as JSON.
static int dump_trace(rmc_model* m, const std::string& fmt, const std::string& file) {
  if (rmc_trace_len(m) <= 0) return 0;
  std::vector<char> a(1 << 24), c(1 << 16);
  std::string path = file, cfgpath;
  if (fmt == "tla") {
    if (path.size() < 4 || path.compare(path.size() - 4, 4, ".tla") != 0) path += ".tla";
    std::string base = path.substr(0, path.size() - 4);
    size_t sl = base.find_last_of('/');
    std::string name = sl == std::string::npos ? base : base.substr(sl + 1);
    if (rmc_trace_module(m, name.c_str(), a.data(), a.size(), c.data(), c.size()) < 0) return 1;
    cfgpath = base + ".cfg";
  } else if (rmc_trace_json(m, a.data(), a.size()) < 0) {
    return 1;
  }
  FILE* f = fopen(path.c_str(), "w");
  if (!f) { fprintf(stderr, "raftmc: cannot write %s\n", path.c_str()); return 1; }
  fputs(a.data(), f);
  fclose(f);
  if (!cfgpath.empty()) {
    FILE* g = fopen(cfgpath.c_str(), "w");
    if (!g) { fprintf(stderr, "raftmc: cannot write %s\n", cfgpath.c_str()); return 1; }
    fputs(c.data(), g);
    fclose(g);
  }
  printf("The error trace was written to %s%s%s\n", path.c_str(), cfgpath.empty() ? "" : " and ", cfgpath.c_str());
  return 0;
}

int main(int argc, char** argv) {
  rmc_options o;
  rmc_options_default(&o);
  o.deadlock_check = 1;  // TLC default; the reference always passes -deadlock
  std::string tla, cfg, module;
  bool json = false, simulate = false, cpu = false;
  int shards = 0;  // > 0: the fingerprint-sharded protocol with this many logical shards on one GPU
  std::string metadir, recover;
  std::string dump_fmt, dump_file;
  unsigned long long sim_walkers = 1ULL << 20, sim_num = 0, sim_seed = 0;
  unsigned sim_depth = 100;
  std::string next_ops;
  double sim_seconds = 0;
  for (int a = 1; a < argc; a++) {
    std::string k = argv[a];
    auto val = [&]() -> std::string {
      if (a + 1 >= argc) { fprintf(stderr, "missing value for %s\n", k.c_str()); exit(2); }
      return argv[++a];
    };
    if (k == "-deadlock") o.deadlock_check = 0;
    else if (k == "-workers") o.cpu_workers = atoi(val().c_str());
    else if (k == "-config") cfg = val();
    else if (k == "-module") module = val();
    else if (k == "-gpus") o.n_gpus = atoi(val().c_str());
    else if (k == "-msgcap") o.msg_cap_K = (uint32_t)atoi(val().c_str());
    else if (k == "-hashslots") o.hash_slots = strtoull(val().c_str(), nullptr, 10);
    else if (k == "-hostfrontier") o.host_frontier = atoi(val().c_str());  // -1 never, 0 auto, 1 always
    else if (k == "-maxdepth") o.max_depth = atoi(val().c_str());
    else if (k == "-chunk") o.chunk_parents = (uint32_t)atoi(val().c_str());
    else if (k == "-simulate") simulate = true;
    else if (k == "-cpu") cpu = true;
    else if (k == "-shards") shards = atoi(val().c_str());
    else if (k == "-checkpoint") o.checkpoint_minutes = atof(val().c_str());  // TLC: minutes between checkpoints
    else if (k == "-metadir") metadir = val();                                 // TLC: where states/ go
    else if (k == "-recover") recover = val();
    else if (k == "-fpwidth") o.fp_bits = atoi(val().c_str());  // 64 (TLC's) or 128
    else if (k == "-depth") sim_depth = (unsigned)atoi(val().c_str());
    else if (k == "-num") sim_num = strtoull(val().c_str(), nullptr, 10);
    else if (k == "-seed") sim_seed = strtoull(val().c_str(), nullptr, 10);
    else if (k == "-walkers") sim_walkers = strtoull(val().c_str(), nullptr, 10);
    else if (k == "-seconds") sim_seconds = atof(val().c_str());
    else if (k == "-json") json = true;
    else if (k == "-dumpTrace") {
      dump_fmt = val();
      dump_file = val();
      if (dump_fmt != "tla" && dump_fmt != "json") { fprintf(stderr, "raftmc: -dumpTrace tla|json FILE\n"); return 2; }
    }
    else if (k == "-v") o.verbose = 1;
    else if (k == "-next") next_ops = val();  // Next as disjunct names (with -module): the front end's form
    else if (!k.empty() && k[0] == '-') { fprintf(stderr, "raftmc: unknown option %s\n", k.c_str()); return 2; }
    else tla = k;
  }
  if (tla.empty() == module.empty() || (!module.empty() && cfg.empty())) {
    fprintf(stderr, "usage: raftmc [-deadlock] [-workers N] [-cpu] [-shards W] [-fpwidth 64|128] [-hostfrontier -1|0|1] [-checkpoint MIN] [-metadir DIR] [-recover DIR] [-config M.cfg] [-maxdepth D] [-dumpTrace tla|json FILE] [-json] [-v] M.tla\n"
                    "       raftmc [options] -module M -config X.cfg [-next \"A, B, ...\"]   (module M's lowering, no .tla)\n"
                    "       raftmc -simulate [-depth D] [-num BEHAVIOURS] [-seed S] [-walkers W] [-seconds T] ...\n");
    return 2;
  }
  char err[512];
  rmc_model* m = nullptr;
  if (!module.empty()) {
    FILE* f = fopen(cfg.c_str(), "rb");
    if (!f) { fprintf(stderr, "raftmc: cannot read cfg file %s\n", cfg.c_str()); return 1; }
    std::string text;
    char b[4096];
    for (size_t n; (n = fread(b, 1, sizeof b, f)) > 0;) text.append(b, n);
    fclose(f);
    if (rmc_model_load_text(module.c_str(), text.c_str(), &m, err, sizeof err) != 0) {
      fprintf(stderr, "raftmc: %s\n", err);
      return 1;
    }
    tla = module + " (built-in lowering)";
    if (!next_ops.empty() && rmc_model_set_next(m, next_ops.c_str()) != 0) {
      fprintf(stderr, "raftmc: %s\n", rmc_last_error());
      return 1;
    }
  } else if (rmc_model_load(tla.c_str(), cfg.empty() ? nullptr : cfg.c_str(), &m, err, sizeof err) != 0) {
    fprintf(stderr, "raftmc: %s\n", err);
    return 1;
  }
  rmc_result r;
  if (simulate) {
    printf("raftmc %s: random simulation of %s, seed %llu, %llu walkers, depth %u\n", rmc_version(), tla.c_str(),
           sim_seed, sim_walkers, sim_depth);
    int rc = rmc_simulate(m, &o, sim_walkers, sim_depth, sim_seed, sim_num ? sim_num : sim_walkers, sim_seconds, &r);
    if (rc != 0) {
      fprintf(stderr, "raftmc: %s\n", rmc_last_error());
      rmc_model_free(m);
      return 1;
    }
    if (r.status == 1 || r.status == 2) {
      std::vector<char> buf(1 << 22);
      rmc_result rr = r;
      rr.generated = 0;
      rmc_format_report(m, &rr, buf.data(), buf.size());
      std::string s(buf.data());
      size_t cut = s.find(" states generated");
      if (cut != std::string::npos) s = s.substr(0, s.rfind('\n', cut) + 1);
      fputs(s.c_str(), stdout);
      if (!dump_fmt.empty()) dump_trace(m, dump_fmt, dump_file);
    }
    printf("The number of states generated: %llu\n", (unsigned long long)r.generated);
    printf("Simulation using seed %llu generated %llu behaviours (longest %u states)\n", sim_seed,
           (unsigned long long)r.distinct, r.depth);
    printf("Finished in %.3fs\n", r.seconds);
    rmc_model_free(m);
    return r.status == 0 ? 0 : (r.status == 1 ? 12 : 13);
  }
  // TLC takes a checkpoint every 30 minutes into <metadir>/ by default; here
  // snapshots are taken when -checkpoint or -metadir is given
  if (!metadir.empty() || o.checkpoint_minutes > 0) {
    if (metadir.empty()) metadir = "states";
    o.checkpoint_dir = metadir.c_str();
  }
  if (!recover.empty()) o.recover_dir = recover.c_str();
  printf("raftmc %s: model checking %s\n", rmc_version(), tla.c_str());
  int rc = cpu ? rmc_check_cpu(m, &o, &r) : shards > 0 ? rmc_check_logical(m, &o, shards, &r) : rmc_check(m, &o, &r);
  if (rc != 0) {
    fprintf(stderr, "raftmc: %s\n", rmc_last_error());
    rmc_model_free(m);
    return 1;
  }
  printf("Finished computing initial states: 1 distinct state generated.\n");
  std::vector<char> buf(1 << 22);
  rmc_format_report(m, &r, buf.data(), buf.size());
  fputs(buf.data(), stdout);
  if (!dump_fmt.empty() && (r.status == 1 || r.status == 2)) dump_trace(m, dump_fmt, dump_file);
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
