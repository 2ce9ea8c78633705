/*
 * rmc.h — C ABI of librmc.so, the MI355X-native explicit-state model checker
 * for the Raft TLA+ specifications of Vanlightly/raft-tlaplus.
 *
 * What it replaces.  The reference has no code of its own on this path: its
 * specs are run by TLC, invoked as
 *     java -cp tla2tools.jar tlc2.TLC -deadlock [-workers N] [-config M.cfg] M.tla
 * (README.md:6 "run all these specifications with the -deadlock argument").
 * Each entry point below maps to one step of that contract:
 *   rmc_model_load   <- TLC reading M.tla + M.cfg (SANY parse, constant binding,
 *                       INIT/NEXT/VIEW/SYMMETRY/INVARIANT), e.g.
 *                       specifications/standard-raft/Raft.cfg:5-36 bound to
 *                       specifications/standard-raft/Raft.tla:1-638
 *   rmc_check        <- the model-checking run (BFS over Init/Next, Raft.tla:213,527),
 *                       producing TLC's "<G> states generated, <D> distinct states
 *                       found, <Q> states left on queue" and "depth <d>" lines
 *   rmc_trace_len /
 *   rmc_trace_state  <- TLC's "Error: The behavior up to this point is:" block
 *                       (State k: /\ var = value) after an invariant violation
 *                       (invariants Raft.tla:588-620, listed at Raft.cfg:34-36)
 *   rmc_model_free   <- end of run
 * Modules: Raft, FlexibleRaft, RaftFsync, PullRaft, PullRaftVariant2 and KRaft
 * (specifications/pull-raft/KRaft.tla, e.g. with pull-raft/KRaft.cfg:5-50).
 * Plain pointers and sizes only; no torch or HIP types cross this boundary.
 *
 * Ownership: the caller owns rmc_options, rmc_result and text buffers; the
 * library owns the model, device memory and the trace until rmc_model_free.
 * Errors: a negative return is an API/IO error with a message in `err` (or
 * rmc_last_error()); model outcomes are reported in rmc_result.status.
 * Threading: rmc_check is blocking and not re-entrant per model.
 */
#ifndef RMC_H
#define RMC_H
#include <stddef.h>
#include <stdint.h>
#ifdef __cplusplus
extern "C" {
#endif

typedef struct rmc_model rmc_model; /* lowered spec + cfg; library-owned */

typedef struct {
  int n_gpus;          /* GPUs rmc_check uses (default 1).  > 1: the fingerprint-sharded search over GPUs
                          0..n_gpus-1 of this process, one host thread per GPU (rmc_check_multi, RCCL);
                          more than the visible GPUs is an error (-4), never a silent 1-GPU run */
  int cpu_workers;     /* accepted for TLC CLI compatibility (-workers); unused by the GPU path */
  int deadlock_check;  /* 0 = TLC -deadlock (the reference's mode); 1 is rejected */
  int fp_bits;         /* 64 (default, TLC's width) or 128 (rmc_check only): the first 64 bits are the
                          64-bit fingerprint, the rest an independent hash of the same canonical view */
  int tlc_order;       /* 1 (default): first successor in TLC order wins per fingerprint */
  uint64_t hash_slots; /* initial fingerprint-set capacity, main tier (power of two; grows on demand); 0 = auto */
  uint32_t msg_cap_K;  /* message slots per packed state; 0 = auto */
  uint64_t frontier_cap; /* max states per BFS level; 0 = auto */
  uint32_t chunk_parents; /* parents expanded per launch; 0 = auto */
  int verbose;         /* per-level progress on stderr */
  int max_depth;       /* stop after this many levels (0 = exhaustive) */
  int grow_on_overflow; /* test: no fingerprint-set growth ahead of a chunk; a chunk that overflows the set
                           grows it and is redone (the safety net behind the pre-sizing) */
  double time_limit;    /* stop (status 4) at the first level boundary after this many seconds (0 = none) */
  /* TLC's -checkpoint / -recover (its states/ directory, reference .gitignore:1): rmc_check snapshots the
   * search -- fingerprint set, the next level's frontier, trace records, counts -- into checkpoint_dir at
   * the first level boundary checkpoint_minutes after the last snapshot (0 = every level), and resumes
   * from the snapshot in recover_dir (same model and constants; verified).  NULL = off. */
  const char* checkpoint_dir;
  double checkpoint_minutes;
  const char* recover_dir;
  /* BFS levels in pinned host memory (SURVEY.md §7 hard part 5): the current and next level's packed states
   * live in host RAM and stream through HBM in chunk-sized windows, so the fingerprint set may take the
   * whole device.  0 = auto (at a level boundary when the next level is projected past a quarter of HBM, or
   * when HBM runs out), 1 = always, -1 = never (rmc_check only; host memory capped by RMC_HOST_FRONTIER_GIB). */
  int host_frontier;
} rmc_options;

typedef struct {
  uint64_t generated, distinct, left_on_queue;
  uint32_t depth;
  int status; /* 0 ok, 1 invariant violated, 2 evaluation error, 3 capacity overflow, 4 stopped (max_depth, time_limit) */
  char violated[64];
  uint64_t hidden_var_collisions; /* same-level duplicates whose VIEW-hidden variables (acked, electionCtr,
                                     restartCtr; Pull: the counters) differ from the first-in-TLC-order winner's
                                     (SURVEY.md §7 hard part 1); equal to the oracle's hidden_same_level */
  double seconds;
  /* everything below extends SURVEY.md §8b's rmc_result, whose fields above keep its order and offsets */
  char message[256];    /* evaluation-error / capacity text (TLC's error message), "" otherwise */
  /* measurement (filled by rmc_check) */
  double expand_ms, mark_ms, materialize_ms; /* summed device time per kernel family */
  uint64_t expand_launches;
  uint32_t state_bytes; /* packed frontier state size */
  uint32_t max_msgs;    /* largest |DOMAIN messages| seen */
  uint64_t hash_capacity;
  uint64_t device_bytes; /* HBM held by the check's buffers at its end (they only grow within a check): the
                            single-GPU search's total; the sharded search's largest shard on this process */
} rmc_result;

/* Load M.tla + M.cfg, as TLC reads them (`tlc2.TLC -config M.cfg M.tla`; a
 * path without ".tla" gets it appended; the module is its basename; cfg_path
 * NULL = M.cfg beside it).  A .tla whose text (comments and whitespace aside)
 * is a reference module's uses that module's action table directly; any other
 * text goes through the TLA+ front end (rmc_tla.cpp): the module
 * is parsed, its Next decomposed into disjuncts, and each disjunct lowered --
 * matched by closure hash onto the action library, or compiled from its body
 * where the front end compiles that form -- and refused, with the disjunct
 * named, when neither applies.  Returns 0, or -3 when a file cannot be read,
 * -2 when the spec or cfg is rejected. */
int rmc_model_load(const char* tla_path, const char* cfg_path, rmc_model** out, char* err, size_t errlen);
/* The built-in lowering of `module` bound to in-memory cfg text (no .tla needed). */
int rmc_model_load_text(const char* module, const char* cfg_text, rmc_model** out, char* err, size_t errlen);
void rmc_options_default(rmc_options* o);
int rmc_check(rmc_model* m, const rmc_options* o, rmc_result* out); /* blocking */
int rmc_trace_len(const rmc_model* m);                               /* after status 1/2 */
int rmc_trace_state(const rmc_model* m, int k, char* tla_text, size_t len); /* TLC value syntax */
int rmc_trace_action(const rmc_model* m, int k, char* text, size_t len);   /* "Initial predicate" / action label */
/* TLC's -dumpTrace, after status 1/2.  rmc_trace_module writes a TLA+ module
 * `name` that EXTENDS the checked spec, holds the error behaviour as
 * TraceStates == << [var |-> value, ...], ... >> and replays it with the spec's
 * own Init/Next (TraceInit/TraceNext), plus its companion cfg (the model's
 * constants, INVARIANT TraceAccepted): TLC on the pair must report
 * "Invariant TraceAccepted is violated" (the whole trace is a behaviour).
 * rmc_trace_json writes the same behaviour as JSON.  Return the text length
 * (the buffers get a truncated, NUL-terminated copy), or -1. */
int rmc_trace_module(const rmc_model* m, const char* name, char* tla, size_t tla_len, char* cfg, size_t cfg_len);
int rmc_trace_json(const rmc_model* m, char* buf, size_t len);
/* Print the TLC-format report for a finished check into buf. */
int rmc_format_report(const rmc_model* m, const rmc_result* r, char* buf, size_t len);
void rmc_model_free(rmc_model* m);
/* Free the device buffers librmc keeps per GPU between checks (fingerprint set,
 * frontiers, trace records).  They are otherwise reused by the next check. */
void rmc_release_device_memory(void);
const char* rmc_last_error(void);
const char* rmc_version(void);
/* Layout version of rmc_options / rmc_result.  2 (r04): rmc_result.message moved after `seconds` (SURVEY
 * §8b's fields first, in its order) and device_bytes appended.  A binding built against another version must
 * refuse the library; rmc_abi_layout gives the offsets themselves. */
#define RMC_ABI_VERSION 2
int rmc_abi_version(void);
/* Fingerprint-sharded search.  One process per GPU: rank 0
 * calls rmc_comm_unique_id, the 128-byte id is broadcast out of band (e.g.
 * torch.distributed), then every rank calls rmc_check_sharded with its rank,
 * the world size and its GPU; shards exchange over RCCL (xGMI).  Every rank
 * receives the same global result.  rmc_check_logical runs `shards` logical
 * shards of the same protocol in this process on its current GPU (the
 * transport is device copies) -- the multi-GPU path without a cluster. */
int rmc_comm_unique_id(unsigned char* id128);
int rmc_check_sharded(rmc_model* m, const rmc_options* o, int rank, int world, int device, const unsigned char* id128,
                      rmc_result* out);
int rmc_check_logical(rmc_model* m, const rmc_options* o, int shards, rmc_result* out);
/* The in-process multi-GPU check that rmc_check runs for n_gpus > 1 (SURVEY.md
 * §8b: "one host thread per GPU"): shard r on devices[r], one host thread and
 * stream per shard, the protocol of rmc_check_sharded.  transport
 * RMC_XPORT_RCCL: an in-process RCCL communicator (ncclCommInitAll) over xGMI,
 * devices distinct; RMC_XPORT_P2P: the threads pull their peers' buffers with
 * peer device copies behind host barriers -- any device list, including
 * several shards on one GPU (how a one-GPU host tests the threaded driver).
 * rmc_check's choice is RCCL (RMC_MGPU_TRANSPORT=p2p selects peer copies).
 * Every shard computes the global result; shard 0's lands in *out and m. */
#define RMC_XPORT_RCCL 0
#define RMC_XPORT_P2P 1
int rmc_check_multi(rmc_model* m, const rmc_options* o, const int* devices, int n, int transport, rmc_result* out);
/* The same multi-process protocol as rmc_check_sharded with POSIX shared
 * memory (segment `shm_name`, created by the ranks) as the transport instead
 * of RCCL: one process per shard on one host, any GPUs -- including several
 * processes on ONE GPU, which RCCL refuses.  For testing the multi-rank path
 * and for hosts without xGMI peers; world <= 16. */
int rmc_check_sharded_shm(rmc_model* m, const rmc_options* o, int rank, int world, int device, const char* shm_name,
                          rmc_result* out);
/* TLC's random simulation mode (-simulate): rounds of `walkers` random
 * behaviours in parallel on the GPU, each from Init for at most `depth` steps
 * (a uniformly random enabled successor per step), invariants checked on every
 * state, until `behaviors` behaviours are done, `seconds` pass (0 = no limit)
 * or a violation / evaluation error is found (its behaviour is then available
 * through rmc_trace_*).  Results: generated = states generated, distinct =
 * behaviours generated, depth = longest behaviour in states, status as for
 * rmc_check.  The same seed gives the same run (a time limit aside): every
 * behaviour of a round runs to its end and a failure reports the round's
 * lowest-index failing behaviour. */
int rmc_simulate(rmc_model* m, const rmc_options* o, uint64_t walkers, uint32_t depth, uint64_t seed,
                 uint64_t behaviors, double seconds, rmc_result* out);
/* The CPU engine: TLC's -workers N on host threads (o->cpu_workers; 0 = every hardware thread), over the
 * same packed layout, lowered actions, fingerprint and first-in-TLC-order rule as rmc_check, with the same
 * results.  Explicitly requested (raftmc -cpu); rmc_check never falls back to it.  BASELINE.md's CPU baseline. */
int rmc_check_cpu(rmc_model* m, const rmc_options* o, rmc_result* out);
/* Where the last rmc_check's wall time went, as a JSON object of seconds:
 * hip_init (the process's first check only: runtime + device context),
 * model_upload, buffers (allocation and VMM mapping of the arena), launch_enqueue
 * (host time inside kernel launch calls -- a fresh process loads the code
 * objects there), table_growth, buffer_growth, widening, host_frontier, kernels
 * (summed device time) and total.  Returns the text length, or -1. */
int rmc_check_phases(const rmc_model* m, char* json, size_t len);
/* Per-level counts of the last check: fills up to cap pairs (generated, new) and returns the level count. */
int rmc_levels(const rmc_model* m, uint64_t* gen_new_pairs, int cap);
/* Next as a list of disjuncts: comma-separated operator names of the spec
 * family's definitions, in Next order (e.g. Raft's "Restart, RequestVote, ...,
 * HandleAppendEntriesResponse, DuplicateMessage"): the action table a module
 * whose Next lists exactly those disjuncts lowers to through the TLA+ front
 * end -- reordered, reduced or with the network actions
 * Raft.tla:540-541 leaves commented out.  For models loaded without a .tla
 * (rmc_model_load_text).  Returns 0, or a negative value (unknown name;
 * rmc_last_error()).  rmc_model_next writes the model's current Next the same
 * way and returns its length. */
int rmc_model_set_next(rmc_model* m, const char* disjuncts);
/* The guard of one of Next's simple actions (Restart, RequestVote, Timeout,
 * BecomeLeader, ClientRequest) as TLA+ expression text over the state
 * variables, the cfg's constants and the action's parameters (`params`, e.g.
 * "i" or "i, v"), with the family's Quorum and LastTerm in scope -- what a
 * module whose action keeps the reference body but states another guard
 * lowers to through the TLA+ front end (the reference's effect runs behind
 * the compiled guard; rmc_guard.cpp).  E.g. rmc_model_set_guard(m,
 * "RequestVote", "i", "electionCtr <= MaxElections /\ state[i] = Follower").
 * Returns 0, or a negative value (rmc_last_error()). */
int rmc_model_set_guard(rmc_model* m, const char* action, const char* params, const char* expr);
/* Define an action by its TLA+ text, for rmc_model_set_next to put in Next by
 * `name`: `name(params) == body`, read beside the spec family's VARIABLES,
 * their groupings (serverVars, logVars, ...), Quorum, LastTerm and send
 * helpers, and compiled whole -- its guard and its effect (rmc_guard.cpp
 * compile_effect; Raft, FlexibleRaft, RaftFsync; 64-bit fingerprints).
 * `form` is the binding: 0 \E i \in Server, 1 \E i \in Server, v \in Value,
 * 2 \E i, j \in Server.  The same as a module whose Next has a disjunct with
 * that body (rmc_model_load).  Returns 0, or -2 naming what it cannot
 * compile (rmc_last_error). */
int rmc_model_define_action(rmc_model* m, const char* name, int form, const char* params, const char* body);
int rmc_model_next(const rmc_model* m, char* out, size_t len);
/* The TLA+ front end's structural hashes of a module's definitions (the
 * closure hashes the lowering matches against its action library; used by
 * tools/gen_tla_known.py): writes "#module M", "#vars <hash>", then one
 * "name <hash>" line per definition into out and returns the text length,
 * or a negative value with the parse error in out. */
int rmc_tla_hashes(const char* tla_text, char* out, size_t len);
/* "<hash>:<file>,<file>,...": the first 32 hex digits of the SHA-256 of the
 * listed source files (paths relative to raft-tlaplus_amd/), concatenated in
 * that order, as the library was built from them.  A binding compares it with
 * the tree's sources to refuse a stale build (raftmc.lib()). */
const char* rmc_source_id(void);
/* ABI self-description for binding checks (ctypes, JNA): fills up to cap values -- sizeof(rmc_options),
 * the offset of each of its fields in declaration order, then sizeof(rmc_result) and its field offsets --
 * and returns how many there are. */
int rmc_abi_layout(uint64_t* out, int cap);

#ifdef __cplusplus
}
#endif
#endif /* RMC_H */
