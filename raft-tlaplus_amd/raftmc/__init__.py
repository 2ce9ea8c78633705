"""raftmc — Python binding of librmc (ctypes over include/rmc.h).

Mirrors the reference's operator interface for this path, which is TLC's
command line: `tlc2.TLC -deadlock [-workers N] [-config M.cfg] M.tla`
(/root/reference/README.md:6).  `check(tla, cfg)` returns TLC's three counts
(states generated, distinct states, depth), the states left on the queue,
and on an invariant violation the invariant name and the behaviour (a list of
(action label, TLA+ state text)) as TLC prints it.

The HIP path is the only path: if librmc.so is missing or no GPU is present,
calls fail loudly (RaftmcError); there is no CPU fallback.
"""
import ctypes
import hashlib
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
# RAFTMC_BUILD=<dir under raft-tlaplus_amd/>: load an in-tree variant build
# (A/B measurements); the default is build/
LIB_PATH = os.path.join(os.path.dirname(_HERE), os.environ.get("RAFTMC_BUILD", "build"), "librmc.so")

STATUS = {0: "ok", 1: "violation", 2: "error", 3: "capacity", 4: "stopped"}


class RaftmcError(RuntimeError):
    pass


class Options(ctypes.Structure):
    _fields_ = [("n_gpus", ctypes.c_int), ("cpu_workers", ctypes.c_int),
                ("deadlock_check", ctypes.c_int), ("fp_bits", ctypes.c_int),
                ("tlc_order", ctypes.c_int), ("hash_slots", ctypes.c_uint64),
                ("msg_cap_K", ctypes.c_uint32), ("frontier_cap", ctypes.c_uint64),
                ("chunk_parents", ctypes.c_uint32), ("verbose", ctypes.c_int),
                ("max_depth", ctypes.c_int), ("grow_on_overflow", ctypes.c_int),
                ("time_limit", ctypes.c_double), ("checkpoint_dir", ctypes.c_char_p),
                ("checkpoint_minutes", ctypes.c_double), ("recover_dir", ctypes.c_char_p),
                ("host_frontier", ctypes.c_int)]


class Result(ctypes.Structure):
    _fields_ = [("generated", ctypes.c_uint64), ("distinct", ctypes.c_uint64),
                ("left_on_queue", ctypes.c_uint64), ("depth", ctypes.c_uint32),
                ("status", ctypes.c_int), ("violated", ctypes.c_char * 64),
                ("hidden_var_collisions", ctypes.c_uint64), ("seconds", ctypes.c_double),
                ("message", ctypes.c_char * 256),
                ("expand_ms", ctypes.c_double), ("mark_ms", ctypes.c_double),
                ("materialize_ms", ctypes.c_double), ("expand_launches", ctypes.c_uint64),
                ("state_bytes", ctypes.c_uint32), ("max_msgs", ctypes.c_uint32),
                ("hash_capacity", ctypes.c_uint64), ("device_bytes", ctypes.c_uint64)]


# every entry point include/rmc.h declares (checked by tests/test_abi.py)
EXPORTS = ["rmc_model_load", "rmc_model_load_text", "rmc_options_default", "rmc_check",
           "rmc_trace_len", "rmc_trace_state", "rmc_trace_action", "rmc_format_report",
           "rmc_model_free", "rmc_last_error", "rmc_version", "rmc_levels",
           "rmc_release_device_memory", "rmc_comm_unique_id", "rmc_check_sharded", "rmc_check_logical",
           "rmc_simulate", "rmc_trace_module", "rmc_trace_json", "rmc_check_cpu", "rmc_check_sharded_shm",
           "rmc_abi_layout", "rmc_abi_version", "rmc_model_set_next", "rmc_model_next", "rmc_tla_hashes",
           "rmc_model_set_guard", "rmc_source_id", "rmc_model_define_action", "rmc_check_multi",
           "rmc_check_phases"]

# rmc_check_multi transports (include/rmc.h)
XPORT_RCCL, XPORT_P2P = 0, 1

# the rmc_options / rmc_result layout these ctypes mirrors follow (include/rmc.h RMC_ABI_VERSION)
ABI_VERSION = 2

_lib = None


def source_mismatch(source_id):
    """Compare a library's rmc_source_id with the tree's sources: None when they
    match, else a short reason (the sources are raft-tlaplus_amd/-relative)."""
    digest, _, files = source_id.partition(":")
    h = hashlib.sha256()
    base = os.path.dirname(_HERE)
    for f in files.split(","):
        try:
            with open(os.path.join(base, f), "rb") as fh:
                h.update(fh.read())
        except OSError:
            return "source %s is missing" % f
    return None if h.hexdigest()[:32] == digest else "source hash %s, tree %s" % (digest, h.hexdigest()[:32])


def refuse_stale(source_id):
    """Raise unless the library's sources (rmc_source_id) are the tree's."""
    stale = source_mismatch(source_id)
    if stale and os.environ.get("RAFTMC_ALLOW_STALE") != "1":
        raise RaftmcError("%s was built from other sources than the tree's (%s): rebuild it "
                          "(make -C raft-tlaplus_amd OUT=%s)" % (LIB_PATH, stale, os.environ.get("RAFTMC_BUILD", "build")))


def lib():
    """Load librmc.so (built in-tree by `make -C raft-tlaplus_amd`)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise RaftmcError("librmc.so not built: run `make -C raft-tlaplus_amd` (expected %s)" % LIB_PATH)
    L = ctypes.CDLL(LIB_PATH)
    P, c_int, c_size_t = ctypes.c_void_p, ctypes.c_int, ctypes.c_size_t
    L.rmc_model_load.argtypes = [ctypes.c_char_p, ctypes.c_char_p, ctypes.POINTER(P), ctypes.c_char_p, c_size_t]
    L.rmc_model_load_text.argtypes = [ctypes.c_char_p, ctypes.c_char_p, ctypes.POINTER(P), ctypes.c_char_p, c_size_t]
    L.rmc_options_default.argtypes = [ctypes.POINTER(Options)]
    L.rmc_check.argtypes = [P, ctypes.POINTER(Options), ctypes.POINTER(Result)]
    L.rmc_trace_len.argtypes = [P]
    L.rmc_trace_state.argtypes = [P, c_int, ctypes.c_char_p, c_size_t]
    L.rmc_trace_action.argtypes = [P, c_int, ctypes.c_char_p, c_size_t]
    L.rmc_format_report.argtypes = [P, ctypes.POINTER(Result), ctypes.c_char_p, c_size_t]
    L.rmc_model_free.argtypes = [P]
    L.rmc_last_error.restype = ctypes.c_char_p
    L.rmc_version.restype = ctypes.c_char_p
    L.rmc_levels.argtypes = [P, ctypes.POINTER(ctypes.c_uint64), c_int]
    L.rmc_abi_layout.argtypes = [ctypes.POINTER(ctypes.c_uint64), c_int]
    if L.rmc_abi_version() != ABI_VERSION:
        raise RaftmcError("librmc.so has ABI version %d; this binding mirrors version %d (rebuild one of them)"
                          % (L.rmc_abi_version(), ABI_VERSION))
    L.rmc_source_id.restype = ctypes.c_char_p
    # a library built from other sources than the tree's is refused, default
    # build included: a forgotten rebuild would otherwise put
    # stale kernels behind green tests.  RAFTMC_ALLOW_STALE=1 overrides it for
    # a deliberate experiment.
    refuse_stale(L.rmc_source_id().decode())
    L.rmc_model_set_next.argtypes = [P, ctypes.c_char_p]
    L.rmc_model_set_guard.argtypes = [P, ctypes.c_char_p, ctypes.c_char_p, ctypes.c_char_p]
    L.rmc_model_define_action.argtypes = [P, ctypes.c_char_p, ctypes.c_int, ctypes.c_char_p, ctypes.c_char_p]
    L.rmc_model_next.argtypes = [P, ctypes.c_char_p, c_size_t]
    L.rmc_tla_hashes.argtypes = [ctypes.c_char_p, ctypes.c_char_p, c_size_t]
    L.rmc_comm_unique_id.argtypes = [ctypes.c_char_p]
    L.rmc_check_sharded.argtypes = [P, ctypes.POINTER(Options), c_int, c_int, c_int, ctypes.c_char_p,
                                    ctypes.POINTER(Result)]
    L.rmc_check_logical.argtypes = [P, ctypes.POINTER(Options), c_int, ctypes.POINTER(Result)]
    L.rmc_check_multi.argtypes = [P, ctypes.POINTER(Options), ctypes.POINTER(c_int), c_int, c_int,
                                  ctypes.POINTER(Result)]
    L.rmc_selftest_hf_stats.argtypes = [P, ctypes.POINTER(ctypes.c_uint64)]
    L.rmc_check_phases.argtypes = [P, ctypes.c_char_p, c_size_t]
    L.rmc_check_sharded_shm.argtypes = [P, ctypes.POINTER(Options), c_int, c_int, c_int, ctypes.c_char_p,
                                        ctypes.POINTER(Result)]
    L.rmc_check_cpu.argtypes = [P, ctypes.POINTER(Options), ctypes.POINTER(Result)]
    L.rmc_simulate.argtypes = [P, ctypes.POINTER(Options), ctypes.c_uint64, ctypes.c_uint32, ctypes.c_uint64,
                               ctypes.c_uint64, ctypes.c_double, ctypes.POINTER(Result)]
    L.rmc_selftest_host_bfs.argtypes = [P, ctypes.c_uint32, ctypes.c_uint64,
                                        ctypes.POINTER(ctypes.c_uint64), ctypes.POINTER(ctypes.c_uint64), c_int]
    L.rmc_trace_module.argtypes = [P, ctypes.c_char_p, ctypes.c_char_p, c_size_t, ctypes.c_char_p, c_size_t]
    L.rmc_trace_json.argtypes = [P, ctypes.c_char_p, c_size_t]
    L.rmc_selftest_random_trace.argtypes = [P, ctypes.c_uint64, c_int]
    L.rmc_selftest_set_hint_kmax.argtypes = [P, ctypes.c_uint32]
    L.rmc_selftest_widenings.argtypes = [P, ctypes.POINTER(ctypes.c_uint64), c_int]
    L.rmc_selftest_profile_expand.argtypes = [P, ctypes.POINTER(Options), c_int, ctypes.POINTER(ctypes.c_double), c_int]
    L.rmc_selftest_encode_msg.argtypes = [c_int, ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_uint32)]
    L.rmc_selftest_encode_kmsg.argtypes = [ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_uint32)]
    _lib = L
    return L


class Model:
    """A spec + cfg loaded into librmc (TLC's parse/bind step)."""

    def __init__(self, tla_path=None, cfg_path=None, module=None, cfg_text=None):
        """Model("M.tla", "M.cfg") reads both files, as TLC does (the .tla must be
        the reference's text of a supported module).  Model(module="M",
        cfg_text=...) or Model(module="M", cfg_path="X.cfg") binds the built-in
        lowering of module M to a cfg without a .tla."""
        L = lib()
        err = ctypes.create_string_buffer(512)
        h = ctypes.c_void_p()
        if tla_path is None and cfg_text is None and module is not None and cfg_path is not None:
            try:
                with open(cfg_path) as f:
                    cfg_text = f.read()
            except OSError as e:
                raise RaftmcError("cannot read cfg file %s (%s)" % (cfg_path, e.strerror))
        if cfg_text is not None:
            rc = L.rmc_model_load_text(module.encode(), cfg_text.encode(), ctypes.byref(h), err, 512)
        else:
            rc = L.rmc_model_load(tla_path.encode(), cfg_path.encode() if cfg_path else None,
                                  ctypes.byref(h), err, 512)
        if rc != 0:
            raise RaftmcError(err.value.decode())
        self._h = h

    def __del__(self):
        if getattr(self, "_h", None) and _lib is not None:
            _lib.rmc_model_free(self._h)
            self._h = None

    def _options(self, deadlock=False, hash_slots=0, msg_cap_K=0, frontier_cap=0,
                 chunk_parents=0, verbose=False, max_depth=0, workers=0, grow_on_overflow=False,
                 time_limit=0.0, fp_bits=64, checkpoint_dir=None, checkpoint_minutes=0.0, recover_dir=None,
                 host_frontier=0, n_gpus=1):
        L = lib()
        o = Options()
        L.rmc_options_default(ctypes.byref(o))
        # the path bytes stay referenced by the Options object for the call
        if checkpoint_dir is not None:
            o._ckpt = str(checkpoint_dir).encode()
            o.checkpoint_dir = o._ckpt
            o.checkpoint_minutes = float(checkpoint_minutes)
        if recover_dir is not None:
            o._recover = str(recover_dir).encode()
            o.recover_dir = o._recover
        o.deadlock_check = 1 if deadlock else 0
        o.hash_slots, o.msg_cap_K, o.frontier_cap = hash_slots, msg_cap_K, frontier_cap
        o.chunk_parents, o.verbose, o.max_depth, o.cpu_workers = chunk_parents, int(verbose), max_depth, workers
        o.grow_on_overflow = int(grow_on_overflow)
        o.time_limit = float(time_limit)
        o.fp_bits = int(fp_bits)
        o.host_frontier = int(host_frontier)
        o.n_gpus = int(n_gpus)
        return o

    def _result(self, rc, r):
        L = lib()
        if rc != 0:
            raise RaftmcError(L.rmc_last_error().decode())
        levels = (ctypes.c_uint64 * 2048)()
        nl = L.rmc_levels(self._h, levels, 1024)
        out = dict(generated=r.generated, distinct=r.distinct, depth=r.depth,
                   left=r.left_on_queue, status=STATUS.get(r.status, str(r.status)),
                   violated=r.violated.decode(), message=r.message.decode(),
                   seconds=r.seconds, expand_ms=r.expand_ms, mark_ms=r.mark_ms,
                   materialize_ms=r.materialize_ms, expand_launches=r.expand_launches,
                   state_bytes=r.state_bytes, hash_capacity=r.hash_capacity, max_msgs=r.max_msgs,
                   device_bytes=r.device_bytes,
                   hidden_var_collisions=r.hidden_var_collisions,
                   levels=[[levels[2 * k], levels[2 * k + 1]] for k in range(min(nl, 1024))])
        self._last = r
        if r.status in (1, 2):
            out["trace"] = self.trace()
        return out

    def set_next(self, disjuncts):
        """Next as operator names of the spec family's definitions, in order
        (rmc_model_set_next: the TLA+ front end's lowering of such a Next)."""
        if lib().rmc_model_set_next(self._h, ",".join(disjuncts).encode()) != 0:
            raise RaftmcError(lib().rmc_last_error().decode())

    def set_guard(self, action, params, expr):
        """Replace the guard of one of Next's simple actions (Restart,
        RequestVote, Timeout, BecomeLeader, ClientRequest) by TLA+ expression
        text over the state, the cfg's constants and the action's parameters
        (rmc_model_set_guard: the front end's compiled guard, rmc_guard.cpp);
        e.g. set_guard("RequestVote", "i", "electionCtr <= MaxElections")."""
        if isinstance(params, (list, tuple)):
            params = ", ".join(params)
        if lib().rmc_model_set_guard(self._h, action.encode(), params.encode(), expr.encode()) != 0:
            raise RaftmcError(lib().rmc_last_error().decode())

    def define_action(self, name, form, params, body):
        """Define an action by its TLA+ text for set_next to use by name
        (rmc_model_define_action: compiled whole, guard and effect,
        rmc_guard.cpp compile_effect).  form: "i", "iv" or "ij" (the binding
        \\E i \\in Server / i \\in Server, v \\in Value / i, j \\in Server), or "m": a
        message handler, body of \\E m \\in DOMAIN messages (compile_handler)."""
        f = {"i": 0, "iv": 1, "ij": 2, "m": 3}[form] if isinstance(form, str) else int(form)
        if isinstance(params, (list, tuple)):
            params = ", ".join(params)
        if lib().rmc_model_define_action(self._h, name.encode(), f, params.encode(), body.encode()) != 0:
            raise RaftmcError(lib().rmc_last_error().decode())

    def next(self):
        """The model's Next, as the library's operator names in order."""
        buf = ctypes.create_string_buffer(4096)
        lib().rmc_model_next(self._h, buf, len(buf))
        return buf.value.decode().split(",")

    def check(self, **kw):
        """Run the model check; returns a dict of TLC's results.  n_gpus=N > 1 runs
        the fingerprint-sharded search over GPUs 0..N-1 of this process, one host
        thread per GPU (rmc_check_multi over RCCL); more GPUs than visible raise."""
        o, r = self._options(**kw), Result()
        return self._result(lib().rmc_check(self._h, ctypes.byref(o), ctypes.byref(r)), r)

    def check_cpu(self, workers=0, **kw):
        """The CPU engine (TLC -workers N on host threads; same results as check)."""
        o, r = self._options(workers=workers, **kw), Result()
        return self._result(lib().rmc_check_cpu(self._h, ctypes.byref(o), ctypes.byref(r)), r)

    def check_logical(self, shards, **kw):
        """The fingerprint-sharded protocol with `shards` logical shards on this GPU."""
        o, r = self._options(**kw), Result()
        return self._result(lib().rmc_check_logical(self._h, ctypes.byref(o), int(shards), ctypes.byref(r)), r)

    def check_multi(self, devices, transport=XPORT_P2P, **kw):
        """The in-process multi-GPU check with shard r on devices[r] (rmc_check_multi).
        transport XPORT_P2P (peer copies; a device may repeat, e.g. [0, 0]) or
        XPORT_RCCL (distinct devices)."""
        o, r = self._options(**kw), Result()
        devs = (ctypes.c_int * len(devices))(*[int(d) for d in devices])
        rc = lib().rmc_check_multi(self._h, ctypes.byref(o), devs, len(devices), int(transport), ctypes.byref(r))
        return self._result(rc, r)

    def phases(self):
        """Where the last single-GPU check's wall time went, in seconds
        (rmc_check_phases): hip_init, model_upload, buffers, launch_enqueue,
        table_growth, buffer_growth, widening, host_frontier, kernels, total."""
        import json
        buf = ctypes.create_string_buffer(4096)
        if lib().rmc_check_phases(self._h, buf, len(buf)) < 0:
            raise RaftmcError("no check")
        return json.loads(buf.value.decode())

    def selftest_hf_stats(self):
        """TEST HOOK: the last check's host-frontier buffer regrowths while its
        copy streams ran: (pack buffers, output windows)."""
        buf = (ctypes.c_uint64 * 2)()
        lib().rmc_selftest_hf_stats(self._h, buf)
        return int(buf[0]), int(buf[1])

    def check_sharded(self, rank, world, device, unique_id, **kw):
        """One shard of a multi-GPU check (one process per GPU, RCCL).  unique_id =
        comm_unique_id() from rank 0, shared with every rank out of band."""
        o, r = self._options(**kw), Result()
        rc = lib().rmc_check_sharded(self._h, ctypes.byref(o), int(rank), int(world), int(device),
                                     bytes(unique_id), ctypes.byref(r))
        return self._result(rc, r)

    def check_sharded_shm(self, rank, world, device, shm_name, **kw):
        """One shard of a multi-process check with shared memory as the transport
        (several processes may share one GPU; see rmc_check_sharded_shm)."""
        o, r = self._options(**kw), Result()
        rc = lib().rmc_check_sharded_shm(self._h, ctypes.byref(o), int(rank), int(world), int(device),
                                         shm_name.encode(), ctypes.byref(r))
        return self._result(rc, r)

    def simulate(self, walkers=1 << 16, depth=100, seed=0, behaviors=None, seconds=0.0, **kw):
        """TLC -simulate on the GPU.  Returns generated (states), behaviors,
        depth (longest behaviour), status and, on a violation, the trace."""
        o, r = self._options(**kw), Result()
        rc = lib().rmc_simulate(self._h, ctypes.byref(o), int(walkers), int(depth), int(seed) & (2**64 - 1),
                                int(behaviors if behaviors else walkers), float(seconds), ctypes.byref(r))
        out = self._result(rc, r)
        out["behaviors"] = out.pop("distinct")
        out.pop("levels", None)
        return out

    def trace(self):
        L = lib()
        n = L.rmc_trace_len(self._h)
        buf = ctypes.create_string_buffer(1 << 20)
        tr = []
        for k in range(max(n, 0)):
            L.rmc_trace_action(self._h, k, buf, len(buf))
            act = buf.value.decode()
            L.rmc_trace_state(self._h, k, buf, len(buf))
            tr.append((act, buf.value.decode()))
        return tr

    def trace_module(self, name):
        """TLC -dumpTrace tla: (module text, cfg text) replaying the error trace with the spec's Next."""
        L = lib()
        n = L.rmc_trace_module(self._h, name.encode(), None, 0, None, 0)
        if n < 0:
            raise RaftmcError("no trace to dump")
        tla = ctypes.create_string_buffer(n + 1)
        cfg = ctypes.create_string_buffer(1 << 16)
        L.rmc_trace_module(self._h, name.encode(), tla, len(tla), cfg, len(cfg))
        return tla.value.decode(), cfg.value.decode()

    def trace_json(self):
        """TLC -dumpTrace json: the error trace as a dict."""
        import json
        L = lib()
        n = L.rmc_trace_json(self._h, None, 0)
        if n < 0:
            raise RaftmcError("no trace to dump")
        buf = ctypes.create_string_buffer(n + 1)
        L.rmc_trace_json(self._h, buf, len(buf))
        return json.loads(buf.value.decode())

    def selftest_random_trace(self, seed, steps):
        """TEST HOOK: a seeded host random walk replayed into the model's trace (not a product path)."""
        n = lib().rmc_selftest_random_trace(self._h, seed, steps)
        if n < 0:
            raise RaftmcError(lib().rmc_last_error().decode())
        return n

    def report(self):
        L = lib()
        buf = ctypes.create_string_buffer(1 << 22)
        L.rmc_format_report(self._h, ctypes.byref(self._last), buf, len(buf))
        return buf.value.decode()

    def selftest_profile_expand(self, level, **kw):
        """TEST HOOK (RMC_DIAG builds): k_expand phase times on `level`'s first chunk:
        [(diag, ms)], diag 4 staging .. 1 no insert, 0 the real launch."""
        o = self._options(**kw)
        buf = (ctypes.c_double * 64)()
        n = lib().rmc_selftest_profile_expand(self._h, ctypes.byref(o), int(level), buf, 64)
        if n < 0:
            raise RaftmcError(lib().rmc_last_error().decode())
        return [(int(buf[2 * k]), buf[2 * k + 1]) for k in range(n)]

    def selftest_widenings(self):
        """TEST HOOK: the last check's row widenings, [(depth, first parent of the
        redone chunk within its level, message slots after), ...]."""
        buf = (ctypes.c_uint64 * 3072)()
        n = lib().rmc_selftest_widenings(self._h, buf, 3072)
        return [tuple(buf[3 * k:3 * k + 3]) for k in range(min(n, 1024))]

    def selftest_set_hint_kmax(self, k):
        """TEST HOOK: pretend the last check saw at most k messages per state, so the
        next check packs rows to k slots (an overflow must take the re-run path)."""
        lib().rmc_selftest_set_hint_kmax(self._h, int(k))

    def selftest_host_bfs(self, kmax=0, max_distinct=0):
        """TEST HOOK: sequential host BFS over the same lowered actions (not a product path)."""
        L = lib()
        out3 = (ctypes.c_uint64 * 3)()
        levels = (ctypes.c_uint64 * 4096)()
        rc = L.rmc_selftest_host_bfs(self._h, kmax, max_distinct, out3, levels, 2048)
        if rc == -1:
            raise RaftmcError(L.rmc_last_error().decode())
        res = dict(generated=out3[0], distinct=out3[1], depth=out3[2], rc=rc)
        if rc > 0:
            res["levels"] = [[levels[2 * k], levels[2 * k + 1]] for k in range(min(rc, 2048))]
        return res


def release_device_memory():
    """Free the device buffers librmc caches per GPU between checks."""
    lib().rmc_release_device_memory()


def check(tla_path, cfg_path=None, **kw):
    """TLC-equivalent run: check(M.tla, M.cfg) -> dict (generated, distinct, depth, ...)."""
    return Model(tla_path, cfg_path).check(**kw)


def comm_unique_id():
    """128-byte RCCL communicator id (call on rank 0, broadcast to every rank)."""
    buf = ctypes.create_string_buffer(128)
    if lib().rmc_comm_unique_id(buf) != 0:
        raise RaftmcError(lib().rmc_last_error().decode())
    return buf.raw


def check_text(module, cfg_text, **kw):
    return Model(module=module, cfg_text=cfg_text).check(**kw)


def tla_hashes(text):
    """The TLA+ front end's closure hash of every definition of a module text
    (rmc_tla_hashes): {name: hash}, plus "#module" and "#vars"."""
    buf = ctypes.create_string_buffer(1 << 20)
    n = lib().rmc_tla_hashes(text.encode(), buf, len(buf))
    if n < 0:
        raise RaftmcError(buf.value.decode())
    out = {}
    for line in buf.value.decode().splitlines():
        if line.startswith("#unparsed"):
            out.setdefault("#unparsed", []).append(line.split()[1])
        elif line.startswith("#"):
            k, v = line.split(None, 1)
            out[k] = v
        else:
            k, v = line.split()
            out[k] = v
    return out


def abi_layout():
    """librmc's own sizeof/offsetof of rmc_options and rmc_result (rmc_abi_layout)."""
    buf = (ctypes.c_uint64 * 64)()
    n = lib().rmc_abi_layout(buf, 64)
    return [buf[k] for k in range(n)]


def encode_msg(spec, **f):
    """TEST HOOK: the packed word for a message record + codec self-consistency flag."""
    names = ["type", "term", "src", "dst", "lli", "llt", "granted", "pli", "plt", "nent", "eterm",
             "evalue", "commit", "success", "midx", "lci", "lct", "count", "lcenil"]
    arr = (ctypes.c_int * 19)(*[int(f.get(n, 0)) for n in names])
    out = ctypes.c_uint32()
    ok = lib().rmc_selftest_encode_msg(spec, arr, ctypes.byref(out))
    return out.value, ok == 0


def encode_kmsg(**f):
    """TEST HOOK: the packed word of a KRaft record (rmc_spec.h kr_encode) + codec self-consistency flag."""
    names = ["cls", "dst", "src", "epoch", "err", "leader", "granted", "f1", "f2", "cepoch", "cfo", "clfe",
             "elen", "eepoch", "evalue", "hwm", "divend", "divepoch", "count"]
    defaults = dict(err=1, leader=-1)
    arr = (ctypes.c_int * 19)(*[int(f.get(n, defaults.get(n, 0))) for n in names])
    out = ctypes.c_uint32()
    ok = lib().rmc_selftest_encode_kmsg(arr, ctypes.byref(out))
    return out.value, ok == 0
