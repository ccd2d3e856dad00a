// ddpx — native RCCL communicator + gradient-bucket reducer for MI355X.
//
// Replaces, natively, what the reference gets implicitly from PyTorch:
//   * c10d ProcessGroupNCCL  (/root/reference/multigpu.py:32):
//     a communicator per process group, collectives on a dedicated
//     high-priority HIP stream ordered with events, async-error polling and a
//     timeout watchdog that aborts the communicator.
//   * the DDP Reducer        (/root/reference/multigpu.py:89):
//     per-bucket ready counters; the moment a bucket's last gradient is
//     produced, an event on the compute stream gates an all-reduce on the
//     comm stream, so the collective overlaps the rest of backward.
//   * _broadcast_coalesced   (SURVEY §2.2 N4): broadcasts of persistent flat
//     buffers (no per-step flatten).
// On ROCm the RCCL library is the one torch already loaded (same soname), so
// there is one RCCL instance per process.  The unique id travels through the
// c10d TCPStore (Python side).
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <mutex>
#include <thread>
#include <vector>

#define DDPX_API extern "C" __attribute__((visibility("default")))

namespace {

using Clock = std::chrono::steady_clock;

struct Pending {
  hipEvent_t ev;
  Clock::time_point t0;
  char what[64];  // copied: callers (ctypes) pass temporaries
};

// What the watchdog does when a tracked operation exceeds the timeout or RCCL reports an asynchronous
// error (DDPX_COMM_TIMEOUT_ACTION; ProcessGroupNCCL's TORCH_NCCL_ASYNC_ERROR_HANDLING analogue):
//   raise  - set the error flag only; the owning thread's next comm.check() / collective call fails
//   abort  - also ncclCommAbort (serialised against collective issue, see Comm::issue_mu)
//   exit   - raise, then terminate the process with exit code 3 after a grace period
//            (DDPX_COMM_EXIT_GRACE_S, default 10 s) unless the owning thread exited first (default)
// Escalation under raise / abort: an abort that cannot take issue_mu within ~2 s (the owning thread is stuck
// INSIDE an RCCL call, e.g. an enqueue blocked behind a dead peer) cannot free the communicator safely, and
// that thread will never return to observe a raised error either; the error state becomes 4 ("stuck in
// RCCL", readable by any other thread through ddpx_comm_error) and the process ends with exit code 3, as
// the exit action would (csrc/tests/rt_sanitize.cpp scenario "stuck").
enum TimeoutAction : int { ACT_RAISE = 0, ACT_ABORT = 1, ACT_EXIT = 2 };

struct Comm {
  // The RCCL handle is written only under issue_mu (creation, abort, destroy).  Every collective
  // issue holds issue_mu for the duration of the enqueue and checks `aborted` first, so an abort can
  // never free the communicator underneath an ncclAllReduce call on the owning thread.
  ncclComm_t nccl = nullptr;
  std::mutex issue_mu;
  std::atomic<bool> aborted{false};
  int rank = 0, nranks = 1, device = 0;
  hipStream_t stream = nullptr;  // dedicated comm stream (high priority)
  int priority = 0;
  std::vector<hipStream_t> retired;  // streams a failed HIP-graph capture left unusable (ddpx_comm_renew_stream)
  // watchdog
  std::mutex mu;  // guards pending / free_events
  std::deque<Pending> pending;
  std::vector<hipEvent_t> free_events;
  std::thread watchdog;
  std::atomic<bool> stop{false};
  std::atomic<int> error{0};  // 0 ok, 1 async nccl error, 2 timeout, 3 aborted, 4 abort escalated (stuck in RCCL)
  // set by the owning thread (ddpx_comm_set_timeout), read by the watchdog: atomics (a host ThreadSanitizer
  // run of csrc/tests/rt_sanitize.cpp flagged the plain fields as a data race)
  std::atomic<double> timeout_s{0.0};
  std::atomic<bool> track{false};
  std::atomic<int> action{ACT_EXIT};
  double exit_grace_s = 10.0;
  std::atomic<long long> tracked{0};  // operations / graph replays registered with the watchdog
};

int check(ncclResult_t r) { return r == ncclSuccess ? 0 : 1000 + (int)r; }

// Abort the communicator from the watchdog thread.  Waits (bounded) for an in-flight issue call to
// return.  If the owning thread is still inside an RCCL call after the bound (e.g. a connection handshake
// with a dead peer), aborting under it would free the communicator that call is using, so the watchdog
// escalates to the exit action instead: the process ends with exit code 3 (what ACT_EXIT does for any
// timeout).  The handle is never touched without the lock: issuers test `aborted` under issue_mu.
void abort_comm(Comm* c) {
  bool locked = false;
  for (int i = 0; i < 200 && !locked; ++i) {  // ~2 s
    locked = c->issue_mu.try_lock();
    if (!locked) std::this_thread::sleep_for(std::chrono::milliseconds(10));
  }
  if (!locked) {
    c->error.store(4);
    fprintf(stderr, "[ddpx rank %d] abort: a collective call is stuck inside RCCL; terminating (exit code 3)\n",
            c->rank);
    fflush(stderr);
    std::this_thread::sleep_for(std::chrono::milliseconds(200));  // other threads' monitors can read code 4
    std::_Exit(3);
  }
  if (!c->aborted.exchange(true) && c->nccl) ncclCommAbort(c->nccl);
  c->issue_mu.unlock();
}

void on_failure(Comm* c, int code, const char* what) {
  c->error.store(code);
  if (c->action == ACT_ABORT) {
    abort_comm(c);
  } else if (c->action == ACT_EXIT) {
    fprintf(stderr, "[ddpx rank %d] %s: process exits in %.1fs unless it terminates first\n", c->rank, what,
            c->exit_grace_s);
    fflush(stderr);
    const auto t_end = Clock::now() + std::chrono::duration<double>(c->exit_grace_s);
    while (!c->stop.load() && Clock::now() < t_end) std::this_thread::sleep_for(std::chrono::milliseconds(20));
    if (!c->stop.load()) {
      fprintf(stderr, "[ddpx rank %d] %s: terminating (exit code 3)\n", c->rank, what);
      fflush(stderr);
      std::_Exit(3);
    }
  }
}

void watchdog_loop(Comm* c) {
  while (!c->stop.load()) {
    std::this_thread::sleep_for(std::chrono::milliseconds(50));
    if (c->error.load() || c->aborted.load()) continue;
    ncclResult_t ae = ncclSuccess;
    // ncclCommGetAsyncError is documented as callable concurrently with operations on the comm;
    // the handle is stable until abort/destroy, which only this thread (abort) or the owner after
    // joining this thread (destroy) perform.
    if (c->nccl && ncclCommGetAsyncError(c->nccl, &ae) == ncclSuccess && ae != ncclSuccess &&
        ae != ncclInProgress) {
      fprintf(stderr, "[ddpx rank %d] RCCL async error %d (%s)\n", c->rank, (int)ae, ncclGetErrorString(ae));
      fflush(stderr);
      on_failure(c, 1, "RCCL async error");
      continue;
    }
    char late[64] = {0};
    double late_age = 0.0;
    {
      std::lock_guard<std::mutex> g(c->mu);
      while (!c->pending.empty()) {
        Pending& p = c->pending.front();
        hipError_t q = hipEventQuery(p.ev);
        if (q == hipSuccess) {
          c->free_events.push_back(p.ev);
          c->pending.pop_front();
          continue;
        }
        const double age = std::chrono::duration<double>(Clock::now() - p.t0).count();
        const double to = c->timeout_s.load();
        if (to > 0 && age > to) {
          memcpy(late, p.what, sizeof(late));
          late_age = age;
        }
        break;
      }
    }
    if (late[0]) {
      fprintf(stderr, "[ddpx rank %d] collective '%s' timed out: not complete after %.1fs (timeout %.1fs)\n",
              c->rank, late, late_age, c->timeout_s.load());
      fflush(stderr);
      on_failure(c, 2, "collective timed out");
    }
  }
}

// Register "everything enqueued on s so far" with the watchdog: an event recorded now must complete
// within the timeout.  Collectives issued eagerly are tracked one by one; collectives inside a HIP graph
// are tracked per replay (ddpx_comm_track after hipGraphLaunch), since at capture time nothing runs.
void track_op(Comm* c, hipStream_t s, const char* what) {
  if (!c->track) return;
  hipStreamCaptureStatus st = hipStreamCaptureStatusNone;
  if (hipStreamIsCapturing(s, &st) == hipSuccess && st != hipStreamCaptureStatusNone) return;
  std::lock_guard<std::mutex> g(c->mu);
  hipEvent_t ev;
  if (!c->free_events.empty()) {
    ev = c->free_events.back();
    c->free_events.pop_back();
  } else if (hipEventCreateWithFlags(&ev, hipEventDisableTiming) != hipSuccess) {
    return;
  }
  if (hipEventRecord(ev, s) != hipSuccess) {
    c->free_events.push_back(ev);
    return;
  }
  Pending p{ev, Clock::now(), {0}};
  snprintf(p.what, sizeof(p.what), "%s", what ? what : "?");
  c->pending.push_back(p);
  c->tracked.fetch_add(1);
}

// Issue guard: holds issue_mu while a collective is enqueued; fails if the communicator is gone.
struct IssueGuard {
  Comm* c;
  std::lock_guard<std::mutex> g;
  explicit IssueGuard(Comm* c_) : c(c_), g(c_->issue_mu) {}
  bool ok() const { return c->nccl && !c->aborted.load() && c->error.load() == 0; }
};

// ---------------------------------------------------------------------------
// Reducer: gradient buckets -> all-reduce on the comm stream.
// mode 0: all-reduce the bucket in place (replicated optimizer).
// mode 1: reduce-scatter in place (sharded optimizer, ZeRO-1): rank r receives the reduced
//         shard [r*count/n, (r+1)*count/n) at its own position; after the optimizer updated
//         that shard, gather() all-gathers the bucket's parameter copy in place.
struct Bucket {
  void* ptr = nullptr;
  size_t count = 0;
  int dtype = ncclFloat32;
  int expected = 0;
  int pending = 0;
  int mode = 0;
  bool launched = false;
  hipEvent_t ready = nullptr, done = nullptr;
  void* gptr = nullptr;  // gather target (bf16 shadow or fp32 master slice of the bucket)
  size_t gcount = 0;
  int gdtype = ncclBfloat16;
  bool gathering = false;
  hipEvent_t gready = nullptr, gdone = nullptr;
};

struct Reducer {
  Comm* comm = nullptr;
  std::vector<int> lazy;  // buckets whose collective is not issued yet (lazy_comm)
  int op = ncclAvg;
  std::vector<Bucket> buckets;
  int launched = 0;
  // per-iteration communication timing (timing-enabled events; also valid inside HIP graphs):
  // t_first before the first collective, t_last after the latest one (comm stream), t_bwd on the
  // compute stream when backward ended (finalize) -> comm time and the part not hidden by backward
  hipEvent_t t_first = nullptr, t_last = nullptr, t_bwd = nullptr;
  bool timed = false, bwd_marked = false;
};

}  // namespace

DDPX_API int ddpx_comm_unique_id(char* out, int nbytes) {
  if (nbytes < (int)sizeof(ncclUniqueId)) return -1;
  ncclUniqueId id;
  int e = check(ncclGetUniqueId(&id));
  if (e) return e;
  memcpy(out, &id, sizeof(id));
  return 0;
}

DDPX_API int ddpx_comm_version() {
  int v = 0;
  ncclGetVersion(&v);
  return v;
}

// min_ctas / max_ctas > 0: the communicator's channel (CTA) bounds through ncclCommInitRankConfig
// (ncclConfig_t.minCTAs / maxCTAs, per communicator, unlike the process-wide NCCL_MIN/MAX_NCHANNELS).  On an
// 8 x MI355X node each ring channel drives one xGMI link direction, so a bucket only reaches the 7-link
// aggregate with >= 7 channels; more channels cost CUs taken from the overlapped backward GEMMs
// (benchmarks/rccl_sweep.py measures the trade).
DDPX_API void* ddpx_comm_create2(const char* uid, int nranks, int rank, int device, int high_priority,
                                 double timeout_s, int min_ctas, int max_ctas, int* err) {
  *err = 0;
  hipError_t he = hipSetDevice(device);
  if (he != hipSuccess) {
    *err = (int)he;
    return nullptr;
  }
  Comm* c = new Comm();
  c->rank = rank;
  c->nranks = nranks;
  c->device = device;
  int lo = 0, hi = 0;
  hipDeviceGetStreamPriorityRange(&lo, &hi);
  c->priority = high_priority ? hi : lo;
  he = hipStreamCreateWithPriority(&c->stream, hipStreamNonBlocking, c->priority);
  if (he != hipSuccess) {
    *err = (int)he;
    delete c;
    return nullptr;
  }
  ncclUniqueId id;
  memcpy(&id, uid, sizeof(id));
  int e;
  if (min_ctas > 0 || max_ctas > 0) {
    ncclConfig_t cfg = NCCL_CONFIG_INITIALIZER;
    if (min_ctas > 0) cfg.minCTAs = min_ctas;
    if (max_ctas > 0) cfg.maxCTAs = max_ctas;
    e = check(ncclCommInitRankConfig(&c->nccl, nranks, id, rank, &cfg));
  } else {
    e = check(ncclCommInitRank(&c->nccl, nranks, id, rank));
  }
  if (e) {
    *err = e;
    hipStreamDestroy(c->stream);
    delete c;
    return nullptr;
  }
  c->timeout_s = timeout_s;
  c->track = timeout_s > 0;
  if (const char* a = getenv("DDPX_COMM_TIMEOUT_ACTION")) {
    if (!strcmp(a, "raise")) c->action = ACT_RAISE;
    else if (!strcmp(a, "abort")) c->action = ACT_ABORT;
    else c->action = ACT_EXIT;
  }
  if (const char* g = getenv("DDPX_COMM_EXIT_GRACE_S")) c->exit_grace_s = atof(g);
  c->watchdog = std::thread(watchdog_loop, c);
  return c;
}

DDPX_API void* ddpx_comm_create(const char* uid, int nranks, int rank, int device, int high_priority,
                                double timeout_s, int* err) {
  return ddpx_comm_create2(uid, nranks, rank, device, high_priority, timeout_s, 0, 0, err);
}

// Track a graph replay (or any stream position): call right after hipGraphLaunch on `s`.
DDPX_API int ddpx_comm_track(void* h, hipStream_t s, const char* what) {
  Comm* c = static_cast<Comm*>(h);
  if (c->error.load()) return 3;
  track_op(c, s, what ? what : "graph replay");
  return 0;
}

DDPX_API long long ddpx_comm_tracked(void* h) { return static_cast<Comm*>(h)->tracked.load(); }
DDPX_API int ddpx_comm_set_timeout(void* h, double timeout_s, int action) {
  Comm* c = static_cast<Comm*>(h);
  c->timeout_s = timeout_s;
  c->track = timeout_s > 0;
  if (action >= 0) c->action = action;
  return 0;
}

DDPX_API void* ddpx_comm_stream(void* h) { return static_cast<Comm*>(h)->stream; }

// Replace the comm stream by a fresh one (same priority).  A HIP-graph capture that failed after forking onto
// the comm stream can leave it in the capture status "invalidated" on ROCm 7, and RCCL refuses to enqueue on such
// a stream (profiles/r5_capture/NOTES.md).  RCCL communicators are not bound to a stream, so swapping it is safe
// once the caller synchronised the device; the old stream is kept (never destroyed while it may still be
// referenced by a graph) and released at destroy.
DDPX_API int ddpx_comm_renew_stream(void* h) {
  Comm* c = static_cast<Comm*>(h);
  std::lock_guard<std::mutex> g(c->issue_mu);
  hipStream_t s = nullptr;
  hipError_t he = hipStreamCreateWithPriority(&s, hipStreamNonBlocking, c->priority);
  if (he != hipSuccess) return (int)he;
  c->retired.push_back(c->stream);
  c->stream = s;
  return 0;
}
DDPX_API int ddpx_comm_error(void* h) { return static_cast<Comm*>(h)->error.load(); }

DDPX_API int ddpx_comm_destroy(void* h, int abort) {
  Comm* c = static_cast<Comm*>(h);
  c->stop.store(true);
  if (c->watchdog.joinable()) c->watchdog.join();
  int e = 0;
  {
    // scoped: the guard must release issue_mu before `delete c` destroys it (the host ThreadSanitizer
    // harness csrc/tests/rt_sanitize.cpp caught the unlock-after-free of the unscoped guard)
    std::lock_guard<std::mutex> g(c->issue_mu);
    if (c->nccl && !c->aborted.load()) {
      if (abort || c->error.load()) e = check(ncclCommAbort(c->nccl));
      else {
        hipStreamSynchronize(c->stream);
        e = check(ncclCommDestroy(c->nccl));
      }
    }
    c->nccl = nullptr;
  }
  for (auto& p : c->pending) hipEventDestroy(p.ev);
  for (auto ev : c->free_events) hipEventDestroy(ev);
  hipStreamDestroy(c->stream);
  for (auto s : c->retired) (void)hipStreamDestroy(s);
  delete c;
  return e;
}

static hipStream_t pick_stream(Comm* c, hipStream_t s) { return s ? s : c->stream; }

static size_t dtype_size(int dt) {
  switch (dt) {
    case ncclInt8: case ncclUint8: return 1;
    case ncclFloat16: case ncclBfloat16: return 2;
    case ncclInt32: case ncclUint32: case ncclFloat32: return 4;
    case ncclInt64: case ncclUint64: case ncclFloat64: return 8;
    default: return 0;
  }
}

// World size 1 with send == recv: every collective is the identity.  DDPX_COMM_SKIP_IDENTITY=1 skips
// the launch (bench.py --ddp_single sets it, so that mode times the DDP machinery, not RCCL's one-rank
// copy kernels); by default RCCL still runs, so the ws=1 tests exercise real RCCL calls.
static bool skip_identity(const Comm* c, const void* send, const void* recv) {
  static const bool on = [] {
    const char* e = getenv("DDPX_COMM_SKIP_IDENTITY");
    return e && e[0] == '1';
  }();
  return on && c->nranks == 1 && send == recv;
}

DDPX_API int ddpx_comm_allreduce(void* h, const void* send, void* recv, size_t count, int dtype, int op,
                                 hipStream_t s) {
  Comm* c = static_cast<Comm*>(h);
  IssueGuard ig(c);
  if (!ig.ok()) return 3;
  if (skip_identity(c, send, recv)) return 0;
  s = pick_stream(c, s);
  int e = check(ncclAllReduce(send, recv, count, (ncclDataType_t)dtype, (ncclRedOp_t)op, c->nccl, s));
  track_op(c, s, "all_reduce");
  return e;
}

DDPX_API int ddpx_comm_broadcast(void* h, const void* send, void* recv, size_t count, int dtype, int root,
                                 hipStream_t s) {
  Comm* c = static_cast<Comm*>(h);
  IssueGuard ig(c);
  if (!ig.ok()) return 3;
  if (skip_identity(c, send, recv)) return 0;
  s = pick_stream(c, s);
  int e = check(ncclBroadcast(send, recv, count, (ncclDataType_t)dtype, root, c->nccl, s));
  track_op(c, s, "broadcast");
  return e;
}

DDPX_API int ddpx_comm_reduce_scatter(void* h, const void* send, void* recv, size_t recvcount, int dtype, int op,
                                      hipStream_t s) {
  Comm* c = static_cast<Comm*>(h);
  IssueGuard ig(c);
  if (!ig.ok()) return 3;
  if (skip_identity(c, send, recv)) return 0;
  s = pick_stream(c, s);
  int e = check(ncclReduceScatter(send, recv, recvcount, (ncclDataType_t)dtype, (ncclRedOp_t)op, c->nccl, s));
  track_op(c, s, "reduce_scatter");
  return e;
}

DDPX_API int ddpx_comm_allgather(void* h, const void* send, void* recv, size_t sendcount, int dtype,
                                 hipStream_t s) {
  Comm* c = static_cast<Comm*>(h);
  IssueGuard ig(c);
  if (!ig.ok()) return 3;
  if (skip_identity(c, send, recv)) return 0;
  s = pick_stream(c, s);
  int e = check(ncclAllGather(send, recv, sendcount, (ncclDataType_t)dtype, c->nccl, s));
  track_op(c, s, "all_gather");
  return e;
}

// Grouped collectives of one communicator (RCCL launches them at ncclGroupEnd): both ends run under the
// issue guard, so an abort can never free the communicator while the group is being launched.
DDPX_API int ddpx_comm_group_start(void* h) {
  Comm* c = static_cast<Comm*>(h);
  IssueGuard ig(c);
  if (!ig.ok()) return 3;
  return check(ncclGroupStart());
}
DDPX_API int ddpx_comm_group_end(void* h) {
  Comm* c = static_cast<Comm*>(h);
  IssueGuard ig(c);
  if (!ig.ok()) return 3;
  return check(ncclGroupEnd());
}

// ---------------------------------------------------------------------------
DDPX_API void* ddpx_reducer_create(void* comm, int nbuckets, int op) {
  Reducer* r = new Reducer();
  r->comm = static_cast<Comm*>(comm);
  r->op = op;
  r->buckets.resize(nbuckets);
  hipEventCreate(&r->t_first);
  hipEventCreate(&r->t_last);
  hipEventCreate(&r->t_bwd);
  for (auto& b : r->buckets) {
    hipEventCreateWithFlags(&b.ready, hipEventDisableTiming);
    hipEventCreateWithFlags(&b.done, hipEventDisableTiming);
    hipEventCreateWithFlags(&b.gready, hipEventDisableTiming);
    hipEventCreateWithFlags(&b.gdone, hipEventDisableTiming);
  }
  return r;
}

DDPX_API int ddpx_reducer_set_bucket(void* h, int i, void* ptr, size_t count, int dtype, int expected, int mode) {
  Reducer* r = static_cast<Reducer*>(h);
  if (i < 0 || i >= (int)r->buckets.size()) return -1;
  if (mode != 0 && mode != 1) return -2;
  if (mode == 1 && (count % (size_t)r->comm->nranks) != 0) return -3;  // shards must be equal
  if (dtype_size(dtype) == 0) return -4;
  Bucket& b = r->buckets[i];
  b.ptr = ptr;
  b.count = count;
  b.dtype = dtype;
  b.expected = expected;
  b.pending = expected;
  b.mode = mode;
  b.launched = false;
  return 0;
}

// Parameter copy that gather() all-gathers in place after the owner updated its shard.
DDPX_API int ddpx_reducer_set_gather(void* h, int i, void* ptr, size_t count, int dtype) {
  Reducer* r = static_cast<Reducer*>(h);
  if (i < 0 || i >= (int)r->buckets.size()) return -1;
  if (count % (size_t)r->comm->nranks != 0) return -3;
  if (dtype_size(dtype) == 0) return -4;
  Bucket& b = r->buckets[i];
  b.gptr = ptr;
  b.gcount = count;
  b.gdtype = dtype;
  return 0;
}

DDPX_API int ddpx_reducer_prepare(void* h) {
  Reducer* r = static_cast<Reducer*>(h);
  for (auto& b : r->buckets) {
    b.pending = b.expected;
    b.launched = false;
  }
  r->lazy.clear();
  r->launched = 0;
  return 0;
}

// Lazy issue (DDPX_LAZY_COMM=1): the bucket's ready event is recorded on the compute stream at once,
// but the comm-stream wait + collective are issued at the reducer's next call, i.e. after the caller
// has enqueued its next compute kernel.  Same dependencies and collective order; inside a HIP graph
// capture the next compute node is then created before the collective node.
static bool lazy_comm() {
  static const bool v = [] {
    const char* e = getenv("DDPX_LAZY_COMM");
    return e && e[0] == '1';
  }();
  return v;
}

static int issue_bucket(Reducer* r, Bucket& b);

static int flush_lazy(Reducer* r) {
  for (int i : r->lazy) {
    int e = issue_bucket(r, r->buckets[i]);
    if (e) return e;
  }
  r->lazy.clear();
  return 0;
}

static int launch_bucket(Reducer* r, Bucket& b, hipStream_t compute) {
  hipError_t he = hipEventRecord(b.ready, compute);
  if (he != hipSuccess) return (int)he;
  b.launched = true;
  if (lazy_comm()) {
    r->lazy.push_back((int)(&b - r->buckets.data()));
    return 0;
  }
  return issue_bucket(r, b);
}

static int issue_bucket(Reducer* r, Bucket& b) {
  Comm* c = r->comm;
  hipError_t he = hipStreamWaitEvent(c->stream, b.ready, 0);
  if (he != hipSuccess) return (int)he;
  if (r->launched == 0) hipEventRecord(r->t_first, c->stream);
  int e;
  if (b.mode == 1) {
    size_t shard = b.count / (size_t)c->nranks;
    char* recv = static_cast<char*>(b.ptr) + (size_t)c->rank * shard * dtype_size(b.dtype);
    e = ddpx_comm_reduce_scatter(c, b.ptr, recv, shard, b.dtype, r->op, c->stream);
  } else {
    e = ddpx_comm_allreduce(c, b.ptr, b.ptr, b.count, b.dtype, r->op, c->stream);
  }
  if (e) return e;
  // the timing marker goes BEFORE the completion event the consumers join: recorded after it, it would be a
  // trailing node of the communicator stream that no stream waits for (an unjoined fork inside a captured step)
  hipEventRecord(r->t_last, c->stream);
  he = hipEventRecord(b.done, c->stream);
  if (he != hipSuccess) return (int)he;
  r->timed = true;
  r->launched++;
  return 0;
}

// Mark n gradients of bucket i as produced on `compute`.  Launches the bucket's
// all-reduce when it becomes complete.  Returns 1 if launched, 0 if not yet,
// <0 / >1 error code.
DDPX_API int ddpx_reducer_mark_ready(void* h, int i, int n, hipStream_t compute) {
  Reducer* r = static_cast<Reducer*>(h);
  if (i < 0 || i >= (int)r->buckets.size()) return -1;
  Bucket& b = r->buckets[i];
  if (b.launched) return -2;  // marked twice in one backward
  int e = flush_lazy(r);
  if (e) return e;
  b.pending -= n;
  if (b.pending > 0) return 0;
  if (b.pending < 0) return -3;
  e = launch_bucket(r, b, compute);
  return e ? e : 1;
}

// Make `s` wait for bucket i's all-reduce (e.g. so the optimizer can update
// that bucket's parameters while later buckets are still on the wire).
DDPX_API int ddpx_reducer_wait_bucket(void* h, int i, hipStream_t s) {
  Reducer* r = static_cast<Reducer*>(h);
  Bucket& b = r->buckets[i];
  if (!b.launched) return -1;
  if (int e = flush_lazy(r)) return e;
  if (s == r->comm->stream) return 0;  // already in stream order (and a captured self-wait is invalid)
  return (int)hipStreamWaitEvent(s, b.done, 0);
}

// End of backward: launch stragglers (unused parameters), then join every
// bucket's completion into `compute`.  Returns the number of buckets that had
// to be force-launched.
DDPX_API int ddpx_reducer_finalize(void* h, hipStream_t compute) {
  Reducer* r = static_cast<Reducer*>(h);
  hipEventRecord(r->t_bwd, compute);
  r->bwd_marked = true;
  if (int e = flush_lazy(r)) return -1000 - e;
  int forced = 0;
  for (auto& b : r->buckets) {
    if (!b.launched) {
      int e = launch_bucket(r, b, compute);
      if (e) return -1000 - e;
      forced++;
    }
  }
  if (int e = flush_lazy(r)) return -1000 - e;
  for (auto& b : r->buckets) {
    hipError_t he = hipStreamWaitEvent(compute, b.done, 0);
    if (he != hipSuccess) return -(int)he;
  }
  return forced;
}

// End of backward on `compute` (overlap mode, where finalize does not join): timing marker only.
DDPX_API int ddpx_reducer_mark_backward_end(void* h, hipStream_t compute) {
  Reducer* r = static_cast<Reducer*>(h);
  r->bwd_marked = true;
  hipError_t he = hipEventRecord(r->t_bwd, compute);
  if (int e = flush_lazy(r)) return e;
  return (int)he;
}

// Communication time of the last completed iteration and the part of it after backward ended
// (exposed).  Synchronises on the timing events; call outside the hot loop.
DDPX_API int ddpx_reducer_comm_stats(void* h, float* comm_ms, float* exposed_ms) {
  Reducer* r = static_cast<Reducer*>(h);
  *comm_ms = 0.f;
  *exposed_ms = 0.f;
  if (!r->timed) return 1;
  if (hipEventSynchronize(r->t_last) != hipSuccess) return 2;
  float t = 0.f;
  if (hipEventElapsedTime(&t, r->t_first, r->t_last) == hipSuccess) *comm_ms = t;
  if (r->bwd_marked && hipEventElapsedTime(&t, r->t_bwd, r->t_last) == hipSuccess) *exposed_ms = t > 0.f ? t : 0.f;
  return 0;
}

// Sharded optimizer: after `compute` wrote this rank's shard of bucket i's parameter copy,
// all-gather the copy in place on the comm stream (ordered after the reduce-scatters already
// queued there).  wait_gather() joins it into a stream that is about to read the parameters.
DDPX_API int ddpx_reducer_gather(void* h, int i, hipStream_t compute) {
  Reducer* r = static_cast<Reducer*>(h);
  if (i < 0 || i >= (int)r->buckets.size()) return -1;
  Bucket& b = r->buckets[i];
  if (!b.gptr) return -2;
  if (int e = flush_lazy(r)) return e;
  Comm* c = r->comm;
  hipError_t he;
  if (compute != c->stream) {  // issued from the comm stream itself: stream order suffices
    he = hipEventRecord(b.gready, compute);
    if (he != hipSuccess) return (int)he;
    he = hipStreamWaitEvent(c->stream, b.gready, 0);
    if (he != hipSuccess) return (int)he;
  }
  size_t shard = b.gcount / (size_t)c->nranks;
  const char* send = static_cast<const char*>(b.gptr) + (size_t)c->rank * shard * dtype_size(b.gdtype);
  int e = ddpx_comm_allgather(c, send, b.gptr, shard, b.gdtype, c->stream);
  if (e) return e;
  he = hipEventRecord(b.gdone, c->stream);
  if (he != hipSuccess) return (int)he;
  b.gathering = true;
  return 0;
}

DDPX_API int ddpx_reducer_wait_gather(void* h, int i, hipStream_t s) {
  Reducer* r = static_cast<Reducer*>(h);
  if (i < 0 || i >= (int)r->buckets.size()) return -1;
  Bucket& b = r->buckets[i];
  if (!b.gathering) return 0;
  hipError_t he = s == r->comm->stream ? hipSuccess : hipStreamWaitEvent(s, b.gdone, 0);
  b.gathering = false;
  return (int)he;
}

DDPX_API int ddpx_reducer_destroy(void* h) {
  Reducer* r = static_cast<Reducer*>(h);
  for (auto& b : r->buckets) {
    hipEventDestroy(b.ready);
    hipEventDestroy(b.done);
    hipEventDestroy(b.gready);
    hipEventDestroy(b.gdone);
  }
  hipEventDestroy(r->t_first);
  hipEventDestroy(r->t_last);
  hipEventDestroy(r->t_bwd);
  delete r;
  return 0;
}

// ---------------------------------------------------------------------------
// Host-mapped int32 flag (fault injection / watchdog tests): pinned host memory the device can read
// through PCIe; the host flips it with a plain store.
DDPX_API int ddpx_hostflag_create(void** host, void** dev) {
  int* p = nullptr;
  hipError_t e = hipHostMalloc(reinterpret_cast<void**>(&p), 64, hipHostMallocMapped | hipHostMallocCoherent);
  if (e != hipSuccess) return (int)e;
  *p = 0;
  e = hipHostGetDevicePointer(dev, p, 0);
  if (e != hipSuccess) {
    hipHostFree(p);
    return (int)e;
  }
  *host = p;
  return 0;
}

DDPX_API void ddpx_hostflag_set(void* host, int v) {
  __atomic_store_n(static_cast<int*>(host), v, __ATOMIC_SEQ_CST);
}

DDPX_API int ddpx_hostflag_destroy(void* host) { return (int)hipHostFree(host); }
