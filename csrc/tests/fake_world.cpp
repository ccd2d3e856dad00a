// Multi-rank, data-moving fakes of HIP streams/events and RCCL for the native runtime
// (csrc/runtime/rccl_comm.cpp), so its world-size > 1 code — the C++ bucket reducer's all-reduce,
// ZeRO-1 reduce-scatter into `ptr + rank*shard`, the in-place all-gather from `gptr + rank*shard`,
// the event ordering between the compute stream and the communicator stream — runs on a CPU with N
// ranks as threads of one process and real host buffers.
//
// Built with rccl_comm.cpp into a host shared library by tests/test_fake_world.py (g++, no GPU), which
// drives the real Reducer through ctypes with the exact bucket layouts ddpx.parallel.ddp builds for the
// toy MLP, at N = 2 / 4 / 8, and compares every rank's buffers with a numpy reduction.
//
//   * streams: one worker thread per stream executing its queue in FIFO order (a kernel launch is a
//     queued host function; fake_launch_copy sleeps first, so a missing stream dependency reads stale
//     bytes and the comparison fails);
//   * events: record = a queued marker; hipStreamWaitEvent queues a wait for the generation recorded
//     at call time (HIP semantics: a later re-record does not move an earlier wait);
//   * RCCL: communicators of one unique id form a world; collectives match by per-communicator issue
//     order (NCCL's rule).  The op runs on the issuing stream: every rank's worker posts its buffers,
//     the last to arrive computes the result once (sum in fp64 for fp32/fp64/bf16 inputs, rank order),
//     everybody copies its part out, and the slot is freed when the last rank leaves.  A mismatch in
//     kind / count / dtype / op / root between ranks, or a rank that never arrives within the timeout,
//     is a recorded violation (never a hang).
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <functional>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

namespace {

using Clock = std::chrono::steady_clock;

std::atomic<int> g_violations{0};
std::mutex g_viol_mu;
std::string g_last_violation;
std::atomic<int> g_timeout_ms{30000};
std::atomic<long long> g_collectives{0};
const Clock::time_point g_t0 = Clock::now();
const bool g_trace = [] {
  const char* e = getenv("FAKE_WORLD_TRACE");
  return e && e[0] == '1';
}();
double now_ms() { return std::chrono::duration<double, std::milli>(Clock::now() - g_t0).count(); }

void violation(const std::string& what) {
  std::lock_guard<std::mutex> g(g_viol_mu);
  fprintf(stderr, "FAKE-WORLD VIOLATION: %s\n", what.c_str());
  g_last_violation = what;
  g_violations.fetch_add(1);
}

// ------------------------------------------------------------------------------------------ streams
struct FakeStream {
  std::mutex mu;
  std::condition_variable cv;
  std::deque<std::function<void()>> q;
  long long submitted = 0, completed = 0;
  bool stop = false;
  std::thread worker;

  FakeStream() {
    worker = std::thread([this] {
      for (;;) {
        std::function<void()> fn;
        {
          std::unique_lock<std::mutex> l(mu);
          cv.wait(l, [this] { return stop || !q.empty(); });
          if (q.empty()) return;  // stop requested and drained
          fn = std::move(q.front());
          q.pop_front();
        }
        fn();
        {
          std::lock_guard<std::mutex> l(mu);
          ++completed;
        }
        cv.notify_all();
      }
    });
  }
  ~FakeStream() {
    {
      std::lock_guard<std::mutex> l(mu);
      stop = true;
    }
    cv.notify_all();
    worker.join();
  }
  void enqueue(std::function<void()> fn) {
    {
      std::lock_guard<std::mutex> l(mu);
      q.push_back(std::move(fn));
      ++submitted;
    }
    cv.notify_all();
  }
  void sync() {
    std::unique_lock<std::mutex> l(mu);
    const long long target = submitted;
    cv.wait(l, [&] { return completed >= target; });
  }
};

FakeStream* S(hipStream_t s);

struct FakeEvent {
  std::mutex mu;
  std::condition_variable cv;
  long long recorded = 0;   // generation of the latest record
  long long completed = 0;  // generation the stream has reached
  Clock::time_point t{};
};

using EventRef = std::shared_ptr<FakeEvent>;
EventRef& R(hipEvent_t e) { return *reinterpret_cast<EventRef*>(e); }
FakeEvent* E(hipEvent_t e) { return R(e).get(); }

// the legacy null stream: one per host thread (each rank of a test is one thread)
FakeStream* S(hipStream_t s) {
  if (s) return reinterpret_cast<FakeStream*>(s);
  thread_local std::unique_ptr<FakeStream> def(new FakeStream());
  return def.get();
}

// ------------------------------------------------------------------------------------------- worlds
enum Kind { K_ALLREDUCE = 1, K_BROADCAST, K_REDUCE_SCATTER, K_ALLGATHER };

struct Desc {
  int kind = 0;
  const void* send = nullptr;
  void* recv = nullptr;
  size_t count = 0;  // all-reduce/broadcast: elements; reduce-scatter: recvcount; all-gather: sendcount
  int dtype = 0, op = 0, root = 0;
};

struct Slot {
  std::vector<Desc> d;
  // each rank's send bytes, copied when ITS stream reached the op (uninitialised allocation: the copy must
  // start reading at once, not after zero-filling a multi-MB vector)
  std::vector<std::unique_ptr<unsigned char[]>> in;
  std::vector<bool> posted;
  int arrived = 0, left = 0;
  bool ready = false, failed = false;
  std::vector<unsigned char> result;  // full result buffer (bytes)
};

struct World {
  int n = 0;
  std::mutex mu;
  std::condition_variable cv;
  std::map<long long, Slot> slots;
  int joined = 0;
};

std::mutex g_worlds_mu;
std::map<std::string, std::shared_ptr<World>> g_worlds;
std::atomic<unsigned long long> g_uid_counter{1};

struct FakeComm {
  std::shared_ptr<World> w;
  int rank = 0;
  std::atomic<long long> seq{0};
  std::atomic<bool> alive{true};
};

size_t dsize(int dt) {
  switch (dt) {
    case ncclInt8: case ncclUint8: return 1;
    case ncclFloat16: case ncclBfloat16: return 2;
    case ncclInt32: case ncclUint32: case ncclFloat32: return 4;
    case ncclInt64: case ncclUint64: case ncclFloat64: return 8;
    default: return 0;
  }
}

double load_elem(const void* p, size_t i, int dt) {
  switch (dt) {
    case ncclFloat32: return static_cast<const float*>(p)[i];
    case ncclFloat64: return static_cast<const double*>(p)[i];
    case ncclInt32: return static_cast<const int*>(p)[i];
    case ncclInt64: return (double)static_cast<const long long*>(p)[i];
    case ncclUint8: return static_cast<const unsigned char*>(p)[i];
    case ncclBfloat16: {
      unsigned u = ((unsigned)static_cast<const unsigned short*>(p)[i]) << 16;
      float f;
      memcpy(&f, &u, 4);
      return f;
    }
    default: return 0.0;
  }
}

void store_elem(void* p, size_t i, int dt, double v) {
  switch (dt) {
    case ncclFloat32: static_cast<float*>(p)[i] = (float)v; break;
    case ncclFloat64: static_cast<double*>(p)[i] = v; break;
    case ncclInt32: static_cast<int*>(p)[i] = (int)v; break;
    case ncclInt64: static_cast<long long*>(p)[i] = (long long)v; break;
    case ncclUint8: static_cast<unsigned char*>(p)[i] = (unsigned char)v; break;
    case ncclBfloat16: {  // round to nearest even (inputs of the tests are finite)
      float f = (float)v;
      unsigned u;
      memcpy(&u, &f, 4);
      u = (u + 0x7fffu + ((u >> 16) & 1u)) >> 16;
      static_cast<unsigned short*>(p)[i] = (unsigned short)u;
      break;
    }
    default: break;
  }
}

bool same_shape(const Desc& a, const Desc& b) {
  return a.kind == b.kind && a.count == b.count && a.dtype == b.dtype && a.op == b.op && a.root == b.root;
}

// Compute the whole result once (called by the last rank to arrive, under the world lock).
void compute(Slot& s, int n) {
  const Desc& d0 = s.d[0];
  const size_t es = dsize(d0.dtype);
  if ((d0.kind == K_ALLREDUCE || d0.kind == K_REDUCE_SCATTER) && d0.dtype == ncclFloat32 &&
      (d0.op == ncclSum || d0.op == ncclAvg)) {
    // fast path (the gradient buckets): fp64 accumulation in rank order, one rounding to fp32
    const size_t total = d0.kind == K_ALLREDUCE ? d0.count : d0.count * (size_t)n;
    s.result.resize(total * es);
    std::vector<double> acc(total, 0.0);
    for (int r = 0; r < n; ++r) {
      const float* x = static_cast<const float*>(s.d[r].send);
      for (size_t i = 0; i < total; ++i) acc[i] += x[i];
    }
    float* out = reinterpret_cast<float*>(s.result.data());
    const double inv = d0.op == ncclAvg ? 1.0 / n : 1.0;
    for (size_t i = 0; i < total; ++i) out[i] = (float)(acc[i] * inv);
  } else if (d0.kind == K_ALLREDUCE || d0.kind == K_REDUCE_SCATTER) {
    const size_t total = d0.kind == K_ALLREDUCE ? d0.count : d0.count * (size_t)n;
    s.result.resize(total * es);
    for (size_t i = 0; i < total; ++i) {
      double acc = 0.0;
      bool first = true;
      for (int r = 0; r < n; ++r) {
        const double v = load_elem(s.d[r].send, i, d0.dtype);
        if (first) { acc = v; first = false; continue; }
        switch (d0.op) {
          case ncclSum: case ncclAvg: acc += v; break;
          case ncclProd: acc *= v; break;
          case ncclMax: acc = v > acc ? v : acc; break;
          case ncclMin: acc = v < acc ? v : acc; break;
          default: break;
        }
      }
      if (d0.op == ncclAvg) acc /= (double)n;
      store_elem(s.result.data(), i, d0.dtype, acc);
    }
  } else if (d0.kind == K_BROADCAST) {
    s.result.resize(d0.count * es);
    memcpy(s.result.data(), s.d[d0.root].send, d0.count * es);
  } else {  // all-gather
    s.result.resize(d0.count * (size_t)n * es);
    for (int r = 0; r < n; ++r) memcpy(s.result.data() + (size_t)r * d0.count * es, s.d[r].send, d0.count * es);
  }
}

void run_collective(FakeComm* c, long long seq, Desc d) {
  World& w = *c->w;
  const int n = w.n, rank = c->rank;
  std::unique_lock<std::mutex> l(w.mu);
  Slot& s = w.slots[seq];
  if (s.d.empty()) {
    s.d.resize(n);
    s.in.resize(n);
    s.posted.assign(n, false);
  }
  {
    // the collective reads this rank's input NOW (its stream has reached it); later writes by other
    // streams of this rank must not leak in — that is exactly a missing stream dependency
    const size_t es = dsize(d.dtype);
    const size_t nb = (d.kind == K_ALLREDUCE || d.kind == K_BROADCAST) ? d.count * es
                      : d.kind == K_REDUCE_SCATTER ? d.count * (size_t)n * es : d.count * es;
    if (d.kind != K_BROADCAST || rank == d.root) {
      s.in[rank].reset(new unsigned char[nb]);
      memcpy(s.in[rank].get(), d.send, nb);
    }
    d.send = s.in[rank].get();
    if (g_trace && d.dtype == ncclFloat32 && nb >= 4)
      fprintf(stderr, "[%9.3f ms] collective #%lld rank %d arrived, first input %g\n", now_ms(), seq, rank,
              (double)static_cast<const float*>(d.send)[0]);
  }
  s.d[rank] = d;
  s.posted[rank] = true;
  if (++s.arrived == n) {
    for (int r = 1; r < n; ++r)
      if (!same_shape(s.d[0], s.d[r])) {
        char buf[256];
        snprintf(buf, sizeof(buf), "collective #%lld differs between rank 0 (kind %d count %zu dtype %d op %d) and "
                 "rank %d (kind %d count %zu dtype %d op %d)", seq, s.d[0].kind, s.d[0].count, s.d[0].dtype,
                 s.d[0].op, r, s.d[r].kind, s.d[r].count, s.d[r].dtype, s.d[r].op);
        violation(buf);
        s.failed = true;
      }
    if (g_trace) fprintf(stderr, "[%9.3f ms] collective #%lld kind %d count %zu: all %d ranks posted\n", now_ms(), seq,
                         d.kind, d.count, n);
    if (!s.failed) compute(s, n);
    if (g_trace) fprintf(stderr, "[%9.3f ms] collective #%lld computed\n", now_ms(), seq);
    s.ready = true;
    g_collectives.fetch_add(1);
    w.cv.notify_all();
  } else {
    const auto deadline = Clock::now() + std::chrono::milliseconds(g_timeout_ms.load());
    if (!w.cv.wait_until(l, deadline, [&] { return s.ready; })) {
      std::string missing;
      for (int r = 0; r < n; ++r)
        if (!s.posted[r]) missing += " " + std::to_string(r);
      violation("collective #" + std::to_string(seq) + " (rank " + std::to_string(rank) +
                ") timed out waiting for ranks" + missing);
      s.failed = true;
      s.ready = true;
      w.cv.notify_all();
    }
  }
  if (!s.failed) {
    const size_t es = dsize(d.dtype);
    if (d.kind == K_REDUCE_SCATTER) {
      memcpy(d.recv, s.result.data() + (size_t)rank * d.count * es, d.count * es);
    } else {
      memcpy(d.recv, s.result.data(), s.result.size());
    }
  }
  if (++s.left == n) w.slots.erase(seq);
}

ncclResult_t enqueue(ncclComm_t comm, hipStream_t stream, Desc d) {
  FakeComm* c = reinterpret_cast<FakeComm*>(comm);
  if (!c || !c->alive.load()) {
    violation("collective on a destroyed/aborted communicator");
    return ncclInvalidUsage;
  }
  if (dsize(d.dtype) == 0) return ncclInvalidArgument;
  const long long seq = c->seq.fetch_add(1);
  S(stream)->enqueue([c, seq, d] { run_collective(c, seq, d); });
  return ncclSuccess;
}

}  // namespace

// ---------------------------------------------------------------------------------------------- HIP
hipError_t hipSetDevice(int) { return hipSuccess; }
hipError_t hipDeviceGetStreamPriorityRange(int* lo, int* hi) {
  *lo = 0;
  *hi = -1;
  return hipSuccess;
}
hipError_t hipStreamCreateWithPriority(hipStream_t* s, unsigned int, int) {
  *s = reinterpret_cast<hipStream_t>(new FakeStream());
  return hipSuccess;
}
hipError_t hipStreamDestroy(hipStream_t s) {
  delete reinterpret_cast<FakeStream*>(s);
  return hipSuccess;
}
hipError_t hipStreamIsCapturing(hipStream_t, hipStreamCaptureStatus* st) {
  *st = hipStreamCaptureStatusNone;
  return hipSuccess;
}
hipError_t hipStreamSynchronize(hipStream_t s) {
  S(s)->sync();
  return hipSuccess;
}
hipError_t hipEventCreate(hipEvent_t* e) {
  *e = reinterpret_cast<hipEvent_t>(new EventRef(std::make_shared<FakeEvent>()));
  return hipSuccess;
}
hipError_t hipEventCreateWithFlags(hipEvent_t* e, unsigned) { return hipEventCreate(e); }
hipError_t hipEventDestroy(hipEvent_t e) {
  delete reinterpret_cast<EventRef*>(e);  // markers still queued hold their own reference
  return hipSuccess;
}
hipError_t hipEventRecord(hipEvent_t e, hipStream_t s) {
  EventRef ev = R(e);
  long long gen;
  {
    std::lock_guard<std::mutex> l(ev->mu);
    gen = ++ev->recorded;
  }
  S(s)->enqueue([ev, gen] {
    {
      std::lock_guard<std::mutex> l(ev->mu);
      if (gen > ev->completed) ev->completed = gen;
      ev->t = Clock::now();
    }
    ev->cv.notify_all();
  });
  return hipSuccess;
}
hipError_t hipStreamWaitEvent(hipStream_t s, hipEvent_t e, unsigned int) {
  EventRef ev = R(e);
  long long gen;
  {
    std::lock_guard<std::mutex> l(ev->mu);
    gen = ev->recorded;
  }
  if (gen == 0) return hipSuccess;  // never recorded: no dependency
  S(s)->enqueue([ev, gen] {
    std::unique_lock<std::mutex> l(ev->mu);
    const auto deadline = Clock::now() + std::chrono::milliseconds(g_timeout_ms.load());
    if (!ev->cv.wait_until(l, deadline, [&] { return ev->completed >= gen; }))
      violation("hipStreamWaitEvent: event never completed (stream dependency deadlock)");
  });
  return hipSuccess;
}
hipError_t hipEventQuery(hipEvent_t e) {
  FakeEvent* ev = E(e);
  std::lock_guard<std::mutex> l(ev->mu);
  return ev->completed >= ev->recorded ? hipSuccess : hipErrorNotReady;
}
hipError_t hipEventSynchronize(hipEvent_t e) {
  FakeEvent* ev = E(e);
  std::unique_lock<std::mutex> l(ev->mu);
  ev->cv.wait(l, [&] { return ev->completed >= ev->recorded; });
  return hipSuccess;
}
hipError_t hipEventElapsedTime(float* ms, hipEvent_t a, hipEvent_t b) {
  Clock::time_point ta, tb;
  {
    std::lock_guard<std::mutex> l(E(a)->mu);
    ta = E(a)->t;
  }
  {
    std::lock_guard<std::mutex> l(E(b)->mu);
    tb = E(b)->t;
  }
  *ms = std::chrono::duration<float, std::milli>(tb - ta).count();
  return hipSuccess;
}
hipError_t hipHostMalloc(void** p, size_t n, unsigned int) {
  *p = calloc(1, n);
  return hipSuccess;
}
hipError_t hipHostFree(void* p) {
  free(p);
  return hipSuccess;
}
hipError_t hipHostGetDevicePointer(void** d, void* h, unsigned int) {
  *d = h;
  return hipSuccess;
}

// --------------------------------------------------------------------------------------------- RCCL
ncclResult_t ncclGetUniqueId(ncclUniqueId* id) {
  memset(id, 0, sizeof(*id));
  const unsigned long long k = g_uid_counter.fetch_add(1);
  memcpy(id->internal, &k, sizeof(k));
  return ncclSuccess;
}
ncclResult_t ncclGetVersion(int* v) {
  *v = 0;
  return ncclSuccess;
}
const char* ncclGetErrorString(ncclResult_t) { return "fake"; }
ncclResult_t ncclCommInitRank(ncclComm_t* comm, int nranks, ncclUniqueId id, int rank) {
  std::shared_ptr<World> w;
  {
    std::lock_guard<std::mutex> g(g_worlds_mu);
    const std::string key(id.internal, sizeof(id.internal));
    auto& slot = g_worlds[key];
    if (!slot) {
      slot = std::make_shared<World>();
      slot->n = nranks;
    }
    w = slot;
  }
  if (w->n != nranks || rank < 0 || rank >= nranks) {
    violation("ncclCommInitRank: inconsistent world size / rank");
    return ncclInvalidArgument;
  }
  FakeComm* c = new FakeComm();
  c->w = w;
  c->rank = rank;
  {
    std::lock_guard<std::mutex> g(w->mu);
    ++w->joined;
  }
  *comm = reinterpret_cast<ncclComm_t>(c);
  return ncclSuccess;
}

// channel bounds are a performance setting: the fake world checks them and otherwise ignores them
ncclResult_t ncclCommInitRankConfig(ncclComm_t* comm, int nranks, ncclUniqueId id, int rank, ncclConfig_t* config) {
  if (config && config->minCTAs > 0 && config->maxCTAs > 0 && config->minCTAs > config->maxCTAs) {
    violation("ncclCommInitRankConfig: minCTAs > maxCTAs");
    return ncclInvalidArgument;
  }
  return ncclCommInitRank(comm, nranks, id, rank);
}
static ncclResult_t release_comm(ncclComm_t comm, const char* what) {
  FakeComm* c = reinterpret_cast<FakeComm*>(comm);
  if (!c->alive.exchange(false)) {
    violation(std::string(what) + " of a communicator already destroyed");
    return ncclInvalidUsage;
  }
  // the communicator object stays allocated: queued collectives may still reference it
  return ncclSuccess;
}
ncclResult_t ncclCommAbort(ncclComm_t comm) { return release_comm(comm, "ncclCommAbort"); }
ncclResult_t ncclCommDestroy(ncclComm_t comm) { return release_comm(comm, "ncclCommDestroy"); }
ncclResult_t ncclCommGetAsyncError(ncclComm_t, ncclResult_t* e) {
  *e = ncclSuccess;
  return ncclSuccess;
}
ncclResult_t ncclGroupStart() { return ncclSuccess; }
ncclResult_t ncclGroupEnd() { return ncclSuccess; }
ncclResult_t ncclAllReduce(const void* s, void* r, size_t n, ncclDataType_t dt, ncclRedOp_t op, ncclComm_t c,
                           hipStream_t st) {
  Desc d;
  d.kind = K_ALLREDUCE;
  d.send = s;
  d.recv = r;
  d.count = n;
  d.dtype = (int)dt;
  d.op = (int)op;
  return enqueue(c, st, d);
}
ncclResult_t ncclBroadcast(const void* s, void* r, size_t n, ncclDataType_t dt, int root, ncclComm_t c,
                           hipStream_t st) {
  Desc d;
  d.kind = K_BROADCAST;
  d.send = s;
  d.recv = r;
  d.count = n;
  d.dtype = (int)dt;
  d.root = root;
  return enqueue(c, st, d);
}
ncclResult_t ncclReduceScatter(const void* s, void* r, size_t n, ncclDataType_t dt, ncclRedOp_t op, ncclComm_t c,
                               hipStream_t st) {
  Desc d;
  d.kind = K_REDUCE_SCATTER;
  d.send = s;
  d.recv = r;
  d.count = n;
  d.dtype = (int)dt;
  d.op = (int)op;
  return enqueue(c, st, d);
}
ncclResult_t ncclAllGather(const void* s, void* r, size_t n, ncclDataType_t dt, ncclComm_t c, hipStream_t st) {
  Desc d;
  d.kind = K_ALLGATHER;
  d.send = s;
  d.recv = r;
  d.count = n;
  d.dtype = (int)dt;
  return enqueue(c, st, d);
}

// ------------------------------------------------------------------------------------- test controls
#define FAKE_API extern "C" __attribute__((visibility("default")))

FAKE_API void* fake_stream_create() { return new FakeStream(); }
FAKE_API void fake_stream_destroy(void* s) { delete static_cast<FakeStream*>(s); }
FAKE_API void fake_stream_sync(void* s) { S(static_cast<hipStream_t>(s))->sync(); }

// A "kernel" on stream s: after delay_us, copy nbytes src -> dst (the test's gradient producer).
FAKE_API void fake_launch_copy(void* s, void* dst, const void* src, size_t nbytes, int delay_us) {
  S(static_cast<hipStream_t>(s))->enqueue([=] {
    if (delay_us > 0) std::this_thread::sleep_for(std::chrono::microseconds(delay_us));
    memcpy(dst, src, nbytes);
    if (g_trace) fprintf(stderr, "[%9.3f ms] copy of %zu bytes landed\n", now_ms(), nbytes);
  });
}

// A "kernel" on stream s: dst[i] (dst_dtype) = src[i] (src_dtype) for i < count — the shard update of a
// sharded optimizer, writing the parameter copy the all-gather then distributes (fp32 -> bf16 shadow).
FAKE_API void fake_launch_convert(void* s, void* dst, int dst_dtype, const void* src, int src_dtype, size_t count,
                                  int delay_us) {
  S(static_cast<hipStream_t>(s))->enqueue([=] {
    if (delay_us > 0) std::this_thread::sleep_for(std::chrono::microseconds(delay_us));
    for (size_t i = 0; i < count; ++i) store_elem(dst, i, dst_dtype, load_elem(src, i, src_dtype));
  });
}

FAKE_API int fake_violations() { return g_violations.load(); }
FAKE_API void fake_reset_violations() { g_violations.store(0); }
FAKE_API long long fake_collectives() { return g_collectives.load(); }
FAKE_API void fake_set_timeout_ms(int ms) { g_timeout_ms.store(ms); }
FAKE_API int fake_last_violation(char* out, int n) {
  std::lock_guard<std::mutex> g(g_viol_mu);
  snprintf(out, (size_t)n, "%s", g_last_violation.c_str());
  return (int)g_last_violation.size();
}
