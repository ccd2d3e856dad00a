// Host-only sanitizer harness for the native runtime (csrc/runtime/rccl_comm.cpp), SURVEY §5.2.
//
// rccl_comm.cpp is compiled for the host with -fsanitize=thread (or address,undefined) and linked against
// the fakes below instead of libamdhip64 / librccl, so its threads (owning thread issuing collectives,
// RCCL watchdog polling events / aborting) run on a CPU with no GPU and the sanitizer sees every access.
//
//   * events: complete on record unless g_hang is set (then they never complete -> the watchdog times out);
//   * communicators: a collective on an aborted / destroyed communicator is a use-after-abort and fails
//     the run; ncclCommAbort while a collective is being enqueued on it is a violation of the issue lock;
//   * scenarios: (1) timeout + abort racing a hot issue loop and a second thread re-arming the timeout and
//     polling the error, (2) the bucket reducer through prepare / mark_ready / finalize for many
//     iterations with graph-replay tracking from another thread, (3) destroy with pending events.
// Build + run: tests/test_runtime_sanitize.py (CPU, no GPU marker).
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <mutex>
#include <thread>
#include <vector>

// ---------------------------------------------------------------------------------------------- fakes
namespace {
std::atomic<bool> g_hang{false};
std::atomic<bool> g_stuck{false};  // the next collective's enqueue never returns (scenario "stuck")
std::atomic<int> g_violations{0};

struct FakeEvent {
  std::atomic<bool> done{true};
};
struct FakeComm {
  std::atomic<bool> alive{true};
  std::atomic<int> in_flight{0};
};
// aborted communicators stay allocated until exit, so a late use is reported as a violation
std::mutex g_comms_mu;
std::vector<std::unique_ptr<FakeComm>> g_comms;

void violation(const char* what) {
  fprintf(stderr, "VIOLATION: %s\n", what);
  g_violations.fetch_add(1);
}

int collective(ncclComm_t comm) {
  FakeComm* c = reinterpret_cast<FakeComm*>(comm);
  c->in_flight.fetch_add(1);
  if (!c->alive.load()) violation("collective issued on an aborted/destroyed communicator");
  while (g_stuck.load()) std::this_thread::sleep_for(std::chrono::milliseconds(5));
  std::this_thread::sleep_for(std::chrono::microseconds(50));  // the enqueue takes a while
  if (!c->alive.load()) violation("communicator aborted while a collective was being enqueued");
  c->in_flight.fetch_sub(1);
  return 0;
}
}  // namespace

hipError_t hipSetDevice(int) { return hipSuccess; }
hipError_t hipDeviceGetStreamPriorityRange(int* lo, int* hi) {
  *lo = 0;
  *hi = -1;
  return hipSuccess;
}
hipError_t hipStreamCreateWithPriority(hipStream_t* s, unsigned int, int) {
  *s = reinterpret_cast<hipStream_t>(new int(0));
  return hipSuccess;
}
hipError_t hipStreamDestroy(hipStream_t s) {
  delete reinterpret_cast<int*>(s);
  return hipSuccess;
}
hipError_t hipStreamIsCapturing(hipStream_t, hipStreamCaptureStatus* st) {
  *st = hipStreamCaptureStatusNone;
  return hipSuccess;
}
hipError_t hipStreamSynchronize(hipStream_t) { return hipSuccess; }
hipError_t hipStreamWaitEvent(hipStream_t, hipEvent_t, unsigned int) { return hipSuccess; }
hipError_t hipEventCreate(hipEvent_t* e) {
  *e = reinterpret_cast<hipEvent_t>(new FakeEvent());
  return hipSuccess;
}
hipError_t hipEventCreateWithFlags(hipEvent_t* e, unsigned) { return hipEventCreate(e); }
hipError_t hipEventDestroy(hipEvent_t e) {
  delete reinterpret_cast<FakeEvent*>(e);
  return hipSuccess;
}
hipError_t hipEventRecord(hipEvent_t e, hipStream_t) {
  reinterpret_cast<FakeEvent*>(e)->done.store(!g_hang.load());
  return hipSuccess;
}
hipError_t hipEventQuery(hipEvent_t e) {
  return reinterpret_cast<FakeEvent*>(e)->done.load() ? hipSuccess : hipErrorNotReady;
}
hipError_t hipEventSynchronize(hipEvent_t) { return hipSuccess; }
hipError_t hipEventElapsedTime(float* ms, hipEvent_t, hipEvent_t) {
  *ms = 0.f;
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

ncclResult_t ncclGetUniqueId(ncclUniqueId* id) {
  memset(id, 7, sizeof(*id));
  return ncclSuccess;
}
ncclResult_t ncclGetVersion(int* v) {
  *v = 0;
  return ncclSuccess;
}
const char* ncclGetErrorString(ncclResult_t) { return "fake"; }
ncclResult_t ncclCommInitRank(ncclComm_t* c, int, ncclUniqueId, int) {
  std::lock_guard<std::mutex> g(g_comms_mu);
  g_comms.emplace_back(new FakeComm());
  *c = reinterpret_cast<ncclComm_t>(g_comms.back().get());
  return ncclSuccess;
}
ncclResult_t ncclCommInitRankConfig(ncclComm_t* c, int n, ncclUniqueId id, int r, ncclConfig_t*) {
  return ncclCommInitRank(c, n, id, r);
}
ncclResult_t ncclCommAbort(ncclComm_t comm) {
  FakeComm* c = reinterpret_cast<FakeComm*>(comm);
  if (c->in_flight.load()) violation("ncclCommAbort while a collective is being enqueued");
  if (!c->alive.exchange(false)) violation("communicator aborted twice");
  return ncclSuccess;  // kept allocated: a later use is reported as a violation, not a crash
}
ncclResult_t ncclCommDestroy(ncclComm_t comm) {
  FakeComm* c = reinterpret_cast<FakeComm*>(comm);
  if (!c->alive.exchange(false)) violation("communicator destroyed after abort");
  return ncclSuccess;
}
ncclResult_t ncclCommGetAsyncError(ncclComm_t, ncclResult_t* e) {
  *e = ncclSuccess;
  return ncclSuccess;
}
ncclResult_t ncclGroupStart() { return ncclSuccess; }
ncclResult_t ncclGroupEnd() { return ncclSuccess; }
ncclResult_t ncclAllReduce(const void*, void*, size_t, ncclDataType_t, ncclRedOp_t, ncclComm_t c, hipStream_t) {
  return (ncclResult_t)collective(c);
}
ncclResult_t ncclBroadcast(const void*, void*, size_t, ncclDataType_t, int, ncclComm_t c, hipStream_t) {
  return (ncclResult_t)collective(c);
}
ncclResult_t ncclReduceScatter(const void*, void*, size_t, ncclDataType_t, ncclRedOp_t, ncclComm_t c,
                               hipStream_t) {
  return (ncclResult_t)collective(c);
}
ncclResult_t ncclAllGather(const void*, void*, size_t, ncclDataType_t, ncclComm_t c, hipStream_t) {
  return (ncclResult_t)collective(c);
}

// ---------------------------------------------------------------------------------------------- runtime API
extern "C" {
void* ddpx_comm_create(const char*, int, int, int, int, double, int*);
int ddpx_comm_destroy(void*, int);
int ddpx_comm_allreduce(void*, const void*, void*, size_t, int, int, hipStream_t);
int ddpx_comm_track(void*, hipStream_t, const char*);
int ddpx_comm_set_timeout(void*, double, int);
int ddpx_comm_error(void*);
void* ddpx_comm_stream(void*);
void* ddpx_reducer_create(void*, int, int);
int ddpx_reducer_set_bucket(void*, int, void*, size_t, int, int, int);
int ddpx_reducer_prepare(void*);
int ddpx_reducer_mark_ready(void*, int, int, hipStream_t);
int ddpx_reducer_finalize(void*, hipStream_t);
int ddpx_reducer_destroy(void*);
}

static int fail(const char* what) {
  fprintf(stderr, "FAIL: %s\n", what);
  return 1;
}

// (1) the watchdog times out a hung collective and aborts the communicator while the owner keeps issuing
static int scenario_timeout_abort() {
  setenv("DDPX_COMM_TIMEOUT_ACTION", "abort", 1);
  char uid[128] = {0};
  int err = 0;
  void* c = ddpx_comm_create(uid, 2, 0, 0, 1, 0.2, &err);
  if (!c) return fail("create");
  g_hang.store(true);
  std::atomic<bool> done{false};
  std::thread poker([&] {  // a second host thread re-arms the timeout and polls, as a monitor would
    while (!done.load()) {
      ddpx_comm_set_timeout(c, 0.2, 1);
      (void)ddpx_comm_error(c);
      std::this_thread::sleep_for(std::chrono::milliseconds(1));
    }
  });
  std::vector<float> buf(16);
  int rc = 0;
  const auto t_end = std::chrono::steady_clock::now() + std::chrono::seconds(5);
  while (std::chrono::steady_clock::now() < t_end) {
    rc = ddpx_comm_allreduce(c, buf.data(), buf.data(), buf.size(), (int)ncclFloat32, (int)ncclSum, nullptr);
    if (rc) break;
  }
  done.store(true);
  poker.join();
  g_hang.store(false);
  const int e = ddpx_comm_error(c);
  ddpx_comm_destroy(c, 0);
  if (rc != 3) return fail("collectives kept succeeding after the timeout");
  if (e != 2) return fail("error code is not 'timed out'");
  return 0;
}

// (2) reducer iterations + graph-replay tracking from another thread, watchdog polling throughout
static int scenario_reducer() {
  setenv("DDPX_COMM_TIMEOUT_ACTION", "raise", 1);
  char uid[128] = {0};
  int err = 0;
  void* c = ddpx_comm_create(uid, 2, 1, 0, 1, 5.0, &err);
  if (!c) return fail("create");
  void* r = ddpx_reducer_create(c, 4, (int)ncclAvg);
  std::vector<float> grads(4 * 64);
  for (int i = 0; i < 4; ++i)
    if (ddpx_reducer_set_bucket(r, i, grads.data() + 64 * i, 64, (int)ncclFloat32, 2, i & 1)) return fail("bucket");
  std::atomic<bool> done{false};
  hipStream_t side = nullptr;
  hipStreamCreateWithPriority(&side, 0, 0);
  std::thread replays([&] {
    while (!done.load()) {
      ddpx_comm_track(c, side, "graph replay");
      std::this_thread::sleep_for(std::chrono::microseconds(200));
    }
  });
  for (int it = 0; it < 200; ++it) {
    ddpx_reducer_prepare(r);
    for (int i = 3; i >= 0; --i) {
      if (ddpx_reducer_mark_ready(r, i, 1, nullptr) != 0) return fail("bucket launched early");
      if (ddpx_reducer_mark_ready(r, i, 1, nullptr) != 1) return fail("bucket not launched");
    }
    if (ddpx_reducer_finalize(r, nullptr) != 0) return fail("finalize forced buckets");
  }
  done.store(true);
  replays.join();
  const int e = ddpx_comm_error(c);
  ddpx_reducer_destroy(r);
  hipStreamDestroy(side);
  ddpx_comm_destroy(c, 0);
  return e ? fail("spurious watchdog error") : 0;
}

// (3) destroy while collectives are pending (events never complete), no timeout
static int scenario_destroy_pending() {
  setenv("DDPX_COMM_TIMEOUT_ACTION", "raise", 1);
  char uid[128] = {0};
  int err = 0;
  void* c = ddpx_comm_create(uid, 2, 0, 0, 0, 100.0, &err);
  if (!c) return fail("create");
  g_hang.store(true);
  std::vector<float> buf(8);
  for (int i = 0; i < 50; ++i)
    if (ddpx_comm_allreduce(c, buf.data(), buf.data(), 8, (int)ncclFloat32, (int)ncclSum, nullptr))
      return fail("allreduce");
  g_hang.store(false);
  return ddpx_comm_destroy(c, 1) ? fail("destroy") : 0;
}

// (4) "stuck": the owning thread blocks inside an RCCL enqueue (issue_mu held) while an earlier collective
// times out under the abort action.  The watchdog cannot abort underneath the call: it must set error 4 and
// end the process with exit code 3 (checked by the caller: tests/test_runtime_sanitize.py).
static int scenario_stuck() {
  setenv("DDPX_COMM_TIMEOUT_ACTION", "abort", 1);
  char uid[128] = {0};
  int err = 0;
  void* c = ddpx_comm_create(uid, 2, 0, 0, 1, 0.2, &err);
  if (!c) return fail("create");
  std::vector<float> buf(16);
  g_hang.store(true);  // this collective's completion event never fires -> timeout after 0.2 s
  if (ddpx_comm_allreduce(c, buf.data(), buf.data(), buf.size(), (int)ncclFloat32, (int)ncclSum, nullptr))
    return fail("first allreduce");
  g_stuck.store(true);
  std::thread monitor([&] {  // another thread sees the escalation code before the process ends
    for (;;) {
      if (ddpx_comm_error(c) == 4) {
        printf("rt_sanitize: stuck escalation observed\n");
        fflush(stdout);
        return;
      }
      std::this_thread::sleep_for(std::chrono::milliseconds(1));
    }
  });
  monitor.detach();
  (void)ddpx_comm_allreduce(c, buf.data(), buf.data(), buf.size(), (int)ncclFloat32, (int)ncclSum, nullptr);
  return fail("the stuck enqueue returned");  // unreachable: the watchdog ends the process first
}

int main(int argc, char** argv) {
  if (argc > 1 && !strcmp(argv[1], "stuck")) return scenario_stuck();
  int rc = scenario_timeout_abort();
  rc |= scenario_reducer();
  rc |= scenario_destroy_pending();
  if (g_violations.load()) rc |= fail("fake RCCL saw protocol violations");
  g_comms.clear();
  printf(rc ? "rt_sanitize: FAILED\n" : "rt_sanitize: OK\n");
  return rc;
}
