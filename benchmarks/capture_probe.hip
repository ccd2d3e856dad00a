// Stream-capture semantics probe (ROCm 7 / MI355X): what a capture that fails (invalidated, unjoined, or
// left open) does to the streams involved, and which calls from which thread invalidate a thread-local
// capture.  Every case runs on fresh streams.  Backs profiles/r5_capture/NOTES.md.
//   hipcc --offload-arch=gfx950 -O2 -std=c++17 benchmarks/capture_probe.hip -o capture_probe -lpthread
#include <hip/hip_runtime.h>

#include <cstdio>
#include <functional>
#include <thread>

__global__ void touch(float* p) { p[threadIdx.x] += 1.f; }

static const char* st_name(hipStreamCaptureStatus s) {
  switch (s) {
    case hipStreamCaptureStatusNone: return "none";
    case hipStreamCaptureStatusActive: return "active";
    case hipStreamCaptureStatusInvalidated: return "invalidated";
    default: return "?";
  }
}

static hipStreamCaptureStatus status(const char* tag, hipStream_t s) {
  hipStreamCaptureStatus st = hipStreamCaptureStatusNone;
  hipError_t e = hipStreamGetCaptureInfo(s, &st, nullptr);
  printf("    %-46s err=%-26s status=%s\n", tag, hipGetErrorName(e), st_name(st));
  return st;
}

static void rc(const char* tag, hipError_t e) { printf("    %-46s -> %s\n", tag, hipGetErrorName(e)); }

static float* d = nullptr;
static float h[64];

static hipStream_t mk() {
  hipStream_t s;
  (void)hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
  return s;
}

// capture on a fresh stream, run `during` while capturing, end, report
static void case_(const char* name, const std::function<void(hipStream_t)>& during) {
  printf("[%s]\n", name);
  hipStream_t a = mk();
  rc("begin(thread_local)", hipStreamBeginCapture(a, hipStreamCaptureModeThreadLocal));
  touch<<<1, 64, 0, a>>>(d);
  during(a);
  hipGraph_t g = nullptr;
  rc("end", hipStreamEndCapture(a, &g));
  if (g) (void)hipGraphDestroy(g);
  status("a after end", a);
  (void)hipGetLastError();
}

int main() {
  (void)hipMalloc(&d, 256);
  hipEvent_t done_ev;
  (void)hipEventCreateWithFlags(&done_ev, hipEventDisableTiming);
  hipStream_t x = mk();
  (void)hipEventRecord(done_ev, x);
  (void)hipStreamSynchronize(x);

  // --- which calls invalidate a thread-local capture
  case_("baseline: nothing else", [](hipStream_t) {});
  case_("other thread: hipEventQuery(completed event)", [&](hipStream_t) {
    std::thread t([&] { rc("eventQuery (other thread)", hipEventQuery(done_ev)); });
    t.join();
  });
  case_("other thread: memcpyWithStream(null)", [&](hipStream_t) {
    std::thread t([&] { rc("memcpyWithStream null (other)", hipMemcpyWithStream(d, h, 256, hipMemcpyHostToDevice, nullptr)); });
    t.join();
  });
  case_("other thread: hipStreamSynchronize(other stream)", [&](hipStream_t) {
    hipStream_t y = mk();
    std::thread t([&] { rc("streamSync y (other)", hipStreamSynchronize(y)); });
    t.join();
  });
  case_("other thread: hipMalloc", [&](hipStream_t) {
    std::thread t([&] {
      float* p = nullptr;
      rc("hipMalloc (other)", hipMalloc(&p, 4096));
    });
    t.join();
  });
  case_("same thread: hipEventQuery(completed event)", [&](hipStream_t) { rc("eventQuery", hipEventQuery(done_ev)); });
  case_("same thread: hipStreamQuery(other stream)", [&](hipStream_t) { rc("streamQuery x", hipStreamQuery(x)); });
  case_("same thread: memcpyWithStream(other stream)", [&](hipStream_t) {
    hipStream_t y = mk();
    rc("memcpyWithStream y", hipMemcpyWithStream(d, h, 256, hipMemcpyHostToDevice, y));
  });
  case_("same thread: hipMalloc", [&](hipStream_t) {
    float* p = nullptr;
    rc("hipMalloc", hipMalloc(&p, 4096));
  });
  case_("same thread: hipEventDestroy(unrelated)", [&](hipStream_t) {
    hipEvent_t e;
    (void)hipEventCreateWithFlags(&e, hipEventDisableTiming);
    rc("eventDestroy", hipEventDestroy(e));
  });
  case_("same thread: waitEvent(event recorded outside the capture)", [&](hipStream_t a) {
    rc("waitEvent(external)", hipStreamWaitEvent(a, done_ev, 0));
  });

  // --- what an invalidated capture leaves behind, and whether the stream is usable again
  printf("[after an invalidated capture]\n");
  {
    hipStream_t a = mk(), y = mk();
    (void)hipStreamBeginCapture(a, hipStreamCaptureModeThreadLocal);
    touch<<<1, 64, 0, a>>>(d);
    (void)hipMemcpyWithStream(d, h, 256, hipMemcpyHostToDevice, y);  // invalidates (same thread)
    hipGraph_t g = nullptr;
    rc("end", hipStreamEndCapture(a, &g));
    status("a after end", a);
    touch<<<1, 64, 0, a>>>(d);
    rc("launch on a (getLastError)", hipGetLastError());
    rc("memcpyWithStream a", hipMemcpyWithStream(d, h, 256, hipMemcpyHostToDevice, a));
    rc("streamSynchronize a", hipStreamSynchronize(a));
    status("a now", a);
    rc("begin again on a", hipStreamBeginCapture(a, hipStreamCaptureModeThreadLocal));
    touch<<<1, 64, 0, a>>>(d);
    g = nullptr;
    rc("end again", hipStreamEndCapture(a, &g));
    if (g) (void)hipGraphDestroy(g);
    status("a after a clean capture", a);
    (void)hipGetLastError();
  }

  // --- unjoined side stream: can the capture be repaired by joining and ending again?
  printf("[unjoined side stream, then repair]\n");
  {
    hipStream_t a = mk(), b = mk();
    hipEvent_t fork, join;
    (void)hipEventCreateWithFlags(&fork, hipEventDisableTiming);
    (void)hipEventCreateWithFlags(&join, hipEventDisableTiming);
    (void)hipStreamBeginCapture(a, hipStreamCaptureModeThreadLocal);
    touch<<<1, 64, 0, a>>>(d);
    (void)hipEventRecord(fork, a);
    (void)hipStreamWaitEvent(b, fork, 0);
    touch<<<1, 64, 0, b>>>(d);
    unsigned long long ida = 0, idb = 0;
    hipStreamCaptureStatus s;
    (void)hipStreamGetCaptureInfo(a, &s, &ida);
    (void)hipStreamGetCaptureInfo(b, &s, &idb);
    printf("    capture ids a=%llu b=%llu\n", ida, idb);
    hipGraph_t g = nullptr;
    rc("end (unjoined)", hipStreamEndCapture(a, &g));
    printf("    graph=%p\n", (void*)g);
    status("a", a);
    status("b", b);
    rc("record join on b", hipEventRecord(join, b));
    rc("a waits join", hipStreamWaitEvent(a, join, 0));
    hipGraph_t g2 = nullptr;
    rc("end again", hipStreamEndCapture(a, &g2));
    printf("    graph=%p\n", (void*)g2);
    if (g2) (void)hipGraphDestroy(g2);
    status("a after repair", a);
    status("b after repair", b);
    rc("memcpyWithStream b", hipMemcpyWithStream(d, h, 256, hipMemcpyHostToDevice, b));
    rc("memcpyWithStream a", hipMemcpyWithStream(d, h, 256, hipMemcpyHostToDevice, a));
    (void)hipGetLastError();
  }

  // --- capture never ended, other streams / threads
  printf("[capture left open]\n");
  {
    hipStream_t a = mk(), y = mk();
    (void)hipStreamBeginCapture(a, hipStreamCaptureModeThreadLocal);
    touch<<<1, 64, 0, a>>>(d);
    status("null stream (main)", nullptr);
    rc("memcpyWithStream null (main)", hipMemcpyWithStream(d, h, 256, hipMemcpyHostToDevice, nullptr));
    status("a", a);
    hipGraph_t g = nullptr;
    rc("end", hipStreamEndCapture(a, &g));
    if (g) (void)hipGraphDestroy(g);
    status("a after end", a);
    (void)y;
  }
  rc("deviceSynchronize", hipDeviceSynchronize());
  printf("done\n");
  return 0;
}
