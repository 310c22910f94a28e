// Why torch's process-group watchdog aborted during a torch-collective capture:
// does hipEventQuery fail on an event recorded OUTSIDE any capture, on a stream that later
// joins a capture?  Mimics ProcessGroupNCCL: an eager work's end event E on the process
// group's internal stream S; the watchdog thread polls E; the main thread then captures a
// collective, which forks S into the capture (S waits on the capturing stream C, runs, and C
// waits on S).  Each query is made from a second thread (as the watchdog's) and from the
// capturing thread.
//   hipcc --offload-arch=gfx950 -O2 -o /tmp/evq tools/micro/event_query_capture.hip && /tmp/evq
#include <hip/hip_runtime.h>

#include <cstdio>
#include <thread>

__global__ void k_bump(float* x) { x[threadIdx.x] += 1.0f; }

#define CK(x)                                                                      \
  do {                                                                             \
    hipError_t e_ = (x);                                                           \
    if (e_ != hipSuccess) {                                                        \
      std::printf("%s:%d %s -> %s\n", __FILE__, __LINE__, #x, hipGetErrorName(e_)); \
      return 1;                                                                    \
    }                                                                              \
  } while (0)

static const char* query_other_thread(hipEvent_t e) {
  hipError_t r = hipSuccess;
  std::thread t([&] { r = hipEventQuery(e); });
  t.join();
  return hipGetErrorName(r);
}

int main() {
  float* d = nullptr;
  CK(hipMalloc(&d, 256 * sizeof(float)));
  hipStream_t S, C;
  CK(hipStreamCreateWithFlags(&S, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&C, hipStreamNonBlocking));
  hipEvent_t E, F, G, E2;
  CK(hipEventCreateWithFlags(&E, hipEventDisableTiming));
  CK(hipEventCreateWithFlags(&F, hipEventDisableTiming));
  CK(hipEventCreateWithFlags(&G, hipEventDisableTiming));
  CK(hipEventCreateWithFlags(&E2, hipEventDisableTiming));

  k_bump<<<1, 64, 0, S>>>(d);            // the eager collective on S
  CK(hipEventRecord(E, S));              // its end event (the watchdog's)
  CK(hipDeviceSynchronize());
  std::printf("1 eager, complete:                  other thread %s, this thread %s\n",
              query_other_thread(E), hipGetErrorName(hipEventQuery(E)));

  CK(hipStreamBeginCapture(C, hipStreamCaptureModeThreadLocal));
  k_bump<<<1, 64, 0, C>>>(d);
  std::printf("2 capture on C, S not in it:        other thread %s, this thread %s\n",
              query_other_thread(E), hipGetErrorName(hipEventQuery(E)));
  CK(hipEventRecord(F, C));              // S forks from the capture (torch: ncclStream waits
  CK(hipStreamWaitEvent(S, F, 0));       // on the current stream)
  k_bump<<<1, 64, 0, S>>>(d);            // the captured collective on S
  std::printf("3 S joined the capture (E from before): other thread %s, this thread %s\n",
              query_other_thread(E), hipGetErrorName(hipEventQuery(E)));
  CK(hipEventRecord(E2, S));             // the captured work's own end event
  std::printf("4 event recorded inside the capture: other thread %s, this thread %s\n",
              query_other_thread(E2), hipGetErrorName(hipEventQuery(E2)));
  CK(hipEventRecord(G, S));
  CK(hipStreamWaitEvent(C, G, 0));       // joined back
  hipGraph_t g;
  CK(hipStreamEndCapture(C, &g));
  std::printf("5 capture ended (E from before):    other thread %s, this thread %s\n",
              query_other_thread(E), hipGetErrorName(hipEventQuery(E)));
  hipGraphExec_t ge;
  CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
  CK(hipGraphLaunch(ge, C));
  CK(hipStreamSynchronize(C));
  float h[64];
  CK(hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost));
  std::printf("replayed: x[0] = %.0f (eager 1 + replay 2 = 3)\n", h[0]);
  CK(hipGraphExecDestroy(ge));
  CK(hipGraphDestroy(g));
  return 0;
}
