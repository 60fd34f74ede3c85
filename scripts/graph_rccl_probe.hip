// Probe: can a step of {kernel, event fork/join, RCCL grouped send/recv to
// self, kernel} be captured into a hipGraph and replayed, and what does each
// form cost on the host?  One process, world 1.  Built as a shared library and
// called from scripts/graph_rccl_probe.py after torch is imported, so that it
// runs on torch's HIP runtime and RCCL, as the engine does in bench.py.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                         \
  do {                                                                                \
    hipError_t e_ = (x);                                                              \
    if (e_ != hipSuccess) {                                                           \
      std::printf("HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); \
      std::fflush(stdout);                                                            \
      std::exit(1);                                                                   \
    }                                                                                 \
  } while (0)
#define NK(x)                                                                          \
  do {                                                                                 \
    ncclResult_t r_ = (x);                                                             \
    if (r_ != ncclSuccess) {                                                           \
      std::printf("RCCL error %s at %s:%d\n", ncclGetErrorString(r_), __FILE__, __LINE__); \
      std::fflush(stdout);                                                             \
      std::exit(1);                                                                    \
    }                                                                                  \
  } while (0)

__global__ void fill(int* p, int n, int v) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) p[i] = v + i;
}
__global__ void check(const int* p, int n, int v, int* bad) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n && p[i] != v + i) atomicAdd(bad, 1);
}

static double now_us() {
  return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

// mode: capture mode (0 global, 1 thread-local, 2 relaxed); n: int32 per
// send; pairs: send/recv pairs per group (the engine's step has 2)
extern "C" int probe(int mode, int n, int pairs) {
  CK(hipSetDevice(0));
  ncclUniqueId id;
  NK(ncclGetUniqueId(&id));
  ncclComm_t comm;
  NK(ncclCommInitRank(&comm, 1, id, 0));
  hipStream_t st, cs;
  CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&cs, hipStreamNonBlocking));
  hipEvent_t e0, e1;
  CK(hipEventCreateWithFlags(&e0, hipEventDisableTiming));
  CK(hipEventCreateWithFlags(&e1, hipEventDisableTiming));
  int *sbuf, *rbuf, *bad;
  CK(hipMalloc(&sbuf, n * sizeof(int)));
  CK(hipMalloc(&rbuf, n * sizeof(int)));
  CK(hipMalloc(&bad, sizeof(int)));
  CK(hipMemset(bad, 0, sizeof(int)));
  auto step = [&](int v) {
    fill<<<(n + 255) / 256, 256, 0, st>>>(sbuf, n, v);
    CK(hipEventRecord(e0, st));
    CK(hipStreamWaitEvent(cs, e0, 0));
    NK(ncclGroupStart());
    for (int p = 0; p < pairs; ++p) {
      NK(ncclSend(sbuf, n, ncclInt32, 0, comm, cs));
      NK(ncclRecv(rbuf, n, ncclInt32, 0, comm, cs));
    }
    NK(ncclGroupEnd());
    CK(hipEventRecord(e1, cs));
    CK(hipStreamWaitEvent(st, e1, 0));
    check<<<(n + 255) / 256, 256, 0, st>>>(rbuf, n, v, bad);
  };
  // eager
  for (int i = 0; i < 20; ++i) step(7);
  CK(hipStreamSynchronize(st));
  double t = now_us();
  for (int i = 0; i < 200; ++i) step(7);
  const double eager = (now_us() - t) / 200;
  CK(hipStreamSynchronize(st));
  std::printf("n %d pairs %d eager: host %.1f us/step\n", n, pairs, eager);
  std::fflush(stdout);
  // captured
  const hipStreamCaptureMode cm = mode == 0 ? hipStreamCaptureModeGlobal
                                  : mode == 1 ? hipStreamCaptureModeThreadLocal
                                              : hipStreamCaptureModeRelaxed;
  CK(hipStreamBeginCapture(st, cm));
  step(11);
  hipGraph_t g;
  CK(hipStreamEndCapture(st, &g));
  std::printf("captured (mode %d)\n", mode);
  std::fflush(stdout);
  hipGraphExec_t ex;
  CK(hipGraphInstantiate(&ex, g, nullptr, nullptr, 0));
  std::printf("instantiated\n");
  std::fflush(stdout);
  for (int i = 0; i < 20; ++i) CK(hipGraphLaunch(ex, st));
  CK(hipStreamSynchronize(st));
  t = now_us();
  for (int i = 0; i < 200; ++i) CK(hipGraphLaunch(ex, st));
  const double graph = (now_us() - t) / 200;
  CK(hipStreamSynchronize(st));
  int h_bad = -1;
  CK(hipMemcpy(&h_bad, bad, sizeof(int), hipMemcpyDeviceToHost));
  std::printf("graph: host %.1f us/step, mismatches %d\n", graph, h_bad);
  CK(hipGraphExecDestroy(ex));
  CK(hipGraphDestroy(g));
  NK(ncclCommDestroy(comm));
  (void)hipStreamDestroy(st);
  (void)hipStreamDestroy(cs);
  (void)hipFree(sbuf);
  (void)hipFree(rbuf);
  (void)hipFree(bad);
  return h_bad == 0 ? 0 : 2;
}
