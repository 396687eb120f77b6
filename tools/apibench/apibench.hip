// Host cost of async HIP API calls on this image (diagnostic): kernel launch,
// memset, pinned H2D / D2H copy, event record, stream query; per call, no syncs
// inside the timed loop except where noted.
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>

__global__ void k_empty(int* p) {
  if (p && threadIdx.x == 1000000) p[0] = 1;
}

static double now() { return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count(); }

#define CK(x)                                                          \
  do {                                                                 \
    hipError_t e = (x);                                                \
    if (e != hipSuccess) {                                             \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e));          \
      return 1;                                                        \
    }                                                                  \
  } while (0)

int main() {
  hipStream_t st;
  CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  int* d;
  CK(hipMalloc(&d, 1 << 20));
  void* h;
  CK(hipHostMalloc(&h, 1 << 20, hipHostMallocDefault));
  hipEvent_t ev;
  CK(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
  const int N = 2000;
  for (int i = 0; i < 100; ++i) hipLaunchKernelGGL(k_empty, dim3(1), dim3(64), 0, st, d);
  CK(hipStreamSynchronize(st));
  double t0 = now();
  for (int i = 0; i < N; ++i) hipLaunchKernelGGL(k_empty, dim3(1), dim3(64), 0, st, d);
  double t1 = now();
  CK(hipStreamSynchronize(st));
  double t2 = now();
  printf("launch empty: host %.2f us/call, gpu drain %.2f us/kernel\n", (t1 - t0) / N * 1e6, (t2 - t0) / N * 1e6);
  t0 = now();
  for (int i = 0; i < N; ++i) CK(hipMemsetAsync(d, 0, 64, st));
  t1 = now();
  CK(hipStreamSynchronize(st));
  t2 = now();
  printf("memset 64B: host %.2f us/call, drain %.2f us/op\n", (t1 - t0) / N * 1e6, (t2 - t0) / N * 1e6);
  t0 = now();
  for (int i = 0; i < N; ++i) CK(hipMemcpyAsync(d, h, 512, hipMemcpyHostToDevice, st));
  t1 = now();
  CK(hipStreamSynchronize(st));
  t2 = now();
  printf("H2D 512B pinned: host %.2f us/call, drain %.2f us/op\n", (t1 - t0) / N * 1e6, (t2 - t0) / N * 1e6);
  t0 = now();
  for (int i = 0; i < N; ++i) CK(hipEventRecord(ev, st));
  t1 = now();
  printf("event record: host %.2f us/call\n", (t1 - t0) / N * 1e6);
  t0 = now();
  for (int i = 0; i < N; ++i) (void)hipStreamQuery(st);
  t1 = now();
  printf("stream query (idle): host %.2f us/call\n", (t1 - t0) / N * 1e6);
  // round trip: launch one kernel, spin on query until done
  double rt = 0;
  for (int i = 0; i < 200; ++i) {
    t0 = now();
    hipLaunchKernelGGL(k_empty, dim3(1), dim3(64), 0, st, d);
    while (hipStreamQuery(st) == hipErrorNotReady) {
    }
    rt += now() - t0;
  }
  printf("launch + query-spin round trip: %.2f us\n", rt / 200 * 1e6);
  rt = 0;
  for (int i = 0; i < 200; ++i) {
    t0 = now();
    hipLaunchKernelGGL(k_empty, dim3(1), dim3(64), 0, st, d);
    CK(hipStreamSynchronize(st));
    rt += now() - t0;
  }
  printf("launch + hipStreamSynchronize round trip: %.2f us\n", rt / 200 * 1e6);
  // big grid launch
  t0 = now();
  for (int i = 0; i < N; ++i) hipLaunchKernelGGL(k_empty, dim3(600), dim3(256), 0, st, d);
  t1 = now();
  CK(hipStreamSynchronize(st));
  t2 = now();
  printf("launch 600x256: host %.2f us/call, drain %.2f us/kernel\n", (t1 - t0) / N * 1e6, (t2 - t0) / N * 1e6);
  return 0;
}
