// Host cost of the launch forms the rollout chain can use (tools only; not part of the library):
// hipLaunchKernelGGL of a small kernel, hipEventRecord, and hipGraphLaunch of graphs of 1 / 6 / 18
// kernel nodes, each timed on the host over many calls with the GPU kept busy behind a spin
// kernel (so the measured cost is the enqueue, not completion).
//   hipcc --offload-arch=gfx950 -O2 tools/launch_cost.hip -o tools/launch_cost && ./tools/launch_cost
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>
#include <vector>

#define CK(x)                                                                   \
  do {                                                                          \
    hipError_t e_ = (x);                                                        \
    if (e_ != hipSuccess) {                                                     \
      std::printf("%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));     \
      return 1;                                                                 \
    }                                                                           \
  } while (0)

__global__ void tiny(float *p, int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) p[i] += 1.f;
}

// keeps the stream busy for ~us microseconds (s_memrealtime: 100 MHz), bounded
__global__ void busy(unsigned us) {
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  while (__builtin_amdgcn_s_memrealtime() - t0 < 100ull * us) __builtin_amdgcn_s_sleep(2);
}

static double now_us() {
  return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

int main() {
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  float *d;
  CK(hipMalloc(&d, 1 << 20));
  hipEvent_t ev;
  CK(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
  const int reps = 200;
  // warm up
  for (int i = 0; i < 50; ++i) hipLaunchKernelGGL(tiny, dim3(288), dim3(256), 0, s, d, 1 << 18);
  CK(hipStreamSynchronize(s));

  // 1. plain launches, stream busy
  for (int grid : {32, 288}) {
    hipLaunchKernelGGL(busy, dim3(1), dim3(64), 0, s, 20000u);
    double t0 = now_us();
    for (int i = 0; i < reps; ++i) hipLaunchKernelGGL(tiny, dim3(grid), dim3(256), 0, s, d, 1 << 18);
    double t1 = now_us();
    CK(hipStreamSynchronize(s));
    std::printf("hipLaunchKernelGGL grid %3d: %.2f us / launch (stream busy)\n", grid, (t1 - t0) / reps);
  }
  // 2. event records
  {
    hipLaunchKernelGGL(busy, dim3(1), dim3(64), 0, s, 20000u);
    double t0 = now_us();
    for (int i = 0; i < reps; ++i) CK(hipEventRecord(ev, s));
    double t1 = now_us();
    CK(hipStreamSynchronize(s));
    std::printf("hipEventRecord: %.2f us / call\n", (t1 - t0) / reps);
  }
  // 3. launches interleaved with event records (the chain pattern: 3 kernels + 1 record)
  {
    hipLaunchKernelGGL(busy, dim3(1), dim3(64), 0, s, 20000u);
    double t0 = now_us();
    for (int i = 0; i < reps / 4; ++i) {
      hipLaunchKernelGGL(tiny, dim3(288), dim3(640), 0, s, d, 1 << 18);
      hipLaunchKernelGGL(tiny, dim3(144), dim3(256), 0, s, d, 1 << 18);
      hipLaunchKernelGGL(tiny, dim3(32), dim3(256), 0, s, d, 1 << 18);
      CK(hipEventRecord(ev, s));
    }
    double t1 = now_us();
    CK(hipStreamSynchronize(s));
    std::printf("chain (3 launches + record): %.2f us / chain (stream busy)\n", (t1 - t0) / (reps / 4));
  }
  // 4. graphs of n nodes
  for (int n : {1, 6, 18, 30}) {
    hipGraph_t g;
    hipGraphExec_t ge;
    hipStream_t cs;
    CK(hipStreamCreateWithFlags(&cs, hipStreamNonBlocking));
    CK(hipStreamBeginCapture(cs, hipStreamCaptureModeGlobal));
    for (int i = 0; i < n; ++i) hipLaunchKernelGGL(tiny, dim3(288), dim3(256), 0, cs, d, 1 << 18);
    CK(hipStreamEndCapture(cs, &g));
    CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
    for (int i = 0; i < 5; ++i) CK(hipGraphLaunch(ge, s));
    CK(hipStreamSynchronize(s));
    hipLaunchKernelGGL(busy, dim3(1), dim3(64), 0, s, 40000u);
    const int gr = 50;
    double t0 = now_us();
    for (int i = 0; i < gr; ++i) CK(hipGraphLaunch(ge, s));
    double t1 = now_us();
    CK(hipStreamSynchronize(s));
    // idle-stream latency: launch + wait for one graph
    double lat = 0;
    for (int i = 0; i < 20; ++i) {
      double a = now_us();
      CK(hipGraphLaunch(ge, s));
      CK(hipStreamSynchronize(s));
      lat += now_us() - a;
    }
    std::printf("hipGraphLaunch %2d nodes: %.2f us / launch (stream busy), launch+sync idle %.2f us\n", n,
                (t1 - t0) / gr, lat / 20);
    CK(hipGraphExecDestroy(ge));
    CK(hipGraphDestroy(g));
    CK(hipStreamDestroy(cs));
  }
  CK(hipFree(d));
  std::printf("ok\n");
  return 0;
}
