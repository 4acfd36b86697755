// Microbenchmark (experiment only, not part of the product): latency of an in-launch producer ->
// consumer hand-off (sc1 payload stores + agent-scope counter, consumer polls then sc1 loads)
// versus a kernel boundary (plain stores, next kernel's plain loads), at the NIPS trunk's shape:
// 288 producer blocks (32 envs x 9 rows) each writing 288 floats, 144 consumer blocks (16 column
// blocks x 9 rows) each reading the 32 envs' rows of its row.
//   hipcc --offload-arch=gfx950 -O3 -o /tmp/handoff tools/handoff_probe.hip && /tmp/handoff
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
#include <algorithm>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e_)); return 1; } } while (0)

constexpr int E = 32, ROWS = 9, FEAT = 288, NP = E * ROWS, NC = 16 * ROWS;

__device__ __forceinline__ unsigned long long now() { return __builtin_amdgcn_s_memrealtime(); }

// fused: blocks [0, NP) produce, [NP, NP + NC) consume
__global__ __launch_bounds__(256) void fused(float *act, unsigned *cnt, unsigned target, unsigned long long *tp,
                                             unsigned long long *tc, float *sink) {
  const int b = blockIdx.x;
  if (b < NP) {
    const int e = b / ROWS, i = b % ROWS;
    // some "work" so producers finish at slightly different times
    float v = (float)b;
    for (int k = 0; k < 200 + 20 * (b % 7); ++k) v = v * 0.999f + 1.0f;
    for (int f = threadIdx.x; f < FEAT; f += 256)
      __hip_atomic_store(act + ((size_t)e * ROWS + i) * FEAT + f, v + f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) {
      tp[b] = now();
      __hip_atomic_fetch_add(cnt + i * 32, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    return;
  }
  const int c = b - NP, i = c % ROWS;
  __shared__ int ok;
  if (threadIdx.x == 0) {
    const unsigned long long t0 = now();
    int good = 1;
    while (__hip_atomic_load(cnt + i * 32, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target) {
      __builtin_amdgcn_s_sleep(1);
      if (now() - t0 > 200000000ull) { good = 0; break; }
    }
    ok = good;
    tc[c * 2] = now();
  }
  __syncthreads();
  if (!ok) return;
  float acc = 0.f;
  for (int q = threadIdx.x; q < E * FEAT; q += 256) {
    const int e = q / FEAT, f = q % FEAT;
    acc += __hip_atomic_load(act + ((size_t)e * ROWS + i) * FEAT + f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  sink[c * 256 + threadIdx.x] = acc;
  __syncthreads();
  if (threadIdx.x == 0) tc[c * 2 + 1] = now();
}

__global__ __launch_bounds__(256) void prod(float *act, unsigned long long *tp) {
  const int b = blockIdx.x, e = b / ROWS, i = b % ROWS;
  float v = (float)b;
  for (int k = 0; k < 200 + 20 * (b % 7); ++k) v = v * 0.999f + 1.0f;
  for (int f = threadIdx.x; f < FEAT; f += 256) act[((size_t)e * ROWS + i) * FEAT + f] = v + f;
  __syncthreads();
  if (threadIdx.x == 0) tp[b] = now();
}
__global__ __launch_bounds__(256) void cons(const float *act, unsigned long long *tc, float *sink) {
  const int c = blockIdx.x, i = c % ROWS;
  if (threadIdx.x == 0) tc[c * 2] = now();
  float acc = 0.f;
  for (int q = threadIdx.x; q < E * FEAT; q += 256) {
    const int e = q / FEAT, f = q % FEAT;
    acc += act[((size_t)e * ROWS + i) * FEAT + f];
  }
  sink[c * 256 + threadIdx.x] = acc;
  __syncthreads();
  if (threadIdx.x == 0) tc[c * 2 + 1] = now();
}

int main() {
  float *act, *sink;
  unsigned *cnt;
  unsigned long long *tp, *tc;
  CK(hipMalloc(&act, sizeof(float) * NP * FEAT));
  CK(hipMalloc(&sink, sizeof(float) * NC * 256));
  CK(hipMalloc(&cnt, sizeof(unsigned) * ROWS * 32));
  CK(hipMalloc(&tp, 8 * NP));
  CK(hipMalloc(&tc, 16 * NC));
  CK(hipMemset(cnt, 0, sizeof(unsigned) * ROWS * 32));
  std::vector<unsigned long long> hp(NP), hc(2 * NC);
  std::vector<float> hs(NC * 256), ref(NC * 256);
  auto report = [&](const char *name) {
    unsigned long long pmax = *std::max_element(hp.begin(), hp.end());
    unsigned long long pmin = *std::min_element(hp.begin(), hp.end());
    std::vector<double> seen, done;
    for (int c = 0; c < NC; ++c) {
      seen.push_back((double)((long long)hc[2 * c] - (long long)pmax) * 0.01);
      done.push_back((double)((long long)hc[2 * c + 1] - (long long)pmax) * 0.01);
    }
    std::sort(seen.begin(), seen.end());
    std::sort(done.begin(), done.end());
    printf("%-9s producers span %.2f us; consumer start vs last producer: min %+.2f med %+.2f max %+.2f us; "
           "loads done: med %+.2f max %+.2f us\n", name, (pmax - pmin) * 0.01, seen.front(), seen[NC / 2], seen.back(),
           done[NC / 2], done.back());
  };
  for (int rep = 0; rep < 5; ++rep) {
    hipLaunchKernelGGL(prod, dim3(NP), dim3(256), 0, 0, act, tp);
    hipLaunchKernelGGL(cons, dim3(NC), dim3(256), 0, 0, act, tc, sink);
    CK(hipDeviceSynchronize());
  }
  CK(hipMemcpy(hp.data(), tp, 8 * NP, hipMemcpyDeviceToHost));
  CK(hipMemcpy(hc.data(), tc, 16 * NC, hipMemcpyDeviceToHost));
  CK(hipMemcpy(ref.data(), sink, 4 * NC * 256, hipMemcpyDeviceToHost));
  report("2-kernel");
  int bad = 0;
  for (int rep = 1; rep <= 200; ++rep) {
    CK(hipMemset(act, 0, sizeof(float) * NP * FEAT));
    hipLaunchKernelGGL(fused, dim3(NP + NC), dim3(256), 0, 0, act, cnt, (unsigned)(rep * E), tp, tc, sink);
    CK(hipDeviceSynchronize());
    CK(hipMemcpy(hs.data(), sink, 4 * NC * 256, hipMemcpyDeviceToHost));
    for (int k = 0; k < NC * 256; ++k)
      if (hs[k] != ref[k]) { ++bad; break; }
  }
  CK(hipMemcpy(hp.data(), tp, 8 * NP, hipMemcpyDeviceToHost));
  CK(hipMemcpy(hc.data(), tc, 16 * NC, hipMemcpyDeviceToHost));
  report("fused");
  printf("fused runs with a stale or wrong sum: %d / 200\n", bad);
  return 0;
}
