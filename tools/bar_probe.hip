// Host -> GPU hand-off probe: where should the emulator threads publish an env's frames
// and ready word — pinned host memory the GPU polls over PCIe (the current stacking rollout), or
// fine-grained device memory (hipExtMallocWithFlags(hipDeviceMallocFinegrained)) the CPU writes
// through the PCIe BAR, so the GPU's polls and frame reads stay local?
//   1. can the host write fine-grained VRAM at all, and does a kernel see the bytes;
//   2. ping-pong round trip: one lane polls a flag (system-scope loads, bounded wait) and answers
//      into a pinned host word the host polls; the host's flag store goes to pinned host memory
//      (mode 0, today's ready words) or to fine-grained VRAM (mode 1);
//   3. host write bandwidth of 28 KB frames into pinned host memory vs fine-grained VRAM.
// hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/bar_probe.hip -o tools/bin/bar_probe
#include <hip/hip_runtime.h>

#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <vector>

#define CK(x)                                                                          \
  do {                                                                                 \
    hipError_t e_ = (x);                                                               \
    if (e_ != hipSuccess) {                                                            \
      fprintf(stderr, "%s: %s (line %d)\n", #x, hipGetErrorString(e_), __LINE__);      \
      exit(2);                                                                         \
    }                                                                                  \
  } while (0)

__global__ void sum_kernel(const uint32_t *p, size_t n, uint64_t *out) {
  uint64_t s = 0;
  for (size_t i = threadIdx.x; i < n; i += blockDim.x) s += __hip_atomic_load(p + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  atomicAdd(reinterpret_cast<unsigned long long *>(out), (unsigned long long)s);
}

// Lane 0: for k = 1..iters wait until *flag == k (bounded: ~1 s per wait), then store k into *ack
// (pinned host memory). status[0] = iterations completed, status[1] = 1 on timeout.
__global__ void pong_kernel(const uint32_t *flag, uint32_t *ack, int iters, uint32_t *status) {
  if (threadIdx.x != 0) return;
  int k = 1;
  for (; k <= iters; ++k) {
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    while (__hip_atomic_load(flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != (uint32_t)k) {
      __builtin_amdgcn_s_sleep(1);
      if (__builtin_amdgcn_s_memrealtime() - t0 > 100000000ull) {
        status[1] = 1;
        status[0] = k - 1;
        return;
      }
    }
    __hip_atomic_store(ack, (uint32_t)k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
  status[0] = k - 1;
}

static double now_us() {
  return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

static double ping(uint32_t *flag_host_view, uint32_t *flag_dev_view, uint32_t *ack_host, uint32_t *ack_dev,
                   uint32_t *status, int iters, bool *ok) {
  std::atomic_thread_fence(std::memory_order_seq_cst);
  *reinterpret_cast<volatile uint32_t *>(flag_host_view) = 0;
  *reinterpret_cast<volatile uint32_t *>(ack_host) = 0;
  std::atomic_thread_fence(std::memory_order_seq_cst);
  CK(hipMemset(status, 0, 8));
  CK(hipDeviceSynchronize());
  hipLaunchKernelGGL(pong_kernel, dim3(1), dim3(64), 0, 0, flag_dev_view, ack_dev, iters, status);
  CK(hipGetLastError());
  const double t0 = now_us();
  double tk = t0;
  *ok = true;
  for (int k = 1; k <= iters; ++k) {
    __atomic_store_n(flag_host_view, (uint32_t)k, __ATOMIC_RELEASE);
    while (__atomic_load_n(reinterpret_cast<volatile uint32_t *>(ack_host), __ATOMIC_ACQUIRE) != (uint32_t)k) {
      if (now_us() - tk > 2e6) {
        *ok = false;
        break;
      }
    }
    if (!*ok) break;
    if (k == 10) tk = now_us();  // (the first iterations include the kernel launch)
  }
  const double t1 = now_us();
  CK(hipDeviceSynchronize());
  uint32_t st[2];
  CK(hipMemcpy(st, status, 8, hipMemcpyDeviceToHost));
  if (st[1] || (int)st[0] != iters) *ok = false;
  return (t1 - tk) / (iters - 10);
}

int main() {
  const size_t BYTES = 1 << 20;
  uint32_t *fine = nullptr;
  hipError_t e = hipExtMallocWithFlags(reinterpret_cast<void **>(&fine), BYTES, hipDeviceMallocFinegrained);
  printf("hipExtMallocWithFlags(fine-grained) -> %s, %p\n", hipGetErrorString(e), (void *)fine);
  if (e != hipSuccess) return 1;
  hipPointerAttribute_t attr;
  if (hipPointerGetAttributes(&attr, fine) == hipSuccess)
    printf("  attributes: type %d, device %d, hostPointer %p, devicePointer %p\n", (int)attr.type, attr.device,
           attr.hostPointer, attr.devicePointer);
  // 1. host writes, kernel reads (a host fault here is a segfault of this program, not a GPU fault)
  uint32_t *host_view = fine;  // the same virtual address, if the BAR mapping exists
  for (size_t i = 0; i < 4096; ++i) reinterpret_cast<volatile uint32_t *>(host_view)[i] = (uint32_t)(i * 3 + 1);
  std::atomic_thread_fence(std::memory_order_seq_cst);
  uint64_t *sum;
  CK(hipMalloc(&sum, 8));
  CK(hipMemset(sum, 0, 8));
  hipLaunchKernelGGL(sum_kernel, dim3(1), dim3(256), 0, 0, fine, (size_t)4096, sum);
  CK(hipDeviceSynchronize());
  uint64_t got = 0, want = 0;
  CK(hipMemcpy(&got, sum, 8, hipMemcpyDeviceToHost));
  for (size_t i = 0; i < 4096; ++i) want += i * 3 + 1;
  printf("1. host-written fine-grained VRAM read by a kernel: sum %llu, expected %llu -> %s\n",
         (unsigned long long)got, (unsigned long long)want, got == want ? "OK" : "MISMATCH");
  // 2. ping-pong
  uint32_t *pinned, *pinned_dev, *status;
  CK(hipHostMalloc(reinterpret_cast<void **>(&pinned), 4096, hipHostMallocMapped));
  CK(hipHostGetDevicePointer(reinterpret_cast<void **>(&pinned_dev), pinned, 0));
  CK(hipMalloc(&status, 8));
  const int iters = 2000;
  bool ok0, ok1;
  // mode 0: flag in pinned host memory (word 32), ack in pinned host memory (word 0)
  const double rt0 = ping(pinned + 32, pinned_dev + 32, pinned, pinned_dev, status, iters, &ok0);
  // mode 1: flag in fine-grained VRAM, ack in pinned host memory
  const double rt1 = ping(fine + 8192, fine + 8192, pinned, pinned_dev, status, iters, &ok1);
  printf("2. ping-pong round trip (host flag store -> GPU poll sees it -> GPU ack store -> host sees it):\n"
         "   flag in pinned host memory: %.2f us %s\n   flag in fine-grained VRAM:  %.2f us %s\n", rt0,
         ok0 ? "" : "(TIMEOUT)", rt1, ok1 ? "" : "(TIMEOUT)");
  // 3. host write bandwidth of 28,224-byte frames (16-B stores)
  const size_t FR = 28224, NF = 32;
  uint8_t *pin_frames;
  CK(hipHostMalloc(reinterpret_cast<void **>(&pin_frames), FR * NF, hipHostMallocMapped));
  std::vector<uint8_t> src(FR * NF, 7);
  auto bw = [&](uint8_t *dst) {
    double best = 1e30;
    for (int r = 0; r < 20; ++r) {
      const double t0 = now_us();
      memcpy(dst, src.data(), FR * NF);
      std::atomic_thread_fence(std::memory_order_seq_cst);
      best = std::min(best, now_us() - t0);
    }
    return FR * NF / best * 1e-3;  // GB/s
  };
  printf("3. host memcpy of 32 frames (%zu B): pinned host %.1f GB/s, fine-grained VRAM %.1f GB/s\n", FR * NF,
         bw(pin_frames), bw(reinterpret_cast<uint8_t *>(fine)));
  return (got == want && ok0 && ok1) ? 0 : 1;
}
