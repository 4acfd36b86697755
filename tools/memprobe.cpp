// Experiment: which allocation lets the host CPU write a step's new frames straight into memory
// the GPU then reads at HBM speed? For each allocation kind: is it host-addressable, how long
// the CPU takes to write 226 KB into it (8 threads, as the emulator threads would), and how long
// a 224-block kernel takes to read it (as the stacking kernel would).
//   hipcc --offload-arch=gfx950 -O2 -pthread tools/memprobe.cpp -o tools/memprobe && tools/memprobe
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstring>
#include <thread>
#include <vector>

#define CK(x)                                                                        \
  do {                                                                               \
    hipError_t e_ = (x);                                                             \
    if (e_ != hipSuccess) {                                                          \
      printf("  %s -> %s\n", #x, hipGetErrorString(e_));                             \
      return false;                                                                  \
    }                                                                                \
  } while (0)

__global__ void read_kernel(const uint4 *src, size_t n16, uint4 *dst) {
  for (size_t q = blockIdx.x * 256 + threadIdx.x; q < n16; q += (size_t)gridDim.x * 256) dst[q] = src[q];
}

static double now_us() {
  return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

static bool run(const char *name, int kind) {
  const size_t n = 32 * 7056;  // one step's frames at E = 32
  void *p = nullptr;
  printf("%s\n", name);
  switch (kind) {
    case 0: CK(hipHostMalloc(&p, n, hipHostMallocMapped)); break;
    case 1: CK(hipExtMallocWithFlags(&p, n, hipDeviceMallocFinegrained)); break;
    case 2: CK(hipMallocManaged(&p, n, hipMemAttachGlobal)); break;
    case 3: CK(hipExtMallocWithFlags(&p, n, hipDeviceMallocUncached)); break;
    case 4: CK(hipMalloc(&p, n)); break;
    case 5: CK(hipHostMalloc(&p, n, hipHostMallocMapped | hipHostMallocNonCoherent)); break;
  }
  hipPointerAttribute_t at{};
  if (hipPointerGetAttributes(&at, p) == hipSuccess)
    printf("  type %d hostPointer %p devicePointer %p isManaged %d\n", (int)at.type, at.hostPointer, at.devicePointer,
           (int)at.isManaged);
  void *dev = p;
  if (kind == 0 || kind == 5) CK(hipHostGetDevicePointer(&dev, p, 0));
  uint4 *dst;
  CK(hipMalloc(&dst, n));
  std::vector<uint8_t> src(n, 7);
  // host write (8 threads), only where the pointer is host-addressable
  bool host_ok = kind == 0 || kind == 2 || kind == 5 || (at.hostPointer != nullptr && kind != 4);
  if (kind == 1 || kind == 3) host_ok = at.hostPointer != nullptr;
  if (host_ok) {
    for (int rep = 0; rep < 3; ++rep) {
      const double t0 = now_us();
      std::vector<std::thread> th;
      for (int w = 0; w < 8; ++w)
        th.emplace_back([&, w] { std::memcpy((uint8_t *)p + w * n / 8, src.data() + w * n / 8, n / 8); });
      for (auto &t : th) t.join();
      const double t1 = now_us();
      std::memcpy(p, src.data(), n);
      const double t2 = now_us();
      printf("  host write 226 KB: 8 threads %.1f us (incl. thread start), 1 thread %.1f us\n", t1 - t0, t2 - t1);
    }
  } else {
    printf("  not host-addressable\n");
  }
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  for (int blocks : {224, 1024}) {
    for (int rep = 0; rep < 3; ++rep) {
      CK(hipEventRecord(a, 0));
      hipLaunchKernelGGL(read_kernel, dim3(blocks), dim3(256), 0, 0, (const uint4 *)dev, n / 16, dst);
      CK(hipEventRecord(b, 0));
      CK(hipEventSynchronize(b));
      float ms;
      CK(hipEventElapsedTime(&ms, a, b));
      if (rep == 2) printf("  GPU read 226 KB, %d blocks: %.2f us\n", blocks, ms * 1e3);
    }
  }
  (void)hipFree(dst);
  if (kind == 0 || kind == 5)
    (void)hipHostFree(p);
  else
    (void)hipFree(p);
  return true;
}

int main() {
  int v = 0;
  hipDeviceGetAttribute(&v, hipDeviceAttributeManagedMemory, 0);
  printf("managedMemory %d\n", v);
  hipDeviceGetAttribute(&v, hipDeviceAttributeConcurrentManagedAccess, 0);
  printf("concurrentManagedAccess %d\n", v);
  hipDeviceGetAttribute(&v, hipDeviceAttributePageableMemoryAccess, 0);
  printf("pageableMemoryAccess %d\n", v);
  hipDeviceGetAttribute(&v, hipDeviceAttributeHostNativeAtomicSupported, 0);
  printf("hostNativeAtomic %d\n", v);
  run("hipHostMalloc mapped (pinned host)", 0);
  run("hipHostMalloc mapped non-coherent", 5);
  run("hipExtMallocWithFlags finegrained (device)", 1);
  run("hipExtMallocWithFlags uncached (device)", 3);
  run("hipMallocManaged", 2);
  run("hipMalloc (device, reference)", 4);
  return 0;
}
