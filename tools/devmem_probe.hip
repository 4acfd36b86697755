// Microbenchmark (experiment only, not part of the product): host -> GPU hand-off of one pushed
// frame, the rollout's critical hop. The host writes a 7,056-byte frame into slot i of a ring,
// then a ready word = i; one GPU block polls the word, reads the frame and stores an ack into
// pinned host memory that the host polls. Round trip per iteration, host clock, for the ring and
// word in:
//   host  : pinned host memory (hipHostMalloc mapped; the product's zero-copy staging: the GPU
//           polls and reads over PCIe),
//   fine  : fine-grained device memory (hipExtMallocWithFlags hipDeviceMallocFinegrained) that the
//           host writes over PCIe (non-temporal 16-byte stores + sfence), so the GPU's poll and
//           frame reads are local,
//   uc    : the same with hipDeviceMallocUncached,
//   tagged: pinned host memory, no ready word: every 64-B chunk carries the push's tag (below).
//   hipcc --offload-arch=gfx950 -O3 -o tools/bin/devmem_probe tools/devmem_probe.hip
//   tools/bin/devmem_probe <host|fine|uc> [iters]
#include <hip/hip_runtime.h>
#include <immintrin.h>
#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstring>
#include <vector>

#define CK(x)                                                            \
  do {                                                                   \
    hipError_t e_ = (x);                                                 \
    if (e_ != hipSuccess) {                                              \
      printf("%s: %s\n", #x, hipGetErrorString(e_));                     \
      return 1;                                                          \
    }                                                                    \
  } while (0)

constexpr int FRAME = 7056, SLOTS = 64, SLOT_BYTES = 7168;  // (slots 128-B aligned)

__global__ __launch_bounds__(256) void pingpong(const uint32_t *flag, const uint8_t *ring, uint32_t *ack,
                                                int iters, uint32_t *sink) {
  __shared__ int ok;
  __shared__ uint32_t red[256];
  for (int i = 1; i <= iters; ++i) {
    if (threadIdx.x == 0) {
      const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
      uint32_t v;
      while ((v = __hip_atomic_load(flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM)) != (uint32_t)i &&
             __builtin_amdgcn_s_memrealtime() - t0 < 200000000ull) {
      }
      ok = v == (uint32_t)i;
    }
    __syncthreads();
    if (!ok) {
      if (threadIdx.x == 0) __hip_atomic_store(ack, 0xffffffffu, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      return;
    }
    // the frame, 16 B per lane (a fresh ring slot each iteration: no stale cache lines)
    const uint8_t *f = ring + (size_t)(i % SLOTS) * SLOT_BYTES;
    uint32_t acc = 0;
    for (int o = threadIdx.x * 16; o < FRAME; o += 256 * 16) {
      const uint4 x = *reinterpret_cast<const uint4 *>(f + o);
      acc ^= x.x ^ x.y ^ x.z ^ x.w;
    }
    red[threadIdx.x] = acc;
    __syncthreads();
    if (threadIdx.x == 0) {
      uint32_t a = 0;
      for (int t = 0; t < 256; ++t) a ^= red[t];
      sink[i % 16] = a;
      __hip_atomic_store(ack, (uint32_t)i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
    __syncthreads();
  }
}

// "tagged": no ready word. The frame is staged as 64-byte chunks of 60 bytes of pixels + a 4-byte
// tag (the push's sequence number) that the host writes with the chunk (one write-combined 64-B
// line); the GPU reads every chunk straight away and re-reads the chunks whose tag is stale, so
// one PCIe round trip carries both the publication and the pixels.
constexpr int TCHUNKS = (FRAME + 59) / 60, TSLOT = TCHUNKS * 64;
__global__ __launch_bounds__(256) void pingpong_tagged(const uint8_t *ring, uint32_t *ack, int iters,
                                                       uint32_t *sink) {
  for (int i = 1; i <= iters; ++i) {
    const uint8_t *f = ring + (size_t)(i % SLOTS) * TSLOT;
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    uint32_t acc = 0;
    // lane group of 4 = one 64-B chunk (pieces 0..3; the tag is the last word of piece 3)
    for (int c0 = 0; c0 < TCHUNKS; c0 += 64) {
      const int c = c0 + (threadIdx.x >> 2), pc = threadIdx.x & 3;
      bool have = c >= TCHUNKS;
      uint4 x = make_uint4(0, 0, 0, 0);
      while (true) {
        if (!have) {
          const uint64_t *q = reinterpret_cast<const uint64_t *>(f + (size_t)c * 64 + 16 * pc);
          const uint64_t lo = __hip_atomic_load(q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
          const uint64_t hi = __hip_atomic_load(q + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
          x = make_uint4((uint32_t)lo, (uint32_t)(lo >> 32), (uint32_t)hi, (uint32_t)(hi >> 32));
        }
        // the chunk's tag, from its piece-3 lane
        const uint32_t tag = __shfl(x.w, (threadIdx.x & 63 & ~3) | 3, 64);
        have = have || tag == (uint32_t)i;
        if (!__syncthreads_or(!have)) break;  // (block-uniform decisions only)
        if (__syncthreads_or(threadIdx.x == 0 && __builtin_amdgcn_s_memrealtime() - t0 > 200000000ull)) {
          if (threadIdx.x == 0) __hip_atomic_store(ack, 0xffffffffu, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
          return;
        }
      }
      acc ^= x.x ^ x.y ^ x.z;
    }
    __shared__ uint32_t red[256];
    red[threadIdx.x] = acc;
    __syncthreads();
    if (threadIdx.x == 0) {
      uint32_t a = 0;
      for (int t = 0; t < 256; ++t) a ^= red[t];
      sink[i % 16] = a;
      __hip_atomic_store(ack, (uint32_t)i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
    __syncthreads();
  }
}

int main(int argc, char **argv) {
  const char *mode = argc > 1 ? argv[1] : "host";
  const int iters = argc > 2 ? atoi(argv[2]) : 2000;
  uint8_t *ring = nullptr;
  uint32_t *flag = nullptr, *ack = nullptr, *sink = nullptr;
  const bool tagged = !strcmp(mode, "tagged");
  const size_t bytes = (size_t)SLOTS * (tagged ? TSLOT : SLOT_BYTES) + 256;
  if (!strcmp(mode, "host") || tagged) {
    CK(hipHostMalloc((void **)&ring, bytes, hipHostMallocMapped));
  } else {
    CK(hipExtMallocWithFlags((void **)&ring, bytes, !strcmp(mode, "uc") ? hipDeviceMallocUncached
                                                                         : hipDeviceMallocFinegrained));
    hipPointerAttribute_t at;
    CK(hipPointerGetAttributes(&at, ring));
    printf("device allocation: hostPointer=%p devicePointer=%p\n", at.hostPointer, at.devicePointer);
    if (at.hostPointer) {
      ring = (uint8_t *)at.hostPointer;
    } else if (argc > 3 && !strcmp(argv[3], "direct")) {  // try the device address from the host
      printf("no host pointer: writing through the device address\n");
      fflush(stdout);
    } else {
      printf("not host-accessible\n");
      return 2;
    }
  }
  flag = reinterpret_cast<uint32_t *>(ring + (size_t)SLOTS * (tagged ? TSLOT : SLOT_BYTES));
  if (tagged) memset(ring, 0, (size_t)SLOTS * TSLOT);
  CK(hipHostMalloc((void **)&ack, 64, hipHostMallocMapped));
  CK(hipMalloc((void **)&sink, 64));
  std::vector<uint8_t> src(FRAME);
  for (int k = 0; k < FRAME; ++k) src[k] = (uint8_t)(k * 131 + 7);
  *(volatile uint32_t *)flag = 0;
  *(volatile uint32_t *)ack = 0;
  _mm_sfence();
  if (tagged)
    hipLaunchKernelGGL(pingpong_tagged, dim3(1), dim3(256), 0, 0, ring, ack, iters, sink);
  else
    hipLaunchKernelGGL(pingpong, dim3(1), dim3(256), 0, 0, flag, ring, ack, iters, sink);
  CK(hipGetLastError());
  std::vector<double> rt;
  rt.reserve(iters);
  for (int i = 1; i <= iters; ++i) {
    const auto t0 = std::chrono::steady_clock::now();
    if (tagged) {  // 60 B of pixels + the tag per 64-B chunk, each chunk one write-combined line
      uint8_t *dst = ring + (size_t)(i % SLOTS) * TSLOT;
      alignas(16) uint8_t line[64];
      for (int c = 0; c < TCHUNKS; ++c) {
        const int n = std::min(60, FRAME - 60 * c);
        memcpy(line, &src[60 * c], n);
        memcpy(line + 60, &i, 4);
        for (int q = 0; q < 4; ++q)
          _mm_stream_si128(reinterpret_cast<__m128i *>(dst + 64 * c + 16 * q), _mm_load_si128(reinterpret_cast<const __m128i *>(line + 16 * q)));
      }
      _mm_sfence();
    } else {
      uint8_t *dst = ring + (size_t)(i % SLOTS) * SLOT_BYTES;
      for (int o = 0; o < FRAME; o += 16)
        _mm_stream_si128(reinterpret_cast<__m128i *>(dst + o), _mm_loadu_si128(reinterpret_cast<const __m128i *>(&src[o])));
      _mm_sfence();
      *(volatile uint32_t *)flag = (uint32_t)i;
      _mm_sfence();
    }
    uint32_t a;
    const auto tw = std::chrono::steady_clock::now();
    while ((a = *(volatile uint32_t *)ack) != (uint32_t)i) {
      if (a == 0xffffffffu || std::chrono::steady_clock::now() - tw > std::chrono::seconds(3)) {
        printf("timeout at iteration %d (ack %u)\n", i, a);
        CK(hipDeviceSynchronize());
        return 3;
      }
    }
    rt.push_back(std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count());
  }
  CK(hipDeviceSynchronize());
  std::sort(rt.begin(), rt.end());
  printf("%s: round trip (host write 7,056 B + ready word -> GPU poll + frame read -> ack) over %d: "
         "p10 %.2f  median %.2f  p90 %.2f us\n",
         mode, iters, rt[iters / 10], rt[iters / 2], rt[iters * 9 / 10]);
  return 0;
}
