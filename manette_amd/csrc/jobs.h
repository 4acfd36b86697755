// Block-parallel jobs of the grouped launches (gemm.h launch_group) besides the GEMM products: the
// fixed-order split-K slab sum, the global-norm partials, a conv weight gradient's bias-row sums and
// the pair of two jobs as one. Shared by net.hip and tools/gemm_repro.hip.
#pragma once
#include "gemm.h"

namespace mt {

// out[i] = sum_z P[z*n + i], fixed order. A block owns kSlabCols float4 columns; its 256 threads
// are 16 slab subsets x kSlabCols columns, each thread adding slabs z = sub, sub+16, ... with 16
// loads in flight (a few hundred slabs: one round trip), then the 16 subset sums of a column are
// added in subset order. smem: 4 KB.
constexpr int kSlabCols = 16;
__device__ __forceinline__ void sum_slabs_body(const float *__restrict__ P, int S, size_t n, float *__restrict__ out,
                                               int bid, float *smem, float *__restrict__ sq_out = nullptr) {
  f32x4 *part = reinterpret_cast<f32x4 *>(smem);  // [16][kSlabCols]
  const int col = threadIdx.x % kSlabCols, sub = threadIdx.x / kSlabCols;
  const size_t n4 = n / 4;
  const size_t c = (size_t)bid * kSlabCols + col;  // float4 column
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  if (c < n4) {
    const f32x4 *p = reinterpret_cast<const f32x4 *>(P) + c;
    // batches of up to 16 predicated loads, all issued before the first add (a plain remainder
    // loop would wait out one load latency per slab); the adds stay in slab order
    for (int z = sub; z < S; z += 256) {
      f32x4 v[16];
#pragma unroll
      for (int u = 0; u < 16; ++u) v[u] = p[(size_t)min(z + 16 * u, S - 1) * n4];  // clamped: no branches
#pragma unroll
      for (int u = 0; u < 16; ++u)
        if (z + 16 * u < S) acc += v[u];
    }
  }
  part[sub * kSlabCols + col] = acc;
  __syncthreads();
  double sq = 0.0;  // sq_out: sum of the squares of this block's outputs (global-norm partial)
  if (sub == 0 && c < n4) {
    f32x4 t = part[col];
#pragma unroll
    for (int u = 1; u < 16; ++u) t += part[u * kSlabCols + col];
    reinterpret_cast<f32x4 *>(out)[c] = t;
    sq = (double)(t[0] * t[0]) + (double)(t[1] * t[1]) + (double)(t[2] * t[2]) + (double)(t[3] * t[3]);
  }
  // scalar tail (n not a multiple of 4)
  if (bid == 0) {
    for (size_t i = n4 * 4 + threadIdx.x; i < n; i += 256) {
      float t = 0.f;
      for (int z = 0; z < S; ++z) t += P[(size_t)z * n + i];
      out[i] = t;
      sq += (double)(t * t);
    }
  }
  if (sq_out) {
    double *red = reinterpret_cast<double *>(smem);
    sq = wave_sum_d(sq);
    __syncthreads();  // part[] is no longer read
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = sq;
    __syncthreads();
    if (threadIdx.x == 0) *sq_out = (float)(red[0] + red[1] + red[2] + red[3]);
  }
}

// Global-norm partials of g outside [skip_b, skip_e) (float offsets, multiples of 4), as a job of a
// grouped launch: block b writes partials[b] = sum of the squares of its grid-stride share
// (sumsq_kernel's arithmetic; the grid of this job is fixed, so the partials are deterministic).
struct SumsqJob {
  const float *g = nullptr;
  size_t n = 0, skip_b = 0, skip_e = 0;
  float *partials = nullptr;
  int nb = 0;
  __host__ __device__ int blocks() const { return nb; }
  size_t lds() const { return 64; }
  __device__ __forceinline__ void run(int bid, float *smem) const {
    double acc = 0.0;
    const size_t n4 = n / 4, sb = skip_b / 4, se = skip_e / 4;
    const size_t stride = (size_t)nb * 256;
    for (size_t i = (size_t)bid * 256 + threadIdx.x; i < n4; i += stride) {
      if (i >= sb && i < se) continue;
      const f32x4 v = reinterpret_cast<const f32x4 *>(g)[i];
      acc += (double)(v[0] * v[0]) + (double)(v[1] * v[1]) + (double)(v[2] * v[2]) + (double)(v[3] * v[3]);
    }
    for (size_t i = n4 * 4 + (size_t)bid * 256 + threadIdx.x; i < n; i += stride) acc += (double)(g[i] * g[i]);
    double *red = reinterpret_cast<double *>(smem);
    acc = wave_sum_d(acc);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = acc;
    __syncthreads();
    if (threadIdx.x == 0) partials[bid] = (float)(red[0] + red[1] + red[2] + red[3]);
  }
};

// Slab sum as a job of a grouped launch (gemm.h); n = 0: no job.
struct SlabJob {
  const float *P = nullptr;
  int S = 0;
  size_t n = 0;
  float *out = nullptr;
  float *sq = nullptr;  // optional: per-block global-norm partials sq[block]
  __host__ __device__ int blocks() const {
    const size_t b = (n / 4 + kSlabCols - 1) / kSlabCols;
    return n ? (int)(b ? b : 1) : 0;
  }
  size_t lds() const { return 4096; }
  __device__ __forceinline__ void run(int id, float *smem) const {
    sum_slabs_body(P, S, n, out, id, smem, sq ? sq + id : nullptr);
  }
};

// Bias gradient rows of a split conv weight gradient: block z sums dY over split z's GEMM-K range
// [z*kchunk, min(K, (z+1)*kchunk)) (pixels) for every channel and writes the sum to row KK of slab
// z (the slab sum then adds the splits in z order, as for the weight rows). 256 threads = 16 row
// subsets x 16 channel lanes; subsets summed in fixed order through LDS.
template <int COUT>
struct BiasRowJob {
  const float *dY = nullptr;  // [K][COUT]
  float *out = nullptr;       // slab row KK of split z at out + z * zstride
  size_t zstride = 0;
  int K = 0, kchunk = 0, nz = 0;
  __host__ __device__ int blocks() const { return nz; }
  size_t lds() const { return sizeof(float) * 256; }
  __device__ __forceinline__ void run(int z, float *smem) const {
    static_assert(COUT % 16 == 0 || COUT < 16, "channel lanes");
    const int k0 = z * kchunk, k1 = min(K, k0 + kchunk);
    const int sub = threadIdx.x >> 4, c = threadIdx.x & 15;
    for (int n0 = 0; n0 < COUT; n0 += 16) {
      float acc = 0.f;
      if (n0 + c < COUT)
        for (int k = k0 + sub; k < k1; k += 16 * 8) {  // 8 loads in flight, added in row order
          float v[8];
#pragma unroll
          for (int u = 0; u < 8; ++u) v[u] = dY[(size_t)min(k + 16 * u, k1 - 1) * COUT + n0 + c];
#pragma unroll
          for (int u = 0; u < 8; ++u)
            if (k + 16 * u < k1) acc += v[u];
        }
      smem[threadIdx.x] = acc;
      __syncthreads();
      if (sub == 0 && n0 + c < COUT) {
        float t = smem[c];
#pragma unroll
        for (int u = 1; u < 16; ++u) t += smem[u * 16 + c];
        out[(size_t)z * zstride + n0 + c] = t;
      }
      __syncthreads();
    }
  }
};

// Two jobs as one (blocks of the first, then the second): the dW GEMM and its bias-row sums.
template <class J1, class J2>
struct PairJob {
  J1 a;
  J2 b;
  __host__ __device__ int blocks() const { return a.blocks() + b.blocks(); }
  size_t lds() const { return std::max(a.blocks() ? a.lds() : 0, b.blocks() ? b.lds() : 0); }
  __device__ __forceinline__ void run(int id, float *smem) const {
    if (id < a.blocks())
      a.run(id, smem);
    else
      b.run(id - a.blocks(), smem);
  }
};

}  // namespace mt
