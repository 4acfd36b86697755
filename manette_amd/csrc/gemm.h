// fp32 MFMA (v_mfma_f32_16x16x4_f32) tiled GEMM core with pluggable operand loaders.
//
//   C[m][n] = sum_k A(m, k) * B(k, n)
//
// Every conv / dense forward and backward product of the trunk is one instantiation: the
// loaders gather their operand (im2col of an NHWC activation, a dense matrix, a transposed
// dense matrix, the transposed-conv gather of a backward-data pass) straight from HBM into
// LDS, so no im2col buffer is ever materialised. fp32 in / fp32 accumulate: the MFMA is an
// exact k-ordered fmaf chain (cdna_hip_programming.md §3), the numerics of TF's fp32 path.
//
// Tile: 256 threads = 4 waves laid out WM x WN; each wave owns TM x TN 16x16 accumulators.
// K is walked in BK-deep chunks staged through LDS with a register-staged prefetch: the global
// loads of chunk i+1 are issued before the MFMAs of chunk i (all of a thread's loads of a chunk
// are in flight together). Small-K layers (conv fwd, K <= 256) use BK = K: one fill, one
// latency. Split-K over blockIdx.z.
//
// LDS operand layouts (per loader, chosen to mirror the operand's memory layout):
//   KMAJOR  : L[row][BK + 4]   (k contiguous)  -> fragment = one ds_read_b128
//   !KMAJOR : L[k][ROWS + 4]   (row contiguous) -> fragment = four ds_read_b32
// Fragment element s of lane l (r = l&15, g = l>>4) holds k = kc*16 + g*4 + s for BOTH
// operands, so MFMA s multiplies A[r][k] by B[k][r'] with the same k (the k order inside a
// 16-chunk is permuted, which a sum does not see).
#pragma once
#include <algorithm>
#include <type_traits>

#include "common.h"

namespace mt {

template <int BM_, int BN_, int WM_, int WN_, int BK_ = 32>
struct Tile {
  static constexpr int BM = BM_, BN = BN_, WM = WM_, WN = WN_, BK = BK_;
  static constexpr int TM = BM / (WM * 16);
  static constexpr int TN = BN / (WN * 16);
  static_assert(WM * WN == 4, "4 waves per workgroup");
  static_assert(TM >= 1 && TN >= 1 && TM * WM * 16 == BM && TN * WN * 16 == BN, "tile shape");
  static_assert(BK % 16 == 0, "BK multiple of 16");
};

template <bool KMAJOR, int ROWS, int BK>
struct LdsShape {
  static constexpr int SIZE = KMAJOR ? ROWS * (BK + 4) : BK * (ROWS + 4);
  static constexpr int QUADS = ROWS * BK / 4;             // f32x4 items per fill
  static constexpr int ITEMS = (QUADS + 255) / 256;        // per thread
};

template <bool KMAJOR, int ROWS, int BK>
__device__ __forceinline__ f32x4 load_frag(const float *L, int row, int k) {
  if constexpr (KMAJOR) {
    return *reinterpret_cast<const f32x4 *>(L + row * (BK + 4) + k);
  } else {
    constexpr int LD = ROWS + 4;
    f32x4 v;
    v[0] = L[(k + 0) * LD + row];
    v[1] = L[(k + 1) * LD + row];
    v[2] = L[(k + 2) * LD + row];
    v[3] = L[(k + 3) * LD + row];
    return v;
  }
}

// Item it of a fill -> (row offset, k offset) inside the tile, by layout.
template <bool KMAJOR, int ROWS, int BK>
__device__ __forceinline__ void item_pos(int it, int &rr, int &kk) {
  if constexpr (KMAJOR) {
    rr = it / (BK / 4);
    kk = (it % (BK / 4)) * 4;  // 4 consecutive k of one row
  } else {
    kk = it / (ROWS / 4);
    rr = (it % (ROWS / 4)) * 4;  // 4 consecutive rows at one k
  }
}

template <bool KMAJOR, int ROWS, int BK>
__device__ __forceinline__ void lds_put(float *L, int rr, int kk, f32x4 v) {
  if constexpr (KMAJOR)
    *reinterpret_cast<f32x4 *>(L + rr * (BK + 4) + kk) = v;
  else
    *reinterpret_cast<f32x4 *>(L + kk * (ROWS + 4) + rr) = v;
}

// Optional per-item k state: a loader with `struct KS` gets ks(ctx, k) once at its split's first
// k, fetch_ks(ctx, ks) on interior chunks and next<BK>(ks) after every load. The chunks of a split
// are consecutive BK steps, so the per-k index math (the pixel decomposition of an im2col GEMM-K:
// divisions, quarter-rate integer multiplies) becomes a few adds per chunk.
template <class L, class = void>
struct HasKs : std::false_type {
  struct KS {};
};
template <class L>
struct HasKs<L, std::void_t<typename L::KS>> : std::true_type {
  using KS = typename L::KS;
};

// Stage of one operand: registers for one chunk.
// A thread's items keep their row (or row quad) for the whole K walk, only k advances, so each
// loader splits its address math into a per-row context (the row -> (image, pixel) or
// (tap, channel) decomposition, computed once per tile in init) and the per-k remainder
// (fetch_ctx, or the k state above): the integer divisions of an implicit im2col run once, not
// once per chunk.
template <class LD, int ROWS, int BK>
struct Stage {
  using S = LdsShape<LD::KMAJOR, ROWS, BK>;
  static constexpr bool KST = HasKs<LD>::value;
  f32x4 r[S::ITEMS];
  typename LD::Ctx cx[S::ITEMS];
  typename HasKs<LD>::KS ks[KST ? S::ITEMS : 1];
  __device__ __forceinline__ void init(const LD &ld, int row0, int kb) {
#pragma unroll
    for (int i = 0; i < S::ITEMS; ++i) {
      const int it = threadIdx.x + i * 256;
      if (S::QUADS % 256 == 0 || it < S::QUADS) {
        int rr, kk;
        item_pos<LD::KMAJOR, ROWS, BK>(it, rr, kk);
        cx[i] = ld.ctx(row0 + rr);
        if constexpr (KST) ks[i] = ld.ks(cx[i], kb + kk);
      }
    }
  }
  // Interior tiles (uniform per workgroup) take the branch-free fetch: every load of the chunk
  // is issued back to back and waited for once (a per-element guarded load would make hipcc
  // wait vmcnt(0) per element — cdna_hip_programming.md §5 trap (c)).
  __device__ __forceinline__ void load(const LD &ld, int row0, int k0, int ke, int nrows) {
    if (ld.interior(row0, ROWS, k0, BK, ke, nrows)) {
#pragma unroll
      for (int i = 0; i < S::ITEMS; ++i) {
        const int it = threadIdx.x + i * 256;
        if (S::QUADS % 256 == 0 || it < S::QUADS) {
          int rr, kk;
          item_pos<LD::KMAJOR, ROWS, BK>(it, rr, kk);
          if constexpr (KST)
            r[i] = ld.fetch_ks(cx[i], ks[i]);
          else
            r[i] = ld.fetch_ctx(cx[i], k0 + kk);
        }
      }
    } else {
#pragma unroll
      for (int i = 0; i < S::ITEMS; ++i) {
        const int it = threadIdx.x + i * 256;
        if (S::QUADS % 256 == 0 || it < S::QUADS) {
          int rr, kk;
          item_pos<LD::KMAJOR, ROWS, BK>(it, rr, kk);
          r[i] = ld.fetch(row0, rr, k0, kk, ke, nrows);
        }
      }
    }
    if constexpr (KST) {
#pragma unroll
      for (int i = 0; i < S::ITEMS; ++i) ld.template next<BK>(ks[i]);
    }
  }
  __device__ __forceinline__ void store(float *L) const {
#pragma unroll
    for (int i = 0; i < S::ITEMS; ++i) {
      const int it = threadIdx.x + i * 256;
      if (S::QUADS % 256 == 0 || it < S::QUADS) {
        int rr, kk;
        item_pos<LD::KMAJOR, ROWS, BK>(it, rr, kk);
        lds_put<LD::KMAJOR, ROWS, BK>(L, rr, kk, r[i]);
      }
    }
  }
};

// Quad epilogues (EP::QUAD): ep.quad(m, n, z, v) receives the 4 consecutive rows m..m+3 (m % 4
// == 0) of column n that one lane's accumulator holds — a 2x2 max pool over pool-ordered rows
// (LdIm2col<G, U8, true>) becomes a register reduction. M must be a multiple of 4.
// Two-phase epilogues (EP::Pre): ep.pre(m, n) loads the operands of output (m, n) — called for
// every output of the lane (clamped to the last valid row / column) when the block starts, right
// behind its first chunk's loads, long before any ep(pre, ...) or ep.quad(pre, ...) stores.
template <class E, class = void>
struct HasPre : std::false_type {};
template <class E>
struct HasPre<E, std::void_t<typename E::Pre>> : std::true_type {};

template <class E, bool = HasPre<E>::value>
struct PreOf {
  struct type {};
};
template <class E>
struct PreOf<E, true> {
  using type = typename E::Pre;
};

template <class E, class = void>
struct IsQuadEp : std::false_type {};
template <class E>
struct IsQuadEp<E, std::void_t<decltype(E::QUAD)>> : std::bool_constant<E::QUAD> {};

// One output tile (bx, by) of K-split bz; smem = the dynamic LDS (gemm_lds_bytes). A device
// function so grouped launches (GemmJob, group_kernel) can run several products in one grid.
// B loaders whose operand depends on the output row tile (LdConvBwdBPhase: the stride phase of
// its rows) provide for_mtile(bx); the others are used as they are.
template <class L, class = void>
struct HasForMtile : std::false_type {};
template <class L>
struct HasForMtile<L, std::void_t<decltype(std::declval<const L &>().for_mtile(0))>> : std::true_type {};

template <class T, class LA, class LB, class EP>
__device__ __forceinline__ void gemm_body_t(const LA &la, const LB &lb, const EP &ep, int M, int N, int K,
                                            int kchunk, int bx, int by, int bz, float *smem);

template <class T, class LA, class LB, class EP>
__device__ __forceinline__ void gemm_body(const LA &la, const LB &lb, const EP &ep, int M, int N, int K, int kchunk,
                                          int bx, int by, int bz, float *smem) {
  if constexpr (HasForMtile<LB>::value)
    gemm_body_t<T>(la, lb.for_mtile(bx), ep, M, N, K, kchunk, bx, by, bz, smem);
  else
    gemm_body_t<T>(la, lb, ep, M, N, K, kchunk, bx, by, bz, smem);
}

template <class T, class LA, class LB, class EP>
__device__ __forceinline__ void gemm_body_t(const LA &la, const LB &lb, const EP &ep, int M, int N, int K,
                                            int kchunk, int bx, int by, int bz, float *smem) {
  using SA = LdsShape<LA::KMAJOR, T::BM, T::BK>;
  using SB = LdsShape<LB::KMAJOR, T::BN, T::BK>;
  float *As = smem;
  float *Bs = smem + SA::SIZE;

  const int m0 = bx * T::BM;
  const int n0 = by * T::BN;
  const int kb = bz * kchunk;
  const int ke = min(K, kb + kchunk);
  const int lane = threadIdx.x & 63;
  const int w = threadIdx.x >> 6;
  const int wm = w / T::WN, wn = w % T::WN;
  const int r = lane & 15, g = lane >> 4;

  f32x4 acc[T::TM][T::TN];
#pragma unroll
  for (int i = 0; i < T::TM; ++i)
#pragma unroll
    for (int j = 0; j < T::TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // Register prefetch: chunk c's global loads are issued while chunk c - 1 is multiplied (a second
  // register buffer two chunks ahead measured no faster).
  Stage<LA, T::BM, T::BK> sa;
  Stage<LB, T::BN, T::BK> sb;
  sa.init(la, m0, kb);
  sb.init(lb, n0, kb);
  if (kb < ke) {
    sa.load(la, m0, kb, ke, M);
    sb.load(lb, n0, kb, ke, N);
  }
  // Two-phase epilogue (EP::Pre): every operand load of the lane's outputs (a bias, the activation
  // whose derivative masks a dX, a pool's argmax) depends only on the tile, so it is issued here,
  // behind the first chunk's loads, and its latency hides under the K walk — a block of these
  // latency-bound products otherwise waits one more memory round trip after its last MFMA. (Issued
  // before any store: the stores may alias the loaded arrays as far as the compiler knows.)
  constexpr int NQ = IsQuadEp<EP>::value ? 1 : 4;
  typename PreOf<EP>::type pre[T::TM][T::TN][NQ];
  if constexpr (HasPre<EP>::value) {
#pragma unroll
    for (int i = 0; i < T::TM; ++i)
#pragma unroll
      for (int j = 0; j < T::TN; ++j) {
        const int n = min(n0 + (wn * T::TN + j) * 16 + r, N - 1);
#pragma unroll
        for (int q = 0; q < NQ; ++q) {
          const int m = min(m0 + (wm * T::TM + i) * 16 + g * 4 + q, NQ == 1 ? M - 4 : M - 1);
          pre[i][j][q] = ep.pre(m, n);
        }
      }
  }
  // the MFMAs of one staged chunk starting at k0
  auto compute = [&](int k0) {
    const int kcn = min(T::BK, ke - k0);  // valid k in this chunk (rest is zero-filled)
#pragma unroll
    for (int kc = 0; kc < T::BK / 16; ++kc) {
      if (kc * 16 >= kcn) break;
      f32x4 a[T::TM], b[T::TN];
#pragma unroll
      for (int i = 0; i < T::TM; ++i)
        a[i] = load_frag<LA::KMAJOR, T::BM, T::BK>(As, (wm * T::TM + i) * 16 + r, kc * 16 + g * 4);
#pragma unroll
      for (int j = 0; j < T::TN; ++j)
        b[j] = load_frag<LB::KMAJOR, T::BN, T::BK>(Bs, (wn * T::TN + j) * 16 + r, kc * 16 + g * 4);
#pragma unroll
      for (int s = 0; s < 4; ++s)
#pragma unroll
        for (int i = 0; i < T::TM; ++i)
#pragma unroll
          for (int j = 0; j < T::TN; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[i][s], b[j][s], acc[i][j], 0, 0, 0);
    }
  };
  for (int k0 = kb; k0 < ke; k0 += T::BK) {
    sa.store(As);
    sb.store(Bs);
    __syncthreads();
    if (k0 + T::BK < ke) {  // prefetch the next chunk while this one is multiplied
      sa.load(la, m0, k0 + T::BK, ke, M);
      sb.load(lb, n0, k0 + T::BK, ke, N);
    }
    compute(k0);
    __syncthreads();
  }

  if constexpr (HasPre<EP>::value) {
#pragma unroll
    for (int i = 0; i < T::TM; ++i)
#pragma unroll
      for (int j = 0; j < T::TN; ++j) {
        const int n = n0 + (wn * T::TN + j) * 16 + r;
        if constexpr (IsQuadEp<EP>::value) {
          const int m = m0 + (wm * T::TM + i) * 16 + g * 4;
          if (m < M && n < N) ep.quad(pre[i][j][0], m, n, bz, acc[i][j]);
        } else {
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const int m = m0 + (wm * T::TM + i) * 16 + g * 4 + q;
            if (m < M && n < N) ep(pre[i][j][q], m, n, bz, acc[i][j][q]);
          }
        }
      }
    return;
  }
#pragma unroll
  for (int i = 0; i < T::TM; ++i)
#pragma unroll
    for (int j = 0; j < T::TN; ++j) {
      const int n = n0 + (wn * T::TN + j) * 16 + r;
      if constexpr (IsQuadEp<EP>::value) {
        const int m = m0 + (wm * T::TM + i) * 16 + g * 4;
        if (m < M && n < N) ep.quad(m, n, bz, acc[i][j]);
      } else {
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int m = m0 + (wm * T::TM + i) * 16 + g * 4 + q;
          if (m < M && n < N) ep(m, n, bz, acc[i][j][q]);
        }
      }
    }
}

// XCD-aware tile order. Workgroups are dealt to the 8 XCDs round-robin by launch index (each XCD
// has its own L2), so with the tile index = launch index the M-tiles of one K-split — which read
// the same B columns and, for an implicit im2col, nearly the same input pixels — land on 8 L2s
// and each fetches them from HBM (4.6x the algorithmic bytes on the LSTM conv2 weight gradient).
// The launch indices of one residue class (one XCD) take a contiguous run of tile indices
// instead; the n % 8 remainder keeps its own index. A bijection on [0, n): only placement moves.
__device__ __forceinline__ int xcd_tile(int id, int n) {
  const int per = n >> 3;
  return id < (per << 3) ? (id & 7) * per + (id >> 3) : id;
}

template <class T, class LA, class LB, class EP>
__global__ __launch_bounds__(256) void gemm_f32_kernel(LA la, LB lb, EP ep, int M, int N, int K,
                                                       int kchunk) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int gx = gridDim.x, gy = gridDim.y;
  const int t = xcd_tile(blockIdx.x + gx * (blockIdx.y + gy * blockIdx.z), gx * gy * gridDim.z);
  gemm_body<T>(la, lb, ep, M, N, K, kchunk, t % gx, (t / gx) % gy, t / (gx * gy), smem);
}

template <class T, class LA, class LB>
constexpr size_t gemm_lds_bytes() {
  return sizeof(float) * (LdsShape<LA::KMAJOR, T::BM, T::BK>::SIZE + LdsShape<LB::KMAJOR, T::BN, T::BK>::SIZE);
}

// Number of K splits the launch will actually use (chunks are whole BK multiples).
template <class T>
inline int gemm_splits(int K, int splits) {
  const int nchunks = cdiv(K, T::BK);
  if (splits < 1) splits = 1;
  if (splits > nchunks) splits = nchunks;
  const int kchunk = cdiv(nchunks, splits) * T::BK;
  return cdiv(K, kchunk);
}

template <class T, class LA, class LB, class EP>
inline int launch_gemm(const LA &la, const LB &lb, const EP &ep, int M, int N, int K, int splits,
                       hipStream_t s) {
  if (M <= 0 || N <= 0) return MT_OK;
  const int nchunks = cdiv(K, T::BK);
  if (splits < 1) splits = 1;
  if (splits > nchunks) splits = nchunks;
  const int kchunk = cdiv(nchunks, splits) * T::BK;
  splits = cdiv(K, kchunk);
  constexpr size_t lds = gemm_lds_bytes<T, LA, LB>();
  static_assert(lds <= 160 * 1024, "LDS budget");
  static bool attr_set = false;  // per instantiation: allow > 64 KB dynamic LDS once
  if (!attr_set && lds > 64 * 1024) {
    MT_HIP(hipFuncSetAttribute(reinterpret_cast<const void *>(&gemm_f32_kernel<T, LA, LB, EP>),
                               hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    attr_set = true;
  }
  dim3 grid(cdiv(M, T::BM), cdiv(N, T::BN), splits);
  hipLaunchKernelGGL((gemm_f32_kernel<T, LA, LB, EP>), grid, dim3(256), lds, s, la, lb, ep, M, N,
                     K, kchunk);
  MT_LAUNCHED();
  return MT_OK;
}

// ------------------------------------------------------------------------------------------
// Grouped launches: independent products (and other block-parallel jobs: slab sums, the head
// weight gradient) that become ready together run as ONE grid — each dependent kernel boundary
// costs microseconds at these sizes, more than most of the jobs themselves. A job is a value type
// with blocks() (host and device), lds() (dynamic bytes, host) and run(block, smem) (device).
// ------------------------------------------------------------------------------------------
template <class T, class LA, class LB, class EP>
struct GemmJob {
  LA la;
  LB lb;
  EP ep;
  int M, N, K, kchunk, gx, gy, gz;
  __host__ __device__ int blocks() const { return gx * gy * gz; }
  size_t lds() const { return gemm_lds_bytes<T, LA, LB>(); }
  __device__ __forceinline__ void run(int id, float *smem) const {
    id = xcd_tile(id, blocks());  // (a job's offset in its group only renames the residue classes)
    const int bx = id % gx, t = id / gx;
    gemm_body<T>(la, lb, ep, M, N, K, kchunk, bx, t % gy, t / gy, smem);
  }
};

// The job launch_gemm<T>(la, lb, ep, M, N, K, splits) would run (same grid, same K chunks).
template <class T, class LA, class LB, class EP>
inline GemmJob<T, LA, LB, EP> gemm_job(const LA &la, const LB &lb, const EP &ep, int M, int N, int K, int splits) {
  const int nchunks = cdiv(K, T::BK);
  if (splits < 1) splits = 1;
  if (splits > nchunks) splits = nchunks;
  const int kchunk = cdiv(nchunks, splits) * T::BK;
  splits = cdiv(K, kchunk);
  const bool empty = M <= 0 || N <= 0;
  return GemmJob<T, LA, LB, EP>{la, lb, ep, M, N, K, kchunk, empty ? 0 : cdiv(M, T::BM), cdiv(N, T::BN), splits};
}

struct NoJob {
  __host__ __device__ int blocks() const { return 0; }
  size_t lds() const { return 0; }
  __device__ __forceinline__ void run(int, float *) const {}
};

template <class J1, class... Rest>
__device__ __forceinline__ void run_group(int id, float *smem, const J1 &j1, const Rest &...rest) {
  if (id < j1.blocks()) {
    j1.run(id, smem);
    return;
  }
  if constexpr (sizeof...(Rest) > 0) run_group(id - j1.blocks(), smem, rest...);
}

// Up to four jobs as one (a grouped launch's extra slot), blocks in argument order. The pack's
// block count is rounded up to a multiple of 8 (the padding blocks return at once): it leads its
// grouped launch, and the jobs after it place their tiles by xcd_tile(id & 7 = the hardware XCD),
// which holds only when every job before them starts at a multiple of 8.
template <class A, class B, class C = NoJob, class D = NoJob>
struct JobPack {
  A a;
  B b;
  C c{};
  D d{};
  __host__ __device__ int used() const { return a.blocks() + b.blocks() + c.blocks() + d.blocks(); }
  __host__ __device__ int blocks() const { return (used() + 7) & ~7; }
  size_t lds() const {
    size_t l = 0;
    for (size_t x : {a.blocks() ? a.lds() : 0, b.blocks() ? b.lds() : 0, c.blocks() ? c.lds() : 0,
                     d.blocks() ? d.lds() : 0})
      l = std::max(l, x);
    return l;
  }
  __device__ __forceinline__ void run(int id, float *smem) const {
    if (id < used()) run_group(id, smem, a, b, c, d);
  }
};
template <class A, class B>
JobPack(A, B) -> JobPack<A, B>;
template <class A, class B, class C>
JobPack(A, B, C) -> JobPack<A, B, C>;
template <class A, class B, class C, class D>
JobPack(A, B, C, D) -> JobPack<A, B, C, D>;

template <class... J>
__global__ __launch_bounds__(256) void group_kernel(J... j) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  run_group(blockIdx.x, smem, j...);
}

// One grid for any number of jobs (blocks in argument order: put the critical path first).
template <class... J>
inline int launch_group(hipStream_t s, const J &...j) {
  const int nb = (0 + ... + j.blocks());
  if (nb == 0 || !launch_allowed()) return MT_OK;
  size_t lds = 0;
  ((lds = std::max(lds, j.blocks() ? j.lds() : (size_t)0)), ...);
  if (lds > 160 * 1024) {
    set_error("grouped launch needs %zu bytes of LDS", lds);
    return MT_ERR_ARG;
  }
  static bool attr_set = false;  // per instantiation: allow up to 160 KB of dynamic LDS once
  if (!attr_set && lds > 64 * 1024) {
    MT_HIP(hipFuncSetAttribute(reinterpret_cast<const void *>(&group_kernel<J...>),
                               hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
    attr_set = true;
  }
  hipLaunchKernelGGL((group_kernel<J...>), dim3(nb), dim3(256), lds, s, j...);
  MT_LAUNCHED();
  return MT_OK;
}

// ------------------------------------------------------------------------------------------
// Loaders: fetch(row0, rr, k0, kk, ke, nrows) returns the 4 values of item (row0+rr, k0+kk)
// — 4 consecutive k (KMAJOR) or 4 consecutive rows (!KMAJOR) — zero outside
// [0, nrows) x [.., ke); interior tiles use ctx(row) once per tile and fetch_ctx(ctx, k) per
// chunk (Stage).
// ------------------------------------------------------------------------------------------

// Dense row-major operand X[row][k] (k contiguous, leading dim ld), fp32. KMAJOR.
struct LdRowMajor {
  static constexpr bool KMAJOR = true;
  const float *X;
  int ld;
  __device__ __forceinline__ bool interior(int row0, int rows, int k0, int bk, int ke, int nrows) const {
    return row0 + rows <= nrows && k0 + bk <= ke;
  }
  struct Ctx {
    const float *p;
  };
  __device__ __forceinline__ Ctx ctx(int row) const { return {X + (size_t)row * ld}; }
  __device__ __forceinline__ f32x4 fetch_ctx(const Ctx &c, int k) const {
    return *reinterpret_cast<const f32x4 *>(c.p + k);
  }
  __device__ __forceinline__ f32x4 fetch(int row0, int rr, int k0, int kk, int ke, int nrows) const {
    const int row = row0 + rr, k = k0 + kk;
    f32x4 v = {0.f, 0.f, 0.f, 0.f};
    if (row < nrows) {
      const float *p = X + (size_t)row * ld + k;
      if (k + 3 < ke) {
        v = *reinterpret_cast<const f32x4 *>(p);
      } else {
#pragma unroll
        for (int e = 0; e < 4; ++e)
          if (k + e < ke) v[e] = p[e];
      }
    }
    return v;
  }
};

// Dense operand stored [k][row] (row contiguous, leading dim ld), fp32. !KMAJOR.
// ones_row < 0: every row < nrows comes from X. ones_row >= 0: rows < ones_row come from X,
// row ones_row reads 1.0 (for k < ke) and later rows read 0 — the bias row of a [X, 1]^T
// product, so one GEMM yields dW and db together.
struct LdColMajor {
  static constexpr bool KMAJOR = false;
  const float *X;
  int ld;
  int ones_row;
  __device__ __forceinline__ bool interior(int row0, int rows, int k0, int bk, int ke, int nrows) const {
    const int nx = ones_row >= 0 ? ones_row : nrows;
    return row0 + rows <= nx && k0 + bk <= ke && (ld & 3) == 0;
  }
  struct Ctx {
    const float *p;
  };
  __device__ __forceinline__ Ctx ctx(int row) const { return {X + row}; }
  __device__ __forceinline__ f32x4 fetch_ctx(const Ctx &c, int k) const {
    return *reinterpret_cast<const f32x4 *>(c.p + (size_t)k * ld);
  }
  struct KS {
    const float *p;
  };
  __device__ __forceinline__ KS ks(const Ctx &c, int k) const { return {c.p + (size_t)k * ld}; }
  __device__ __forceinline__ f32x4 fetch_ks(const Ctx &, const KS &s) const {
    return *reinterpret_cast<const f32x4 *>(s.p);
  }
  template <int BK>
  __device__ __forceinline__ void next(KS &s) const {
    s.p += (size_t)BK * ld;
  }
  // The guarded (edge) fetch. A row quad wholly inside [0, nx) — every quad of the conv weight
  // gradients' dY operand — is one load from a clamped k (k0 < ke is always in range) and a
  // zero by select: no branch around the load and no partial register-quad fill.
  __device__ __forceinline__ f32x4 fetch(int row0, int rr, int k0, int kk, int ke, int nrows) const {
    const int row = row0 + rr, k = k0 + kk;
    const int nx = ones_row >= 0 ? ones_row : nrows;
    const bool kok = k < ke;
    if (row + 3 < nx && (ld & 3) == 0) {
      const f32x4 v = *reinterpret_cast<const f32x4 *>(X + (size_t)(kok ? k : k0) * ld + row);
      return kok ? v : f32x4{0.f, 0.f, 0.f, 0.f};
    }
    f32x4 v = {0.f, 0.f, 0.f, 0.f};
    if (kok) {
      const float *p = X + (size_t)k * ld + row;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int rw = row + e;
        if (rw < nx) v[e] = p[e];
        else if (rw == ones_row) v[e] = 1.f;
      }
    }
    return v;
  }
};

// Compile-time conv geometry (NHWC input [B][H][W][CIN], HWIO weights, TF padding).
template <int CIN_, int COUT_, int KS_, int S_, int H_, int W_, bool SAME_>
struct ConvGeom {
  static constexpr int CIN = CIN_, COUT = COUT_, KH = KS_, KW = KS_, S = S_, H = H_, W = W_;
  static constexpr bool SAME = SAME_;
  static constexpr int OH = SAME ? (H + S - 1) / S : (H - KH) / S + 1;
  static constexpr int OW = SAME ? (W + S - 1) / S : (W - KW) / S + 1;
  // TF SAME: pad_total = max((O-1)*S + K - I, 0), pad_before = pad_total / 2.
  static constexpr int PADT_TOTAL = SAME ? (((OH - 1) * S + KH - H) > 0 ? ((OH - 1) * S + KH - H) : 0) : 0;
  static constexpr int PADL_TOTAL = SAME ? (((OW - 1) * S + KW - W) > 0 ? ((OW - 1) * S + KW - W) : 0) : 0;
  static constexpr int PT = PADT_TOTAL / 2, PL = PADL_TOTAL / 2;
  static constexpr int KK = KH * KW * CIN;  // GEMM-K of the forward product
  static_assert(CIN % 4 == 0 && COUT % 4 == 0, "channel quads");
};

template <bool U8>
struct InElem;
template <>
struct InElem<true> {
  typedef uint8_t T;
  __device__ static __forceinline__ f32x4 load4(const uint8_t *p) {
    const uint32_t u = *reinterpret_cast<const uint32_t *>(p);
    const float s = 1.0f / 255.0f;  // networks.py:155 scalar_mul(1/255, cast)
    return f32x4{(float)(u & 0xff) * s, (float)((u >> 8) & 0xff) * s,
                 (float)((u >> 16) & 0xff) * s, (float)(u >> 24) * s};
  }
};
template <>
struct InElem<false> {
  typedef float T;
  __device__ static __forceinline__ f32x4 load4(const float *p) {
    return *reinterpret_cast<const f32x4 *>(p);
  }
};

// Output pixel (b, oy, ox) of GEMM row m of a conv: NHWC order, or (POOL) pool order — m = 4p + q
// with p = (b, py, px) the 2x2/2 VALID pool output and q = (dy, dx) its window position in
// (row, col) order, so a lane's 4 accumulator rows are one pool window (the odd last row / column
// a VALID pool drops are not rows at all).
template <class G, bool POOL>
__device__ __forceinline__ void out_pixel(int m, int &b, int &oy, int &ox) {
  if constexpr (POOL) {
    constexpr int PH = G::OH / 2, PW = G::OW / 2;
    const int p = m >> 2, q = m & 3;
    b = p / (PH * PW);
    const int rem = p - b * (PH * PW);
    const int py = rem / PW;
    oy = 2 * py + (q >> 1);
    ox = 2 * (rem - py * PW) + (q & 1);
  } else {
    b = m / (G::OH * G::OW);
    const int rem = m - b * (G::OH * G::OW);
    oy = rem / G::OW;
    ox = rem - oy * G::OW;
  }
}

// Implicit im2col of the forward conv: A(m = (b, oy, ox), k = (ky, kx, ci)). KMAJOR.
// POOL: rows in pool order (out_pixel), for a pooling epilogue (EpBiasActPool).
template <class G, bool U8, bool POOL = false>
struct LdIm2col {
  static constexpr bool KMAJOR = true;
  const typename InElem<U8>::T *X;
  // k >= KK (a BK that does not divide KK) is zeroed inside fetch_ctx, so only the rows decide.
  __device__ __forceinline__ bool interior(int row0, int rows, int k0, int bk, int ke, int nrows) const {
    return row0 + rows <= nrows && (k0 + bk <= ke || ke == G::KK);
  }
  // Row context: the image of output pixel m and its window's top-left input pixel.
  struct Ctx {
    const typename InElem<U8>::T *img;
    int iy0, ix0;
  };
  __device__ __forceinline__ Ctx ctx(int m) const {
    int b, oy, ox;
    out_pixel<G, POOL>(m, b, oy, ox);
    return {X + (size_t)b * G::H * G::W * G::CIN, oy * G::S - G::PT, ox * G::S - G::PL};
  }
  // Padding (SAME) and the k tail handled branch-free: clamped address, zero by select.
  __device__ __forceinline__ f32x4 fetch_ctx(const Ctx &c, int k) const {
    const bool kok = k < G::KK;
    k = kok ? k : 0;
    const int ky = k / (G::KW * G::CIN);
    const int r2 = k - ky * (G::KW * G::CIN);
    const int kx = r2 / G::CIN, ci = r2 - kx * G::CIN;
    const int iy = c.iy0 + ky, ix = c.ix0 + kx;
    if constexpr (G::SAME) {
      const bool ok = kok && iy >= 0 && iy < G::H && ix >= 0 && ix < G::W;
      const int iyc = min(max(iy, 0), G::H - 1), ixc = min(max(ix, 0), G::W - 1);
      const f32x4 v = InElem<U8>::load4(c.img + ((size_t)iyc * G::W + ixc) * G::CIN + ci);
      return ok ? v : f32x4{0.f, 0.f, 0.f, 0.f};
    } else {
      const f32x4 v = InElem<U8>::load4(c.img + ((size_t)iy * G::W + ix) * G::CIN + ci);
      return kok ? v : f32x4{0.f, 0.f, 0.f, 0.f};
    }
  }
  __device__ __forceinline__ f32x4 fetch(int row0, int rr, int k0, int kk, int ke, int nrows) const {
    const int m = row0 + rr, k = k0 + kk;
    f32x4 v = {0.f, 0.f, 0.f, 0.f};
    if (m < nrows && k < ke) {
      int b, oy, ox;
      out_pixel<G, POOL>(m, b, oy, ox);
      const int ky = k / (G::KW * G::CIN);
      const int r2 = k - ky * (G::KW * G::CIN);
      const int kx = r2 / G::CIN, ci = r2 - kx * G::CIN;
      const int iy = oy * G::S + ky - G::PT, ix = ox * G::S + kx - G::PL;
      if (iy >= 0 && iy < G::H && ix >= 0 && ix < G::W)
        v = InElem<U8>::load4(X + (((size_t)b * G::H + iy) * G::W + ix) * G::CIN + ci);
    }
    return v;
  }
};

// Transposed im2col for the weight gradient: A(row = k (+ bias row KK), gk = m). !KMAJOR.
template <class G, bool U8>
struct LdIm2colT {
  static constexpr bool KMAJOR = false;
  const typename InElem<U8>::T *X;
  __device__ __forceinline__ bool interior(int row0, int rows, int k0, int bk, int ke, int nrows) const {
    return row0 + rows <= G::KK && k0 + bk <= ke;  // the bias-row tile takes the guarded path
  }
  // Row context: the tap (ky - PT, kx - PL) and channel of weight row quad kr, and its element
  // offset from the window origin.
  struct Ctx {
    int dy, dx, ci, toff;
  };
  __device__ __forceinline__ Ctx ctx(int kr) const {
    const int ky = kr / (G::KW * G::CIN);
    const int r2 = kr - ky * (G::KW * G::CIN);
    const int kx = r2 / G::CIN;
    const int dy = ky - G::PT, dx = kx - G::PL, ci = r2 - kx * G::CIN;
    return {dy, dx, ci, (dy * G::W + dx) * G::CIN + ci};
  }
  // k state of GEMM-K pixel m = (b, oy, ox): the window origin (sy, sx) = (oy*S, ox*S) and its
  // element offset pix = ((b*H + sy)*W + sx)*CIN (the host keeps B*H*W*CIN < 2^31), stepped by
  // BK pixels with carries instead of re-divided per chunk.
  struct KS {
    int pix, sy, sx;
  };
  __device__ __forceinline__ KS ks(const Ctx &, int m) const {
    const int b = m / (G::OH * G::OW);
    const int rem = m - b * (G::OH * G::OW);
    const int oy = rem / G::OW, ox = rem - oy * G::OW;
    return {((b * G::H + oy * G::S) * G::W + ox * G::S) * G::CIN, oy * G::S, ox * G::S};
  }
  template <int BK>
  __device__ __forceinline__ void next(KS &s) const {
    constexpr int DY = BK / G::OW, DX = BK % G::OW, S = G::S;
    constexpr int CW = G::W * G::CIN;
    s.pix += (DY * S * G::W + DX * S) * G::CIN;
    s.sx += DX * S;
    s.sy += DY * S;
    const bool cx = s.sx >= G::OW * S;  // row carry: (oy + 1, ox - OW)
    s.sx -= cx ? G::OW * S : 0;
    s.sy += cx ? S : 0;
    s.pix += cx ? (S * CW - G::OW * S * G::CIN) : 0;
#pragma unroll
    for (int w = 0; w < 1 + BK / (G::OH * G::OW); ++w) {  // image carries: (b + 1, oy - OH)
      const bool cy = s.sy >= G::OH * S;
      s.sy -= cy ? G::OH * S : 0;
      s.pix += cy ? (G::H - G::OH * S) * CW : 0;
    }
  }
  __device__ __forceinline__ f32x4 fetch_ks(const Ctx &c, const KS &s) const {
    if constexpr (G::SAME) {
      const int iy = s.sy + c.dy, ix = s.sx + c.dx;
      const bool ok = (unsigned)iy < (unsigned)G::H && (unsigned)ix < (unsigned)G::W;
      const f32x4 v = InElem<U8>::load4(X + (ok ? s.pix + c.toff : s.pix + c.ci));
      return ok ? v : f32x4{0.f, 0.f, 0.f, 0.f};
    } else {
      return InElem<U8>::load4(X + (s.pix + c.toff));
    }
  }
  __device__ __forceinline__ f32x4 fetch_ctx(const Ctx &c, int m) const {
    const int b = m / (G::OH * G::OW);
    const int rem = m - b * (G::OH * G::OW);
    const int oy = rem / G::OW, ox = rem - oy * G::OW;
    const int iy = oy * G::S + c.dy, ix = ox * G::S + c.dx;
    if constexpr (G::SAME) {
      const bool ok = iy >= 0 && iy < G::H && ix >= 0 && ix < G::W;
      const int iyc = min(max(iy, 0), G::H - 1), ixc = min(max(ix, 0), G::W - 1);
      const f32x4 v = InElem<U8>::load4(X + (((size_t)b * G::H + iyc) * G::W + ixc) * G::CIN + c.ci);
      return ok ? v : f32x4{0.f, 0.f, 0.f, 0.f};
    } else {
      return InElem<U8>::load4(X + (((size_t)b * G::H + iy) * G::W + ix) * G::CIN + c.ci);
    }
  }
  __device__ __forceinline__ f32x4 fetch(int row0, int rr, int k0, int kk, int ke, int nrows) const {
    const int m = k0 + kk, kr = row0 + rr;
    f32x4 v = {0.f, 0.f, 0.f, 0.f};
    if (m < ke) {
      if (kr < G::KK) {
        const int b = m / (G::OH * G::OW);
        const int rem = m - b * (G::OH * G::OW);
        const int oy = rem / G::OW, ox = rem - oy * G::OW;
        const int ky = kr / (G::KW * G::CIN);
        const int r2 = kr - ky * (G::KW * G::CIN);
        const int kx = r2 / G::CIN, ci = r2 - kx * G::CIN;
        const int iy = oy * G::S + ky - G::PT, ix = ox * G::S + kx - G::PL;
        if (iy >= 0 && iy < G::H && ix >= 0 && ix < G::W)
          v = InElem<U8>::load4(X + (((size_t)b * G::H + iy) * G::W + ix) * G::CIN + ci);
      } else if (kr == G::KK) {
        v[0] = 1.f;  // bias row
      }
    }
    return v;
  }
};

// Backward-data of a conv, A side: rows = input pixels (b, iy, ix), gk = (ky, kx, co);
// A = dY[b][oy][ox][co] with oy = (iy + PT - ky)/S when that divides and lands in range. KMAJOR.
// Stride 1 (every tap lands): a k state per item (LdConvBwdAKs) — the (oy, ox) the item's tap
// lands on and its channel, stepped by BK per chunk — and one buffer load whose offset is pushed
// past the descriptor's range when the tap falls outside dY (reads zero): a few VALU per quad
// instead of the (tap, channel) divisions, clamps and selects of fetch_ctx. The caller keeps
// dY under 2^31 bytes (trunk_backward). Only for CIN >= 64: the thin CIN-32 tile (Tile<64, 32, 4, 1>)
// goes from 128 to 136 VGPRs with it, a wave per SIMD less (LSTM conv3 group 186.9 vs 180.3 us
// without, profiles/r06ks).
template <class G>
struct LdConvBwdACtx {
  const float *dY;  // [B][OH][OW][COUT]
  struct Ctx {
    const float *img;
    int ty0, tx0;
  };
};
template <class G, bool KSOK = G::S == 1 && G::CIN >= 64>
struct LdConvBwdAKs : LdConvBwdACtx<G> {};
template <class G>
struct LdConvBwdAKs<G, true> : LdConvBwdACtx<G> {
  using Ctx = typename LdConvBwdACtx<G>::Ctx;
  using LdConvBwdACtx<G>::dY;
  struct KS {
    int ty, tx, kx, co;  // (ty, tx): the output pixel tap (ky, kx) of the item's row lands on
  };
  __device__ __forceinline__ KS ks(const Ctx &c, int k) const {
    const int ky = k / (G::KW * G::COUT);
    const int r2 = k - ky * (G::KW * G::COUT);
    const int kx = r2 / G::COUT, co = r2 - kx * G::COUT;
    return {c.ty0 - ky, c.tx0 - kx, kx, co};
  }
  template <int BK>
  __device__ __forceinline__ void next(KS &s) const {
    constexpr int DT = BK / G::COUT, DC = BK % G::COUT;
    if constexpr (DC != 0) {
      s.co += DC;
      const bool c = s.co >= G::COUT;
      s.co -= c ? G::COUT : 0;
      s.kx += c ? 1 : 0;
      s.tx -= c ? 1 : 0;
    }
    s.kx += DT;
    s.tx -= DT;
#pragma unroll
    for (int w = 0; w < 1 + DT / G::KW; ++w) {  // tap-row carries: (ky + 1, kx - KW)
      const bool c = s.kx >= G::KW;
      s.kx -= c ? G::KW : 0;
      s.tx += c ? G::KW : 0;
      s.ty -= c ? 1 : 0;
    }
  }
  __device__ __forceinline__ f32x4 fetch_ks(const Ctx &c, const KS &s) const {
    const bool ok = (unsigned)s.ty < (unsigned)G::OH && (unsigned)s.tx < (unsigned)G::OW;
    const uint32_t off = (uint32_t)((c.img - dY) + (s.ty * G::OW + s.tx) * G::COUT + s.co) * 4u;
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void *)dY, (short)0, 0x7ffffff0, 0x00020000);
    return __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rs, ok ? off : 0x80000000u, 0, 0));
  }
};
template <class G>
struct LdConvBwdA : LdConvBwdAKs<G> {
  static constexpr bool KMAJOR = true;
  using Ctx = typename LdConvBwdACtx<G>::Ctx;
  using LdConvBwdACtx<G>::dY;
  __device__ __forceinline__ bool interior(int row0, int rows, int k0, int bk, int ke, int nrows) const {
    return row0 + rows <= nrows && k0 + bk <= ke;
  }
  // Row context: the image of input pixel m and (iy + PT, ix + PL).
  __device__ __forceinline__ Ctx ctx(int m) const {
    const int b = m / (G::H * G::W);
    const int rem = m - b * (G::H * G::W);
    const int iy = rem / G::W, ix = rem - iy * G::W;
    return {dY + (size_t)b * G::OH * G::OW * G::COUT, iy + G::PT, ix + G::PL};
  }
  // The stride-S holes of the transposed conv are data-dependent: clamped address + select.
  __device__ __forceinline__ f32x4 fetch_ctx(const Ctx &c, int k) const {
    const int ky = k / (G::KW * G::COUT);
    const int r2 = k - ky * (G::KW * G::COUT);
    const int kx = r2 / G::COUT, co = r2 - kx * G::COUT;
    const int ty = c.ty0 - ky, tx = c.tx0 - kx;
    const int oy = ty / G::S, ox = tx / G::S;  // only used when ty, tx >= 0
    const bool ok = ty >= 0 && tx >= 0 && (ty - oy * G::S) == 0 && (tx - ox * G::S) == 0 &&
                    oy < G::OH && ox < G::OW;
    const int oyc = min(max(oy, 0), G::OH - 1), oxc = min(max(ox, 0), G::OW - 1);
    const f32x4 v = *reinterpret_cast<const f32x4 *>(c.img + ((size_t)oyc * G::OW + oxc) * G::COUT + co);
    return ok ? v : f32x4{0.f, 0.f, 0.f, 0.f};
  }
  __device__ __forceinline__ f32x4 fetch(int row0, int rr, int k0, int kk, int ke, int nrows) const {
    const int m = row0 + rr, k = k0 + kk;
    f32x4 v = {0.f, 0.f, 0.f, 0.f};
    if (m < nrows && k < ke) {
      const int b = m / (G::H * G::W);
      const int rem = m - b * (G::H * G::W);
      const int iy = rem / G::W, ix = rem - iy * G::W;
      const int ky = k / (G::KW * G::COUT);
      const int r2 = k - ky * (G::KW * G::COUT);
      const int kx = r2 / G::COUT, co = r2 - kx * G::COUT;
      const int ty = iy + G::PT - ky, tx = ix + G::PL - kx;
      if (ty >= 0 && tx >= 0 && (ty % G::S) == 0 && (tx % G::S) == 0) {
        const int oy = ty / G::S, ox = tx / G::S;
        if (oy < G::OH && ox < G::OW)
          v = *reinterpret_cast<const f32x4 *>(dY + (((size_t)b * G::OH + oy) * G::OW + ox) * G::COUT + co);
      }
    }
    return v;
  }
};

// Backward-data of a conv, B side: rows = ci, gk = (ky, kx, co): W[ky][kx][ci][co]. KMAJOR.
template <class G>
struct LdConvBwdB {
  static constexpr bool KMAJOR = true;
  const float *Wt;  // HWIO
  __device__ __forceinline__ bool interior(int row0, int rows, int k0, int bk, int ke, int nrows) const {
    return row0 + rows <= nrows && k0 + bk <= ke;
  }
  struct Ctx {
    const float *p;
  };
  __device__ __forceinline__ Ctx ctx(int ci) const { return {Wt + (size_t)ci * G::COUT}; }
  // k state: the item's tap and channel, stepped by BK per chunk
  struct KS {
    int tap, co;
  };
  __device__ __forceinline__ KS ks(const Ctx &, int k) const {
    const int tap = k / G::COUT;
    return {tap, k - tap * G::COUT};
  }
  template <int BK>
  __device__ __forceinline__ void next(KS &s) const {
    constexpr int DT = BK / G::COUT, DC = BK % G::COUT;
    if constexpr (DC != 0) {
      s.co += DC;
      const bool c = s.co >= G::COUT;
      s.co -= c ? G::COUT : 0;
      s.tap += c ? 1 : 0;
    }
    s.tap += DT;
  }
  __device__ __forceinline__ f32x4 fetch_ks(const Ctx &c, const KS &s) const {
    return *reinterpret_cast<const f32x4 *>(c.p + (size_t)(s.tap * G::CIN * G::COUT + s.co));
  }
  __device__ __forceinline__ f32x4 fetch_ctx(const Ctx &c, int k) const {
    const int ky = k / (G::KW * G::COUT);
    const int r2 = k - ky * (G::KW * G::COUT);
    const int kx = r2 / G::COUT, co = r2 - kx * G::COUT;
    return *reinterpret_cast<const f32x4 *>(c.p + (size_t)(ky * G::KW + kx) * G::CIN * G::COUT + co);
  }
  __device__ __forceinline__ f32x4 fetch(int row0, int rr, int k0, int kk, int ke, int nrows) const {
    const int ci = row0 + rr, k = k0 + kk;
    f32x4 v = {0.f, 0.f, 0.f, 0.f};
    if (ci < nrows && k < ke) {
      const int ky = k / (G::KW * G::COUT);
      const int r2 = k - ky * (G::KW * G::COUT);
      const int kx = r2 / G::COUT, co = r2 - kx * G::COUT;
      v = *reinterpret_cast<const f32x4 *>(Wt + (((size_t)(ky * G::KW + kx) * G::CIN + ci) * G::COUT + co));
    }
    return v;
  }
};

// Stride-phase decomposition of the backward-data product of a VALID stride-S conv with K % S == 0
// and H, W % S == 0: input pixel (iy, ix) only receives taps ky = py + S*a, kx = px + S*b of its
// phase (py, px) = (iy % S, ix % S), so the dense gather above multiplies (S*S - 1)/(S*S) zeros.
// Rows are regrouped by phase — row m' = phase * MP + l, l = (b, qy, qx) with iy = S*qy + py —
// and K shrinks to (KH/S)(KW/S)*COUT. MP (rows per phase, padded to the tile height) keeps every
// workgroup inside one phase, which the B loader takes from the row tile (for_mtile).
template <class G>
struct PhaseGeom {
  static constexpr bool OK = G::S > 1 && !G::SAME && G::KH % G::S == 0 && G::KW % G::S == 0 &&
                             G::H % G::S == 0 && G::W % G::S == 0;
  static constexpr int HQ = G::H / G::S, WQ = G::W / G::S, KA = G::KH / G::S, KB = G::KW / G::S;
  static constexpr int KP = KA * KB * G::COUT;  // GEMM-K per phase
};

template <class G>
struct LdConvBwdAPhase {
  static constexpr bool KMAJOR = true;
  using P = PhaseGeom<G>;
  const float *dY;  // [B][OH][OW][COUT]
  int mp, B;        // rows per phase (padded), batch
  __device__ __forceinline__ bool interior(int row0, int rows, int k0, int bk, int ke, int nrows) const {
    return row0 + rows <= nrows && k0 + bk <= ke;
  }
  __device__ __forceinline__ f32x4 at(int m, int k) const {
    const int ph = m / mp, l = m - ph * mp;
    const int py = ph / G::S, px = ph - py * G::S;
    const int b = l / (P::HQ * P::WQ);
    const int rem = l - b * (P::HQ * P::WQ);
    const int qy = rem / P::WQ, qx = rem - qy * P::WQ;
    const int a = k / (P::KB * G::COUT);
    const int r2 = k - a * (P::KB * G::COUT);
    const int bb = r2 / G::COUT, co = r2 - bb * G::COUT;
    const int oy = qy - a, ox = qx - bb;  // (iy - ky) / S with ky = py + S*a
    const bool ok = b < B && oy >= 0 && ox >= 0 && oy < G::OH && ox < G::OW;
    (void)py;
    (void)px;
    const int oyc = min(max(oy, 0), G::OH - 1), oxc = min(max(ox, 0), G::OW - 1), bc = min(b, B - 1);
    const f32x4 v = *reinterpret_cast<const f32x4 *>(dY + (((size_t)bc * G::OH + oyc) * G::OW + oxc) * G::COUT + co);
    return ok ? v : f32x4{0.f, 0.f, 0.f, 0.f};
  }
  // Row context: the clamped image of phase row m, its (qy, qx), and whether it is a real row.
  struct Ctx {
    const float *img;
    int qy, qx;
    bool ok;
  };
  __device__ __forceinline__ Ctx ctx(int m) const {
    const int ph = m / mp, l = m - ph * mp;
    const int b = l / (P::HQ * P::WQ);
    const int rem = l - b * (P::HQ * P::WQ);
    const int qy = rem / P::WQ;
    return {dY + (size_t)min(b, B - 1) * G::OH * G::OW * G::COUT, qy, rem - qy * P::WQ, b < B};
  }
  __device__ __forceinline__ f32x4 fetch_ctx(const Ctx &c, int k) const {
    const int a = k / (P::KB * G::COUT);
    const int r2 = k - a * (P::KB * G::COUT);
    const int bb = r2 / G::COUT, co = r2 - bb * G::COUT;
    const int oy = c.qy - a, ox = c.qx - bb;
    const bool ok = c.ok && oy >= 0 && ox >= 0 && oy < G::OH && ox < G::OW;
    const int oyc = min(max(oy, 0), G::OH - 1), oxc = min(max(ox, 0), G::OW - 1);
    const f32x4 v = *reinterpret_cast<const f32x4 *>(c.img + ((size_t)oyc * G::OW + oxc) * G::COUT + co);
    return ok ? v : f32x4{0.f, 0.f, 0.f, 0.f};
  }
  __device__ __forceinline__ f32x4 fetch(int row0, int rr, int k0, int kk, int ke, int nrows) const {
    const int m = row0 + rr, k = k0 + kk;
    return (m < nrows && k < ke) ? at(m, k) : f32x4{0.f, 0.f, 0.f, 0.f};
  }
};

template <class G>
struct LdConvBwdBPhase {
  static constexpr bool KMAJOR = true;
  using P = PhaseGeom<G>;
  const float *Wt;  // HWIO
  int blocks_per_phase;
  int ph = 0;  // set per output tile by for_mtile (gemm_body)
  __device__ __forceinline__ LdConvBwdBPhase for_mtile(int bx) const {
    LdConvBwdBPhase l = *this;
    l.ph = bx / blocks_per_phase;
    return l;
  }
  __device__ __forceinline__ bool interior(int row0, int rows, int k0, int bk, int ke, int nrows) const {
    return row0 + rows <= nrows && k0 + bk <= ke;
  }
  __device__ __forceinline__ f32x4 at(int ci, int k) const {
    const int py = ph / G::S, px = ph - py * G::S;
    const int a = k / (P::KB * G::COUT);
    const int r2 = k - a * (P::KB * G::COUT);
    const int bb = r2 / G::COUT, co = r2 - bb * G::COUT;
    const int ky = py + G::S * a, kx = px + G::S * bb;
    return *reinterpret_cast<const f32x4 *>(Wt + (((size_t)(ky * G::KW + kx) * G::CIN + ci) * G::COUT + co));
  }
  struct Ctx {
    int ci;
  };
  __device__ __forceinline__ Ctx ctx(int ci) const { return {ci}; }
  __device__ __forceinline__ f32x4 fetch_ctx(const Ctx &c, int k) const { return at(c.ci, k); }
  __device__ __forceinline__ f32x4 fetch(int row0, int rr, int k0, int kk, int ke, int nrows) const {
    const int ci = row0 + rr, k = k0 + kk;
    return (ci < nrows && k < ke) ? at(ci, k) : f32x4{0.f, 0.f, 0.f, 0.f};
  }
};

// ------------------------------------------------------------------------------------------
// Epilogues: ep(m, n, z, value)
// ------------------------------------------------------------------------------------------

__device__ __forceinline__ float act_fwd(float x, int act, float alpha) {
  // networks.py:27-31 relu / max(x, alpha*x)
  return act == MT_ACT_RELU ? fmaxf(x, 0.f) : fmaxf(x, alpha * x);
}
// Gradient factor from the post-activation output y (TF ReluGrad: y > 0; Maximum grad for
// max(x, a*x): x >= a*x, i.e. y >= 0 for 0 < a < 1).
__device__ __forceinline__ float act_bwd(float y, int act, float alpha) {
  return act == MT_ACT_RELU ? (y > 0.f ? 1.f : 0.f) : (y >= 0.f ? 1.f : alpha);
}

struct EpBiasAct {
  float *Y;
  const float *bias;
  int ld;
  int act;
  float alpha;
  __device__ __forceinline__ void operator()(int m, int n, int, float v) const {
    Y[(size_t)m * ld + n] = act_fwd(v + bias[n], act, alpha);
  }
  struct Pre {
    float b;
  };
  __device__ __forceinline__ Pre pre(int, int n) const { return {bias[n]}; }
  __device__ __forceinline__ void operator()(const Pre &p, int m, int n, int, float v) const {
    Y[(size_t)m * ld + n] = act_fwd(v + p.b, act, alpha);
  }
};

// Conv bias + activation + 2x2/2 VALID max pool (networks.py:108-110) over pool-ordered rows
// (LdIm2col<G, U8, true>): the lane's 4 rows are one window; writes the pooled value and the
// window position of its first maximum in (row, col) order — the position TF's MaxPoolGrad routes
// the gradient to — so neither the full-resolution activation nor a pool kernel exists.
template <class G>
struct EpBiasActPool {
  static constexpr bool QUAD = true;
  float *Y;         // [B][OH/2][OW/2][COUT]
  uint8_t *arg;     // [B][OH/2][OW/2][COUT] first-max position 0..3
  const float *bias;
  int act;
  float alpha;
  struct Pre {
    float b;
  };
  __device__ __forceinline__ Pre pre(int, int n) const { return {bias[n]}; }
  __device__ __forceinline__ void quad(int m, int n, int z, f32x4 v) const { quad(pre(m, n), m, n, z, v); }
  __device__ __forceinline__ void quad(const Pre &p, int m, int n, int, f32x4 v) const {
    const float bn = p.b;
    float mx = act_fwd(v[0] + bn, act, alpha);
    int a = 0;
#pragma unroll
    for (int q = 1; q < 4; ++q) {
      const float y = act_fwd(v[q] + bn, act, alpha);
      if (y > mx) {
        mx = y;
        a = q;
      }
    }
    const size_t i = (size_t)(m >> 2) * G::COUT + n;
    Y[i] = mx;
    arg[i] = (uint8_t)a;
  }
};

struct EpSlab {
  float *P;
  int M, N;
  __device__ __forceinline__ void operator()(int m, int n, int z, float v) const {
    P[((size_t)z * M + m) * N + n] = v;
  }
};

struct EpStore {
  float *P;
  int ld;
  __device__ __forceinline__ void operator()(int m, int n, int, float v) const {
    P[(size_t)m * ld + n] = v;
  }
};

// Phase-grouped rows of LdConvBwdAPhase back to pixels, then dX = v * act'(Yact).
template <class G>
struct EpMaskedPhase {
  using P = PhaseGeom<G>;
  float *dX;
  const float *Yact;
  int mp, B, act;
  float alpha;
  // element of phase row m, or -1 for the phase padding rows
  __device__ __forceinline__ long index(int m, int n) const {
    const int ph = m / mp, l = m - ph * mp;
    const int py = ph / G::S, px = ph - py * G::S;
    const int b = l / (P::HQ * P::WQ);
    if (b >= B) return -1;
    const int rem = l - b * (P::HQ * P::WQ);
    const int qy = rem / P::WQ, qx = rem - qy * P::WQ;
    return (((long)b * G::H + G::S * qy + py) * G::W + G::S * qx + px) * G::CIN + n;
  }
  __device__ __forceinline__ void operator()(int m, int n, int, float v) const {
    const long i = index(m, n);
    if (i >= 0) dX[i] = v * act_bwd(Yact[i], act, alpha);
  }
  struct Pre {
    long i;
    float y;
  };
  __device__ __forceinline__ Pre pre(int m, int n) const {
    const long i = index(m, n);
    return {i, Yact[i < 0 ? 0 : i]};
  }
  __device__ __forceinline__ void operator()(const Pre &p, int, int, int, float v) const {
    if (p.i >= 0) dX[p.i] = v * act_bwd(p.y, act, alpha);
  }
};

// MaxPoolGrad fused into the backward-data product of the layer after a pool: row m is pooled
// pixel (b, py, px) of conv GJ's pooled output P, v its gradient; v * act'(P) goes to the window
// position arg[m][n] of GJ's full-resolution output gradient dact, zeros to the other three and
// to the odd last row / column the VALID pool dropped (TF MaxPoolGrad; act'(P) == act' at the max).
template <class GJ>
struct EpMaskedUnpool {
  float *dact;          // [B][OH][OW][COUT] of conv GJ
  const float *P;       // [B][OH/2][OW/2][COUT]
  const uint8_t *arg;
  int act;
  float alpha;
  struct Pre {
    float p;
    int a;
  };
  __device__ __forceinline__ Pre pre(int m, int n) const {
    const size_t i = (size_t)m * GJ::COUT + n;
    return {P[i], arg[i]};
  }
  __device__ __forceinline__ void operator()(int m, int n, int z, float v) const { (*this)(pre(m, n), m, n, z, v); }
  __device__ __forceinline__ void operator()(const Pre &pr, int m, int n, int, float v) const {
    constexpr int PH = GJ::OH / 2, PW = GJ::OW / 2, C = GJ::COUT;
    const float g = v * act_bwd(pr.p, act, alpha);
    const int a = pr.a;
    const int b = m / (PH * PW);
    const int rem = m - b * (PH * PW);
    const int py = rem / PW, px = rem - py * PW;
    float *d = dact + (((size_t)b * GJ::OH + 2 * py) * GJ::OW + 2 * px) * C + n;
    constexpr size_t RW = (size_t)GJ::OW * C;
    d[0] = a == 0 ? g : 0.f;
    d[C] = a == 1 ? g : 0.f;
    d[RW] = a == 2 ? g : 0.f;
    d[RW + C] = a == 3 ? g : 0.f;
    if constexpr (GJ::OW & 1) {
      if (px == PW - 1) {
        d[2 * C] = 0.f;
        d[RW + 2 * C] = 0.f;
      }
    }
    if constexpr (GJ::OH & 1) {
      if (py == PH - 1) {
        d[2 * RW] = 0.f;
        d[2 * RW + C] = 0.f;
        if constexpr (GJ::OW & 1) {
          if (px == PW - 1) d[2 * RW + 2 * C] = 0.f;
        }
      }
    }
  }
};

// dX = v * act'(Yact) (Yact = post-activation output of the layer that produced X).
struct EpMasked {
  float *dX;
  const float *Yact;
  int ld;
  int act;
  float alpha;
  __device__ __forceinline__ void operator()(int m, int n, int, float v) const {
    const size_t i = (size_t)m * ld + n;
    dX[i] = v * act_bwd(Yact[i], act, alpha);
  }
  struct Pre {
    float y;
  };
  __device__ __forceinline__ Pre pre(int m, int n) const { return {Yact[(size_t)m * ld + n]}; }
  __device__ __forceinline__ void operator()(const Pre &p, int m, int n, int, float v) const {
    dX[(size_t)m * ld + n] = v * act_bwd(p.y, act, alpha);
  }
};

}  // namespace mt
