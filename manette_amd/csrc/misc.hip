// Streaming kernels of the PAAC hot path on gfx950 (all HBM-bound, no MFMA):
//   A2  frame preprocess + 4-frame stack      (atari_emulator.py:79-124, environment.py:42-80)
//   A3  device multinomial sampling (perf mode) (exploration_policy.py:108-116)
//   A9  n-step return / advantage scan         (paac.py:219-231)
//   A11 global-norm clip + TF1 ApplyRMSProp    (actor_learner.py:47-74)
// plus error reporting and hipGraph capture helpers of the C ABI.
#include <algorithm>
#include <atomic>
#include <cmath>

#include "common.h"

namespace mt {

static thread_local char g_err[512] = "";

void set_error(const char *fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
}

// ---------------------------------------------------------------------------------------------
// A9: y_t = R_t, R_t = r_t + gamma * R_{t+1} * mask_t, R_T = V(s_T); adv_t = R_t - V_t.
// dtype trail of paac.py:226-231 under numpy's promotion rules: estimated_return starts as the
// float32 bootstrap; `self.gamma * estimated_return` is a python float times a float32 array,
// i.e. a float32 product; every later operation meets float64 arrays (rewards, masks, values),
// so the rest runs in float64; the feed casts y/adv to float32 (placeholders are float32).
// ---------------------------------------------------------------------------------------------
__global__ void returns_kernel(const float *__restrict__ r, const float *__restrict__ mask,
                               const float *__restrict__ V, const float *__restrict__ VT,
                               double gamma, int T, int E, float *__restrict__ y,
                               float *__restrict__ adv) {
#pragma clang fp contract(off)
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= E) return;
  // t = T-1: float32 product gamma*R_T, then float64 with the mask and reward.
  const float g32 = __fmul_rn((float)gamma, VT[e]);
  double R = (double)r[(size_t)(T - 1) * E + e] + (double)g32 * (double)mask[(size_t)(T - 1) * E + e];
  y[(size_t)(T - 1) * E + e] = (float)R;
  adv[(size_t)(T - 1) * E + e] = (float)(R - (double)V[(size_t)(T - 1) * E + e]);
  const double gd = gamma;  // python float (float64)
  // steps T-2 .. 0 in batches of 8 whose loads are all in flight before the scan (the rewards and
  // masks may be pinned host memory: one PCIe round trip per step otherwise)
  for (int t0 = T - 2; t0 >= 0; t0 -= 8) {
    float rv[8], mv[8], vv[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const size_t i = (size_t)max(t0 - u, 0) * E + e;
      rv[u] = r[i];
      mv[u] = mask[i];
      vv[u] = V[i];
    }
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int t = t0 - u;
      if (t < 0) break;
      const size_t i = (size_t)t * E + e;
      R = (double)rv[u] + (gd * R) * (double)mv[u];
      y[i] = (float)R;
      adv[i] = (float)(R - (double)vv[u]);
    }
  }
}

// ---------------------------------------------------------------------------------------------
// A11, pass 1: partial sums of (s*g)^2, MT_NORM_PARTIALS blocks, deterministic.
// ---------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void sumsq_kernel(const float *__restrict__ g, size_t n, float s,
                                                    float *__restrict__ partials) {
  __shared__ double red[4];
  double acc = 0.0;
  const size_t n4 = n / 4;
  const size_t stride = (size_t)gridDim.x * blockDim.x;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += stride) {
    const f32x4 v = reinterpret_cast<const f32x4 *>(g)[i] * s;
    acc += (double)(v[0] * v[0]) + (double)(v[1] * v[1]) + (double)(v[2] * v[2]) + (double)(v[3] * v[3]);
  }
  for (size_t i = n4 * 4 + (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    const float v = g[i] * s;
    acc += (double)(v * v);
  }
  acc = wave_sum_d(acc);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = acc;
  __syncthreads();
  if (threadIdx.x == 0) partials[blockIdx.x] = (float)(red[0] + red[1] + red[2] + red[3]);
}

// A11, pass 2: every block reduces the partials (fixed order), then clip + ApplyRMSProp.
// TF1 training_ops ApplyRMSProp (CPU functor):
//   ms  += (grad^2 - ms) * (1 - rho)
//   mom  = mom * momentum + (grad * lr) / sqrt(ms + epsilon)
//   var -= mom
// clip_by_global_norm: scale = clip * min(1/norm, 1/clip) (both factors fp32).
// One float4 of (w, ms, mom, g) per thread (VEC; else one float), its four loads issued before
// the block reduces the norm partials so their latency overlaps that reduction.
template <bool VEC>
__global__ __launch_bounds__(256) void clip_rmsprop_kernel(
    float *__restrict__ w, float *__restrict__ ms, float *__restrict__ mom,
    const float *__restrict__ g, size_t n, const float *__restrict__ partials,
    const float *__restrict__ lr_dev, float decay, float momentum, float eps, float clip,
    int clip_type, float s, float *__restrict__ norm_out) {
#pragma clang fp contract(off)  // TF's operation-by-operation rounding, no fused multiply-add
  constexpr int V = VEC ? 4 : 1;
  __shared__ float sh_scale;
  const size_t i0 = ((size_t)blockIdx.x * blockDim.x + threadIdx.x) * V;
  const bool full = i0 + V <= n;
  f32x4 gv{0.f, 0.f, 0.f, 0.f}, mv{0.f, 0.f, 0.f, 0.f}, ov{0.f, 0.f, 0.f, 0.f}, wv{0.f, 0.f, 0.f, 0.f};
  if (VEC && full) {
    gv = *reinterpret_cast<const f32x4 *>(g + i0);
    mv = *reinterpret_cast<const f32x4 *>(ms + i0);
    ov = *reinterpret_cast<const f32x4 *>(mom + i0);
    wv = *reinterpret_cast<const f32x4 *>(w + i0);
  } else {
    for (int k = 0; k < V; ++k)
      if (i0 + k < n) {
        gv[k] = g[i0 + k];
        mv[k] = ms[i0 + k];
        ov[k] = mom[i0 + k];
        wv[k] = w[i0 + k];
      }
  }
  // the LR word lives in pinned host memory (written between launches; each dispatch's acquire
  // makes it visible): requested with the operands, so its PCIe round trip overlaps the norm
  // reduction instead of following the barrier
  const float lr = *lr_dev;
  if (threadIdx.x < 64) {
    // every partial of the lane requested before the first add (a rolled loop waited out one load
    // latency per partial: 8 round trips); the adds stay in index order
    static_assert(MT_NORM_PARTIALS % 64 == 0, "partials per lane");
    constexpr int PL = MT_NORM_PARTIALS / 64;
    float pv[PL];
#pragma unroll
    for (int u = 0; u < PL; ++u) pv[u] = partials[threadIdx.x + 64 * u];
    double acc = 0.0;
#pragma unroll
    for (int u = 0; u < PL; ++u) acc += (double)pv[u];
    acc = wave_sum_d(acc);
    if (threadIdx.x == 0) {
      const float norm = sqrtf((float)acc);
      float scale = s;
      if (clip_type == MT_CLIP_GLOBAL) {
        const float inv_clip = (float)(1.0 / (double)clip);
        scale = s * (clip * fminf(1.0f / norm, inv_clip));
      }
      sh_scale = scale;
      if (norm_out && blockIdx.x == 0) *norm_out = norm;
    }
  }
  __syncthreads();
  const float scale = sh_scale;
  const float one_m_rho = 1.0f - decay;
#pragma unroll
  for (int k = 0; k < V; ++k) {
    // with s != 1 (data parallel), g is the SUM over ranks: scale folds 1/world and the clip.
    const float gi = (clip_type == MT_CLIP_GLOBAL) ? gv[k] * scale : gv[k] * s;
    float m = mv[k];
    m = m + (gi * gi - m) * one_m_rho;
    const float mo = ov[k] * momentum + (gi * lr) / sqrtf(m + eps);
    mv[k] = m;
    ov[k] = mo;
    wv[k] = wv[k] - mo;
  }
  if (VEC && full) {
    *reinterpret_cast<f32x4 *>(ms + i0) = mv;
    *reinterpret_cast<f32x4 *>(mom + i0) = ov;
    *reinterpret_cast<f32x4 *>(w + i0) = wv;
  } else {
    for (int k = 0; k < V; ++k)
      if (i0 + k < n) {
        ms[i0 + k] = mv[k];
        mom[i0 + k] = ov[k];
        w[i0 + k] = wv[k];
      }
  }
}

// ---------------------------------------------------------------------------------------------
// A2: block = (12 output rows, env). Phase 1 streams the source rows those output rows read
// (row_lut) of both frames of each of the env's p pushes with 16-byte loads — HBM, or host
// memory over PCIe when the staging is read in place — and keeps max(f0, f1) in LDS. Phase 2
// gathers the resize columns (col_lut) from LDS and writes each pixel's 4*depth stacked
// channels: the p new pooled frames after the prev channels they push out.
// ---------------------------------------------------------------------------------------------
constexpr int kPreRows = 12;  // 84 = 7 x 12

typedef unsigned char u8x16 __attribute__((ext_vector_type(16)));

// Source of push j of env e, by mode:
//   kSrcPairs   staging slot push_offset[e] + j holds the push's two SH-row screens;
//   kSrcPooled  staging slot push_offset[e] + j holds ONE SH-row screen, max(f0, f1) already
//               taken by the emulator's frame pool on the host (mt_preprocess_pooled);
//   kSrcBank    frames read where the emulators left them: frame f is screen frame_idx[e*8+2j+f]
//               of a bank of whole 210-row screens (mt_preprocess_frames).
//   kSrcFinal   staging slot push_offset[e] + j holds the push's FINAL 84x84 frame (pool + resize
//               done by the host threads, MH_RUNNER_RESIZED; mt_preprocess_resized): the block
//               streams its 12 output rows (contiguous) and only stacks them.
enum { kSrcPairs = 0, kSrcPooled = 1, kSrcBank = 2, kSrcFinal = 3 };
template <int DEPTH, int SRC>
__global__ __launch_bounds__(256) void preprocess_kernel(
    const uint8_t *__restrict__ raw, const int32_t *__restrict__ push_offset,
    const int32_t *__restrict__ push_count, int SH, const int32_t *__restrict__ row_lut,
    const int32_t *__restrict__ col_lut, const uint8_t *__restrict__ prev, uint8_t *__restrict__ out) {
  constexpr int ROWB = 160 * DEPTH;  // bytes of one screen row
  constexpr int Q = ROWB / 16;
  constexpr int C = 4 * DEPTH;
  __shared__ u8x16 pooled[4][kPreRows][Q];
  __shared__ int rl[kPreRows], cl[84];
  __shared__ size_t foff[8];  // byte offset of (push j, frame f) = foff[2j + f]
  const int e = blockIdx.y, y0 = blockIdx.x * kPreRows;
  const int p = min(max(push_count[e], 1), 4);
  const size_t FR = (size_t)SH * ROWB;  // one screen
  constexpr int FROW = 84 * DEPTH;      // bytes of one final (resized) row
  if constexpr (SRC != kSrcFinal) {
    if (threadIdx.x < kPreRows) rl[threadIdx.x] = row_lut[y0 + threadIdx.x];
    if (threadIdx.x < 84) cl[threadIdx.x] = col_lut[threadIdx.x];
  }
  if (threadIdx.x < 8) {
    const int j = threadIdx.x >> 1, f = threadIdx.x & 1;
    if constexpr (SRC == kSrcBank)
      foff[threadIdx.x] = j < p ? (size_t)push_offset[e * 8 + threadIdx.x] * FR : 0;
    else if constexpr (SRC == kSrcPooled)
      foff[threadIdx.x] = ((size_t)push_offset[e] + j) * FR;
    else if constexpr (SRC == kSrcFinal)
      foff[threadIdx.x] = ((size_t)push_offset[e] + j) * 84 * FROW + (size_t)y0 * FROW;
    else
      foff[threadIdx.x] = ((size_t)push_offset[e] + j) * 2 * FR + f * FR;
  }
  __syncthreads();
  if constexpr (SRC == kSrcFinal) {
    // rows y0 .. y0+11 of each push's final frame are contiguous: 12*84*DEPTH/16 loads per push
    constexpr int N16 = kPreRows * FROW / 16;
    static_assert(kPreRows * FROW % 16 == 0 && N16 <= kPreRows * Q, "final rows fit the LDS stage");
    for (int i = threadIdx.x; i < p * N16; i += 256) {
      const int j = i / N16, q = i - j * N16;
      (&pooled[j][0][0])[q] = reinterpret_cast<const u8x16 *>(raw + foff[2 * j])[q];
    }
    __syncthreads();
    const uint8_t *pl = reinterpret_cast<const uint8_t *>(&pooled[0][0][0]);
    for (int i = threadIdx.x; i < kPreRows * 84; i += 256) {
      const int r = i / 84, x = i - r * 84;
      const size_t o = (((size_t)e * 84 + y0 + r) * 84 + x) * C;
#pragma unroll
      for (int col = 0; col < DEPTH; ++col) {
        uint32_t v = p < 4 ? *reinterpret_cast<const uint32_t *>(prev + o + col * 4) >> (8 * p) : 0u;
        for (int j = 0; j < p; ++j)
          v |= (uint32_t)pl[j * kPreRows * ROWB + r * FROW + x * DEPTH + col] << (8 * (4 - p + j));
        *reinterpret_cast<uint32_t *>(out + o + col * 4) = v;
      }
    }
    return;
  }
  for (int i = threadIdx.x; i < p * kPreRows * Q; i += 256) {
    const int j = i / (kPreRows * Q), rem = i - j * (kPreRows * Q);
    const int r = rem / Q, q = rem - r * Q;
    const size_t ro = (size_t)rl[r] * ROWB;
    const u8x16 a = reinterpret_cast<const u8x16 *>(raw + foff[2 * j] + ro)[q];
    if constexpr (SRC == kSrcPooled) {
      pooled[j][r][q] = a;
    } else {
      const u8x16 b = reinterpret_cast<const u8x16 *>(raw + foff[2 * j + 1] + ro)[q];
      pooled[j][r][q] = __builtin_elementwise_max(a, b);  // np.amax over the 2-frame pool
    }
  }
  __syncthreads();
  const uint8_t *pl = reinterpret_cast<const uint8_t *>(&pooled[0][0][0]);
  for (int i = threadIdx.x; i < kPreRows * 84; i += 256) {
    const int r = i / 84, x = i - r * 84;
    const size_t o = (((size_t)e * 84 + y0 + r) * 84 + x) * C;
    const int src = cl[x] * DEPTH;
#pragma unroll
    for (int col = 0; col < DEPTH; ++col) {
      uint32_t v = p < 4 ? *reinterpret_cast<const uint32_t *>(prev + o + col * 4) >> (8 * p) : 0u;
      for (int j = 0; j < p; ++j)
        v |= (uint32_t)pl[(j * kPreRows + r) * ROWB + src + col] << (8 * (4 - p + j));
      *reinterpret_cast<uint32_t *>(out + o + col * 4) = v;
    }
  }
}

// ---------------------------------------------------------------------------------------------
// A3 perf mode: counter-based uniforms, inverse CDF over (p - epsneg(float32)).
// ---------------------------------------------------------------------------------------------
__global__ void sample_kernel(const float *__restrict__ pi, const float *__restrict__ rep, int B,
                              int A, int R, uint64_t seed, int row0, uint64_t *__restrict__ counters,
                              int32_t *__restrict__ a_idx, int32_t *__restrict__ r_idx,
                              int32_t *__restrict__ pair) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= B) return;
  int a, r;
  sample_row(pi + (size_t)b * A, A, rep + (size_t)b * R, R, seed, b, row0, counters, &a, &r);
  a_idx[b] = a;
  r_idx[b] = r;
  if (pair) {
    pair[b] = a;
    pair[B + b] = r;
  }
}

}  // namespace mt

using namespace mt;

extern "C" const char *mt_last_error(void) { return g_err; }

extern "C" int mt_version(void) { return 1; }

bool mt::g_win_on = false;
int mt::g_win_first = 0, mt::g_win_count = -1, mt::g_win_index = 0;
extern "C" int mt_launch_window(int first, int count) {
  const int seen = g_win_index;
  g_win_on = first >= 0;
  g_win_first = first;
  g_win_count = count;
  g_win_index = 0;
  return seen;
}

extern "C" int mt_returns(const float *rewards, const float *masks, const float *values,
                          const float *v_boot, double gamma, int T, int E, float *y, float *adv,
                          mt_stream_t stream) {
  MT_CHECK_ARG(rewards && masks && values && v_boot && y && adv, "null argument");
  MT_CHECK_ARG(T >= 1 && E >= 1, "T and E must be >= 1");
  hipLaunchKernelGGL(returns_kernel, dim3(cdiv(E, 64)), dim3(64), 0, (hipStream_t)stream, rewards,
                     masks, values, v_boot, gamma, T, E, y, adv);
  MT_LAUNCHED();
  return MT_OK;
}

extern "C" int mt_grad_sumsq(const float *g, size_t n, float inv_scale, float *partials,
                             mt_stream_t stream) {
  MT_CHECK_ARG(g && partials, "null argument");
  hipLaunchKernelGGL(sumsq_kernel, dim3(MT_NORM_PARTIALS), dim3(256), 0, (hipStream_t)stream, g, n,
                     inv_scale, partials);
  MT_LAUNCHED();
  return MT_OK;
}

extern "C" int mt_clip_rmsprop(float *w, float *ms, float *mom, const float *g, size_t n,
                               const float *partials, const float *lr_dev, float decay,
                               float momentum, float eps, float clip, int clip_type,
                               float inv_scale, float *norm_out, mt_stream_t stream) {
  MT_CHECK_ARG(w && ms && mom && g && partials && lr_dev, "null argument");
  MT_CHECK_ARG(clip_type == MT_CLIP_IGNORE || clip_type == MT_CLIP_GLOBAL,
               "clip_type %d not supported (reference 'local' is broken: actor_learner.py:66-67)",
               clip_type);
  MT_CHECK_ARG(clip_type != MT_CLIP_GLOBAL || clip > 0.f, "clip must be > 0");
  MT_CHECK_ARG(n <= ((size_t)1 << 36), "n too large");
  const bool vec = ((((uintptr_t)w) | ((uintptr_t)ms) | ((uintptr_t)mom) | ((uintptr_t)g)) & 15) == 0;
  const size_t per_thread = vec ? 4 : 1;
  int blocks = (int)((n + 256 * per_thread - 1) / (256 * per_thread));
  if (blocks < 1) blocks = 1;
  if (vec)
    hipLaunchKernelGGL(clip_rmsprop_kernel<true>, dim3(blocks), dim3(256), 0, (hipStream_t)stream, w, ms, mom, g, n,
                       partials, lr_dev, decay, momentum, eps, clip, clip_type, inv_scale, norm_out);
  else
    hipLaunchKernelGGL(clip_rmsprop_kernel<false>, dim3(blocks), dim3(256), 0, (hipStream_t)stream, w, ms, mom, g, n,
                       partials, lr_dev, decay, momentum, eps, clip, clip_type, inv_scale, norm_out);
  MT_LAUNCHED();
  return MT_OK;
}

extern "C" int mt_preprocess(const uint8_t *raw, const int32_t *push_offset,
                             const int32_t *push_count, int E, int depth, int src_rows,
                             const int32_t *row_lut, const int32_t *col_lut, const uint8_t *prev,
                             uint8_t *out, mt_stream_t stream) {
  MT_CHECK_ARG(raw && push_offset && push_count && row_lut && col_lut && prev && out,
               "null argument");
  MT_CHECK_ARG(E >= 1, "E must be >= 1");
  MT_CHECK_ARG(src_rows >= 84 && src_rows <= 210, "src_rows must be in [84, 210]");
  MT_CHECK_ARG(prev != out, "out may not alias prev");
  MT_CHECK_ARG(((uintptr_t)raw & 15) == 0, "raw must be 16-byte aligned");
  const dim3 grid(84 / kPreRows, E);
  if (depth == 1) {
    hipLaunchKernelGGL((preprocess_kernel<1, kSrcPairs>), grid, dim3(256), 0, (hipStream_t)stream, raw, push_offset,
                       push_count, src_rows, row_lut, col_lut, prev, out);
  } else if (depth == 3) {
    hipLaunchKernelGGL((preprocess_kernel<3, kSrcPairs>), grid, dim3(256), 0, (hipStream_t)stream, raw, push_offset,
                       push_count, src_rows, row_lut, col_lut, prev, out);
  } else {
    set_error("depth must be 1 or 3");
    return MT_ERR_ARG;
  }
  MT_LAUNCHED();
  return MT_OK;
}

extern "C" int mt_preprocess_pooled(const uint8_t *raw, const int32_t *push_offset,
                                    const int32_t *push_count, int E, int depth, int src_rows,
                                    const int32_t *row_lut, const int32_t *col_lut, const uint8_t *prev,
                                    uint8_t *out, mt_stream_t stream) {
  MT_CHECK_ARG(raw && push_offset && push_count && row_lut && col_lut && prev && out, "null argument");
  MT_CHECK_ARG(E >= 1, "E must be >= 1");
  MT_CHECK_ARG(src_rows >= 84 && src_rows <= 210, "src_rows must be in [84, 210]");
  MT_CHECK_ARG(prev != out, "out may not alias prev");
  MT_CHECK_ARG(((uintptr_t)raw & 15) == 0, "raw must be 16-byte aligned");
  const dim3 grid(84 / kPreRows, E);
  if (depth == 1) {
    hipLaunchKernelGGL((preprocess_kernel<1, kSrcPooled>), grid, dim3(256), 0, (hipStream_t)stream, raw, push_offset,
                       push_count, src_rows, row_lut, col_lut, prev, out);
  } else if (depth == 3) {
    hipLaunchKernelGGL((preprocess_kernel<3, kSrcPooled>), grid, dim3(256), 0, (hipStream_t)stream, raw, push_offset,
                       push_count, src_rows, row_lut, col_lut, prev, out);
  } else {
    set_error("depth must be 1 or 3");
    return MT_ERR_ARG;
  }
  MT_LAUNCHED();
  return MT_OK;
}

extern "C" int mt_preprocess_resized(const uint8_t *frames, const int32_t *push_offset, const int32_t *push_count,
                                     int E, int depth, const uint8_t *prev, uint8_t *out, mt_stream_t stream) {
  MT_CHECK_ARG(frames && push_offset && push_count && prev && out, "null argument");
  MT_CHECK_ARG(E >= 1, "E must be >= 1");
  MT_CHECK_ARG(prev != out, "out may not alias prev");
  MT_CHECK_ARG(((uintptr_t)frames & 15) == 0, "frames must be 16-byte aligned");
  const dim3 grid(84 / kPreRows, E);
  if (depth == 1) {
    hipLaunchKernelGGL((preprocess_kernel<1, kSrcFinal>), grid, dim3(256), 0, (hipStream_t)stream, frames,
                       push_offset, push_count, 84, nullptr, nullptr, prev, out);
  } else if (depth == 3) {
    hipLaunchKernelGGL((preprocess_kernel<3, kSrcFinal>), grid, dim3(256), 0, (hipStream_t)stream, frames,
                       push_offset, push_count, 84, nullptr, nullptr, prev, out);
  } else {
    set_error("depth must be 1 or 3");
    return MT_ERR_ARG;
  }
  MT_LAUNCHED();
  return MT_OK;
}

extern "C" int mt_preprocess_frames(const uint8_t *screens, const int32_t *frame_idx,
                                    const int32_t *push_count, int E, int depth, const int32_t *row_lut,
                                    const int32_t *col_lut, const uint8_t *prev, uint8_t *out,
                                    mt_stream_t stream) {
  MT_CHECK_ARG(screens && frame_idx && push_count && row_lut && col_lut && prev && out, "null argument");
  MT_CHECK_ARG(E >= 1, "E must be >= 1");
  MT_CHECK_ARG(prev != out, "out may not alias prev");
  MT_CHECK_ARG(((uintptr_t)screens & 15) == 0, "screens must be 16-byte aligned");
  const dim3 grid(84 / kPreRows, E);
  if (depth == 1) {
    hipLaunchKernelGGL((preprocess_kernel<1, kSrcBank>), grid, dim3(256), 0, (hipStream_t)stream, screens, frame_idx,
                       push_count, 210, row_lut, col_lut, prev, out);
  } else if (depth == 3) {
    hipLaunchKernelGGL((preprocess_kernel<3, kSrcBank>), grid, dim3(256), 0, (hipStream_t)stream, screens, frame_idx,
                       push_count, 210, row_lut, col_lut, prev, out);
  } else {
    set_error("depth must be 1 or 3");
    return MT_ERR_ARG;
  }
  MT_LAUNCHED();
  return MT_OK;
}

extern "C" int mt_host_device_pointer(void *host, void **dev) {
  MT_CHECK_ARG(host && dev, "null argument");
  MT_HIP(hipHostGetDevicePointer(dev, host, 0));
  return MT_OK;
}

extern "C" int mt_sample(const float *pi, const float *rep, int batch, int num_actions,
                         int num_reps, uint64_t seed, int row0, uint64_t *counters, int32_t *a_idx,
                         int32_t *r_idx, int32_t *pair, mt_stream_t stream) {
  MT_CHECK_ARG(pi && rep && counters && a_idx && r_idx, "null argument");
  MT_CHECK_ARG(batch >= 1 && num_actions >= 1 && num_reps >= 1 && row0 >= 0, "bad sizes");
  hipLaunchKernelGGL(sample_kernel, dim3(cdiv(batch, 64)), dim3(64), 0, (hipStream_t)stream, pi,
                     rep, batch, num_actions, num_reps, seed, row0, counters, a_idx, r_idx, pair);
  MT_LAUNCHED();
  return MT_OK;
}

extern "C" int mt_graph_begin(mt_stream_t stream) {
  MT_CHECK_ARG(stream != nullptr, "graph capture needs a non-default stream");
  MT_HIP(hipStreamBeginCapture((hipStream_t)stream, hipStreamCaptureModeThreadLocal));
  return MT_OK;
}

extern "C" int mt_graph_end(mt_stream_t stream, void **graph_exec) {
  MT_CHECK_ARG(stream && graph_exec, "null argument");
  hipGraph_t g = nullptr;
  MT_HIP(hipStreamEndCapture((hipStream_t)stream, &g));
  hipGraphExec_t ex = nullptr;
  hipError_t e = hipGraphInstantiate(&ex, g, nullptr, nullptr, 0);
  (void)hipGraphDestroy(g);
  if (e != hipSuccess) {
    set_error("hipGraphInstantiate failed: %s", hipGetErrorString(e));
    return MT_ERR_HIP;
  }
  *graph_exec = (void *)ex;
  return MT_OK;
}

extern "C" int mt_graph_launch(void *graph_exec, mt_stream_t stream) {
  MT_CHECK_ARG(graph_exec, "null graph");
  MT_HIP(hipGraphLaunch((hipGraphExec_t)graph_exec, (hipStream_t)stream));
  return MT_OK;
}

extern "C" int mt_graph_destroy(void *graph_exec) {
  if (graph_exec) MT_HIP(hipGraphExecDestroy((hipGraphExec_t)graph_exec));
  return MT_OK;
}

// ---- LSTM memory window (paac.py:79-83, :191-203) --------------------------------------------
// One thread per 16-byte column of a frame of env e: reads that column of the 5 window frames
// and of the new state, writes the window to whole_t (whole_memory[t] = memory), then the
// shifted window (memory[:, :-1] = memory[:, 1:]; memory[:, -1] = new state), or zeros when the
// episode ended (mask == 0, paac.py:202-203). Each thread touches only its own column: no race.
__global__ __launch_bounds__(256) void memory_push_kernel(uint4 *__restrict__ memory, uint4 *__restrict__ whole_t,
                                                          const uint4 *__restrict__ fresh,
                                                          const float *__restrict__ masks, int E, int n16) {
  const int e = blockIdx.y;
  const bool keep = masks[e] != 0.f;
  const uint4 z = make_uint4(0, 0, 0, 0);
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n16; i += gridDim.x * blockDim.x) {
    uint4 m[5];
#pragma unroll
    for (int k = 0; k < 5; ++k) m[k] = memory[((size_t)e * 5 + k) * n16 + i];
    const uint4 f = fresh[(size_t)e * n16 + i];
#pragma unroll
    for (int k = 0; k < 5; ++k) whole_t[((size_t)e * 5 + k) * n16 + i] = m[k];
#pragma unroll
    for (int k = 0; k < 5; ++k) memory[((size_t)e * 5 + k) * n16 + i] = keep ? (k < 4 ? m[k + 1] : f) : z;
  }
}

extern "C" int mt_memory_push(uint8_t *memory, uint8_t *whole_t, const uint8_t *fresh, const float *masks, int E,
                              size_t frame_bytes, mt_stream_t stream) {
  MT_CHECK_ARG(memory && whole_t && fresh && masks, "null argument");
  MT_CHECK_ARG(E >= 1, "E must be >= 1");
  MT_CHECK_ARG(frame_bytes % 16 == 0, "frame_bytes must be a multiple of 16");
  MT_CHECK_ARG((((uintptr_t)memory | (uintptr_t)fresh | (uintptr_t)whole_t) & 15) == 0,
               "buffers must be 16-byte aligned");
  MT_CHECK_ARG(whole_t != memory, "whole_t may not alias memory");
  const int n16 = (int)(frame_bytes / 16);
  const dim3 grid((unsigned)std::min(cdiv(n16, 256), 64), (unsigned)E);
  hipLaunchKernelGGL(memory_push_kernel, grid, dim3(256), 0, (hipStream_t)stream, reinterpret_cast<uint4 *>(memory),
                     reinterpret_cast<uint4 *>(whole_t), reinterpret_cast<const uint4 *>(fresh), masks, E, n16);
  MT_LAUNCHED();
  return MT_OK;
}
