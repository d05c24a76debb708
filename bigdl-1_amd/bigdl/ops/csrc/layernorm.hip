// Layer normalisation over the last dimension (Transformer LayerNormalization, reference
// nn/LayerNormalization.scala): y = (x − μ)·rstd·w + b, eps as given.
//
// One wave per row, fp32 statistics: the mean from a wave reduction, the variance from a second
// pass over (x − μ)² (the row is L2-resident), then the normalised write — 3 row sweeps instead of
// the 8 separate elementwise / reduction launches of the composed formulation.  Backward: per row
// ĝ = gy·w, gx = rstd·(ĝ − mean(ĝ) − x̂·mean(ĝ·x̂)); the parameter gradients Σ gy·x̂ and Σ gy are
// kept per lane for the lane's columns across the rows a wave visits and added once per wave with
// fp32 atomics (columns strided by 64: each lane owns H/64 of them, H ≤ 64·LN_MAX_COLS).
#include "common.h"

constexpr int LN_MAX_COLS = 64;  // H ≤ 4096

template <typename T>
__device__ __forceinline__ float ln_ld(const T* p);
template <>
__device__ __forceinline__ float ln_ld<float>(const float* p) { return *p; }
template <>
__device__ __forceinline__ float ln_ld<bf16_t>(const bf16_t* p) { return bf2f(*p); }
template <typename T>
__device__ __forceinline__ void ln_st(T* p, float v);
template <>
__device__ __forceinline__ void ln_st<float>(float* p, float v) { *p = v; }
template <>
__device__ __forceinline__ void ln_st<bf16_t>(bf16_t* p, float v) { *p = f2bf(v); }

template <typename T>
__global__ void __launch_bounds__(256) k_ln_fwd(const T* __restrict__ x, const float* __restrict__ w,
                                                const float* __restrict__ b, T* __restrict__ y,
                                                float* __restrict__ mean_out, float* __restrict__ rstd_out,
                                                long long rows, int H, float eps) {
  const int lane = threadIdx.x & 63;
  const long long nw = (long long)gridDim.x * 4;
  for (long long r = blockIdx.x * 4ll + (threadIdx.x >> 6); r < rows; r += nw) {
    const T* xr = x + r * H;
    float s = 0.f;
    for (int c = lane; c < H; c += 64) s += ln_ld<T>(xr + c);
    const float mu = wave_sum(s) / H;
    float q = 0.f;
    for (int c = lane; c < H; c += 64) {
      const float d = ln_ld<T>(xr + c) - mu;
      q = fmaf(d, d, q);
    }
    const float rstd = rsqrtf(wave_sum(q) / H + eps);
    T* yr = y + r * H;
    for (int c = lane; c < H; c += 64)
      ln_st<T>(yr + c, fmaf((ln_ld<T>(xr + c) - mu) * rstd, w ? w[c] : 1.f, b ? b[c] : 0.f));
    if (lane == 0) {
      mean_out[r] = mu;
      rstd_out[r] = rstd;
    }
  }
}

template <typename T>
__global__ void __launch_bounds__(256) k_ln_bwd(const T* __restrict__ gy, const T* __restrict__ x,
                                                const float* __restrict__ w, const float* __restrict__ mean,
                                                const float* __restrict__ rstd, T* __restrict__ gx,
                                                float* __restrict__ gw, float* __restrict__ gb, long long rows,
                                                int H) {
  const int lane = threadIdx.x & 63;
  const long long nw = (long long)gridDim.x * 4;
  float aw[LN_MAX_COLS], ab[LN_MAX_COLS];
#pragma unroll
  for (int j = 0; j < LN_MAX_COLS; ++j) {
    aw[j] = 0.f;
    ab[j] = 0.f;
  }
  for (long long r = blockIdx.x * 4ll + (threadIdx.x >> 6); r < rows; r += nw) {
    const T* gr = gy + r * H;
    const T* xr = x + r * H;
    const float mu = mean[r], rs = rstd[r];
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int j = 0; j < LN_MAX_COLS; ++j) {
      const int c = lane + 64 * j;
      if (c >= H) break;
      const float g = ln_ld<T>(gr + c);
      const float xh = (ln_ld<T>(xr + c) - mu) * rs;
      const float gh = g * (w ? w[c] : 1.f);
      s1 += gh;
      s2 = fmaf(gh, xh, s2);
      aw[j] = fmaf(g, xh, aw[j]);
      ab[j] += g;
    }
    const float m1 = wave_sum(s1) / H, m2 = wave_sum(s2) / H;
    T* gxr = gx + r * H;
    for (int c = lane; c < H; c += 64) {
      const float xh = (ln_ld<T>(xr + c) - mu) * rs;
      const float gh = ln_ld<T>(gr + c) * (w ? w[c] : 1.f);
      ln_st<T>(gxr + c, rs * (gh - m1 - xh * m2));
    }
  }
#pragma unroll
  for (int j = 0; j < LN_MAX_COLS; ++j) {
    const int c = lane + 64 * j;
    if (c >= H) break;
    if (gw) atomicAdd(gw + c, aw[j]);
    if (gb) atomicAdd(gb + c, ab[j]);
  }
}

// ---- register-resident vector path: H % V == 0, H ≤ 64·V·J, 16-byte aligned rows.  Each lane
// holds J vectors of V elements (bf16: 8 per 16-byte load, fp32: 4), so a row is read from HBM
// once and written once; statistics come from the registers.
template <typename T>
struct LnVec;
template <>
struct LnVec<bf16_t> {
  static constexpr int V = 8;
  static __device__ __forceinline__ void ld(const bf16_t* p, float* o) { load8(p, o); }
  static __device__ __forceinline__ void st(bf16_t* p, const float* o) { store8(p, o); }
};
template <>
struct LnVec<float> {
  static constexpr int V = 4;
  static __device__ __forceinline__ void ld(const float* p, float* o) {
    const float4 u = *reinterpret_cast<const float4*>(p);
    o[0] = u.x, o[1] = u.y, o[2] = u.z, o[3] = u.w;
  }
  static __device__ __forceinline__ void st(float* p, const float* o) {
    *reinterpret_cast<float4*>(p) = make_float4(o[0], o[1], o[2], o[3]);
  }
};

template <int V>
__device__ __forceinline__ void ln_ldp(const float* p, float* o) {
#pragma unroll
  for (int i = 0; i < V; i += 4) {
    const float4 u = *reinterpret_cast<const float4*>(p + i);
    o[i] = u.x, o[i + 1] = u.y, o[i + 2] = u.z, o[i + 3] = u.w;
  }
}

template <typename T, int J>
__global__ void __launch_bounds__(256) k_ln_fwd_v(const T* __restrict__ x, const float* __restrict__ w,
                                                  const float* __restrict__ b, T* __restrict__ y,
                                                  float* __restrict__ mean_out, float* __restrict__ rstd_out,
                                                  long long rows, int H, float eps) {
  constexpr int V = LnVec<T>::V;
  const int lane = threadIdx.x & 63;
  const long long nw = (long long)gridDim.x * 4;
  for (long long r = blockIdx.x * 4ll + (threadIdx.x >> 6); r < rows; r += nw) {
    const T* xr = x + r * H;
    float v[J][V];
    float s = 0.f;
#pragma unroll
    for (int j = 0; j < J; ++j) {
      const int c0 = (lane + 64 * j) * V;
      if (c0 < H) {
        LnVec<T>::ld(xr + c0, v[j]);
#pragma unroll
        for (int i = 0; i < V; ++i) s += v[j][i];
      }
    }
    const float mu = wave_sum(s) / H;
    float q = 0.f;
#pragma unroll
    for (int j = 0; j < J; ++j) {
      if ((lane + 64 * j) * V < H) {
#pragma unroll
        for (int i = 0; i < V; ++i) {
          v[j][i] -= mu;
          q = fmaf(v[j][i], v[j][i], q);
        }
      }
    }
    const float rstd = rsqrtf(wave_sum(q) / H + eps);
    T* yr = y + r * H;
#pragma unroll
    for (int j = 0; j < J; ++j) {
      const int c0 = (lane + 64 * j) * V;
      if (c0 < H) {
        float wv[V], bv[V], o[V];
        if (w) ln_ldp<V>(w + c0, wv);
        if (b) ln_ldp<V>(b + c0, bv);
#pragma unroll
        for (int i = 0; i < V; ++i) o[i] = fmaf(v[j][i] * rstd, w ? wv[i] : 1.f, b ? bv[i] : 0.f);
        LnVec<T>::st(yr + c0, o);
      }
    }
    if (lane == 0) {
      mean_out[r] = mu;
      rstd_out[r] = rstd;
    }
  }
}

// backward: gx per row from registers; Σ gy·x̂ / Σ gy per lane-owned column across the block's rows,
// folded over the block's 4 waves in LDS in wave order, one partial row [2H] per block (no atomics:
// deterministic), summed over blocks by k_ln_colsum
template <typename T, int J, bool KEEP>
__global__ void __launch_bounds__(256) k_ln_bwd_v(const T* __restrict__ gy, const T* __restrict__ x,
                                                  const float* __restrict__ w, const float* __restrict__ mean,
                                                  const float* __restrict__ rstd, T* __restrict__ gx,
                                                  float* __restrict__ partial, long long rows, int H) {
  constexpr int V = LnVec<T>::V;
  extern __shared__ float lds[];  // [2H]
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const long long nw = (long long)gridDim.x * 4;
  float aw[J][V], ab[J][V];
#pragma unroll
  for (int j = 0; j < J; ++j)
#pragma unroll
    for (int i = 0; i < V; ++i) aw[j][i] = ab[j][i] = 0.f;
  for (long long r = blockIdx.x * 4ll + wid; r < rows; r += nw) {
    const T* gr = gy + r * H;
    const T* xr = x + r * H;
    const float mu = mean[r], rs = rstd[r];
    // KEEP: the row stays in registers between the two sweeps; otherwise (wide rows, where
    // registers go to the parameter-gradient accumulators) the second sweep re-reads it from L2
    float g[KEEP ? J : 1][V], xh[KEEP ? J : 1][V];
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int j = 0; j < J; ++j) {
      const int c0 = (lane + 64 * j) * V;
      if (c0 < H) {
        constexpr int dummy = 0;
        float wv[V];
        float* gj = g[KEEP ? j : dummy];
        float* xj = xh[KEEP ? j : dummy];
        LnVec<T>::ld(gr + c0, gj);
        LnVec<T>::ld(xr + c0, xj);
        if (w) ln_ldp<V>(w + c0, wv);
#pragma unroll
        for (int i = 0; i < V; ++i) {
          xj[i] = (xj[i] - mu) * rs;
          aw[j][i] = fmaf(gj[i], xj[i], aw[j][i]);
          ab[j][i] += gj[i];
          gj[i] *= w ? wv[i] : 1.f;  // ĝ
          s1 += gj[i];
          s2 = fmaf(gj[i], xj[i], s2);
        }
      }
    }
    const float m1 = wave_sum(s1) / H, m2 = wave_sum(s2) / H;
    T* gxr = gx + r * H;
#pragma unroll
    for (int j = 0; j < J; ++j) {
      const int c0 = (lane + 64 * j) * V;
      if (c0 < H) {
        float o[V];
        if constexpr (KEEP) {
#pragma unroll
          for (int i = 0; i < V; ++i) o[i] = rs * (g[j][i] - m1 - xh[j][i] * m2);
        } else {
          float gv[V], xv[V], wv[V];
          LnVec<T>::ld(gr + c0, gv);
          LnVec<T>::ld(xr + c0, xv);
          if (w) ln_ldp<V>(w + c0, wv);
#pragma unroll
          for (int i = 0; i < V; ++i)
            o[i] = rs * (gv[i] * (w ? wv[i] : 1.f) - m1 - (xv[i] - mu) * rs * m2);
        }
        LnVec<T>::st(gxr + c0, o);
      }
    }
  }
  for (int k = 0; k < 4; ++k) {
    if (wid == k) {
#pragma unroll
      for (int j = 0; j < J; ++j) {
        const int c0 = (lane + 64 * j) * V;
        if (c0 < H) {
#pragma unroll
          for (int i = 0; i < V; ++i) {
            lds[c0 + i] = k ? lds[c0 + i] + aw[j][i] : aw[j][i];
            lds[H + c0 + i] = k ? lds[H + c0 + i] + ab[j][i] : ab[j][i];
          }
        }
      }
    }
    __syncthreads();
  }
  float* pr = partial + (long long)blockIdx.x * 2 * H;
  for (int c = threadIdx.x; c < 2 * H; c += 256) pr[c] = lds[c];
}

// Σ over the G block partials: 64 columns per block (one per lane, 256-byte coalesced rows), the
// G rows split over the block's 16 waves and folded in LDS in wave order (deterministic)
__global__ void __launch_bounds__(1024) k_ln_colsum(const float* __restrict__ partial, int G, int H,
                                                    float* __restrict__ gw, float* __restrict__ gb) {
  __shared__ float red[16][64];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int c = blockIdx.x * 64 + lane;
  float s = 0.f;
  if (c < 2 * H) {
#pragma unroll 8
    for (int g = wid; g < G; g += 16) s += partial[(long long)g * 2 * H + c];
  }
  red[wid][lane] = s;
  __syncthreads();
  if (wid == 0 && c < 2 * H) {
    float t = 0.f;
#pragma unroll
    for (int k = 0; k < 16; ++k) t += red[k][lane];
    float* dst = c < H ? gw : gb;
    if (dst) dst[c < H ? c : c - H] += t;
  }
}

template <typename T>
static bool ln_fwd_vec(const void* x, const float* w, const float* b, void* y, float* mean, float* rstd,
                       long long rows, int H, float eps, int grid, hipStream_t s) {
  constexpr int V = LnVec<T>::V;
  if (H % V || ((uintptr_t)x | (uintptr_t)y | (uintptr_t)w | (uintptr_t)b) & 15) return false;
  const int per = 64 * V;
#define LN_FWD(JJ)                                                                                                   \
  hipLaunchKernelGGL((k_ln_fwd_v<T, JJ>), dim3(grid), dim3(256), 0, s, (const T*)x, w, b, (T*)y, mean, rstd, rows, \
                     H, eps)
  if (H <= per) LN_FWD(1);
  else if (H <= 2 * per) LN_FWD(2);
  else if (H <= 4 * per) LN_FWD(4);
  else if (H <= 8 * per) LN_FWD(8);
  else return false;
#undef LN_FWD
  return true;
}

template <typename T>
static bool ln_bwd_vec(const void* gy, const void* x, const float* w, const float* mean, const float* rstd, void* gx,
                       float* gw, float* gb, long long rows, int H, float* scratch, long long scratch_len,
                       hipStream_t s) {
  constexpr int V = LnVec<T>::V;
  if (H % V || ((uintptr_t)gy | (uintptr_t)x | (uintptr_t)gx | (uintptr_t)w) & 15 || !scratch) return false;
  int G = bigdl_grid((rows + 3) / 4, 1, 512);
  if ((long long)G * 2 * H > scratch_len) G = (int)(scratch_len / (2ll * H));
  if (G < 1) return false;
  const int per = 64 * V;
  const size_t shm = 2 * H * sizeof(float);
#define LN_BWD(JJ)                                                                                            \
  hipLaunchKernelGGL((k_ln_bwd_v<T, JJ, (JJ * V <= 16)>), dim3(G), dim3(256), shm, s, (const T*)gy, (const T*)x, w, mean, rstd, \
                     (T*)gx, scratch, rows, H)
  if (H <= per) LN_BWD(1);
  else if (H <= 2 * per) LN_BWD(2);
  else if (H <= 4 * per) LN_BWD(4);
  else if (H <= 8 * per) LN_BWD(8);
  else return false;
#undef LN_BWD
  if (gw || gb)
    hipLaunchKernelGGL(k_ln_colsum, dim3((2 * H + 63) / 64), dim3(1024), 0, s, (const float*)scratch, G, H, gw, gb);
  return true;
}

// dtype 0 = fp32, 1 = bf16; x/y [rows][H] contiguous; w/b fp32 [H] or null; mean/rstd fp32 [rows]
BIGDL_EXPORT int bigdl_ln_fwd(const void* x, int dtype, const float* w, const float* b, void* y, float* mean,
                              float* rstd, long long rows, int H, float eps, hipStream_t s) {
  if (rows <= 0 || H <= 0) return (int)hipErrorInvalidValue;
  const int grid = bigdl_grid((rows + 3) / 4, 1, 16384);
  if (dtype == 0 ? ln_fwd_vec<float>(x, w, b, y, mean, rstd, rows, H, eps, grid, s)
                 : ln_fwd_vec<bf16_t>(x, w, b, y, mean, rstd, rows, H, eps, grid, s))
    BIGDL_CHECK_LAUNCH();
  if (dtype == 0)
    hipLaunchKernelGGL(k_ln_fwd<float>, dim3(grid), dim3(256), 0, s, (const float*)x, w, b, (float*)y, mean, rstd, rows,
                       H, eps);
  else
    hipLaunchKernelGGL(k_ln_fwd<bf16_t>, dim3(grid), dim3(256), 0, s, (const bf16_t*)x, w, b, (bf16_t*)y, mean, rstd,
                       rows, H, eps);
  BIGDL_CHECK_LAUNCH();
}

// gw / gb: fp32 [H], accumulated (zero them for a fresh gradient); scratch: fp32 block partials
// (≥ 2H floats for the vector path, ideally 512·2H; null → the scalar atomic path)
BIGDL_EXPORT int bigdl_ln_bwd(const void* gy, const void* x, int dtype, const float* w, const float* mean,
                              const float* rstd, void* gx, float* gw, float* gb, long long rows, int H,
                              float* scratch, long long scratch_len, hipStream_t s) {
  if (rows <= 0 || H <= 0 || H > 64 * LN_MAX_COLS) return (int)hipErrorInvalidValue;
  if (dtype == 0 ? ln_bwd_vec<float>(gy, x, w, mean, rstd, gx, gw, gb, rows, H, scratch, scratch_len, s)
                 : ln_bwd_vec<bf16_t>(gy, x, w, mean, rstd, gx, gw, gb, rows, H, scratch, scratch_len, s))
    BIGDL_CHECK_LAUNCH();
  // enough waves to fill the chip, few enough that the per-wave atomics stay cheap
  const int grid = bigdl_grid((rows + 3) / 4, 1, g_bigdl_deterministic ? 1 : 1024);
  if (dtype == 0)
    hipLaunchKernelGGL(k_ln_bwd<float>, dim3(grid), dim3(256), 0, s, (const float*)gy, (const float*)x, w, mean, rstd,
                       (float*)gx, gw, gb, rows, H);
  else
    hipLaunchKernelGGL(k_ln_bwd<bf16_t>, dim3(grid), dim3(256), 0, s, (const bf16_t*)gy, (const bf16_t*)x, w, mean,
                       rstd, (bf16_t*)gx, gw, gb, rows, H);
  BIGDL_CHECK_LAUNCH();
}
