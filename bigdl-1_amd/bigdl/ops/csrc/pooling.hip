// K10: max pooling, NHWC bf16 (SpatialMaxPooling.updateOutput / updateGradInput,
// DL/nn/SpatialMaxPooling.scala:175-216; NNPrimitive.maxPoolingForwardFloat :654).
//
// Forward: one thread per (output pixel, 8-channel group) — 16-B loads per window tap, the argmax
// kept as an int8 offset kh·kW + kw inside the window (1 B/element instead of torch's int64).
// Index math is 32-bit whenever the element count allows (64-bit division is a long software
// sequence on CDNA), 64-bit otherwise.
// Backward is a GATHER: each input pixel sums gy over the ≤⌈k/s⌉² windows that chose it, so gx is
// written exactly once (no zero-fill, no atomics).  Padding is implicit (-inf); ceil mode allowed.
#include "common.h"

struct PoolGeom {
  int N, H, W, C, P, Q, kh, kw, sh, sw, ph, pw;
};

// 8 consecutive channels of either element type (bf16: one 16-B access; fp32: two) — the fp32
// instantiations serve bigdl.compute.dtype=fp32 (the reference's precision), the bf16 ones the default.
__device__ __forceinline__ void pld8(const bf16_t* p, float* o) { load8(p, o); }
__device__ __forceinline__ void pld8(const float* p, float* o) {
  const float4 a = *reinterpret_cast<const float4*>(p), b = *reinterpret_cast<const float4*>(p + 4);
  o[0] = a.x; o[1] = a.y; o[2] = a.z; o[3] = a.w; o[4] = b.x; o[5] = b.y; o[6] = b.z; o[7] = b.w;
}
__device__ __forceinline__ void pst8(bf16_t* p, const float* o) { store8(p, o); }
__device__ __forceinline__ void pst8(float* p, const float* o) {
  *reinterpret_cast<float4*>(p) = make_float4(o[0], o[1], o[2], o[3]);
  *reinterpret_cast<float4*>(p + 4) = make_float4(o[4], o[5], o[6], o[7]);
}

template <typename IT, typename T = bf16_t>
__global__ void __launch_bounds__(256) k_maxpool_fwd(const T* __restrict__ x, T* __restrict__ y,
                                                     int8_t* __restrict__ idx, PoolGeom g) {
  const int CG = g.C >> 3;
  const IT total = (IT)g.N * g.P * g.Q * CG;
  for (IT t = blockIdx.x * (IT)blockDim.x + threadIdx.x; t < total; t += (IT)gridDim.x * blockDim.x) {
    const int cg = (int)(t % CG);
    IT pix = t / CG;
    const int q = (int)(pix % g.Q);
    pix /= g.Q;
    const int p = (int)(pix % g.P);
    const int n = (int)(pix / g.P);
    float best[8];
    int arg[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) { best[e] = -INFINITY; arg[e] = 0; }
    const int h0 = p * g.sh - g.ph, w0 = q * g.sw - g.pw;
    for (int i = 0; i < g.kh; ++i) {
      const int h = h0 + i;
      if ((unsigned)h >= (unsigned)g.H) continue;
      for (int j = 0; j < g.kw; ++j) {
        const int w = w0 + j;
        if ((unsigned)w >= (unsigned)g.W) continue;
        float v[8];
        pld8(x + (((size_t)n * g.H + h) * g.W + w) * g.C + cg * 8, v);
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          if (v[e] > best[e] || v[e] != v[e]) {  // NaN propagates like torch
            best[e] = v[e];
            arg[e] = i * g.kw + j;
          }
        }
      }
    }
    const size_t o = (((size_t)n * g.P + p) * g.Q + q) * g.C + cg * 8;
    pst8(y + o, best);
    if (!idx) continue;  // inference: no argmax for a backward (uniform per launch)
    uint32_t lo = 0, hi = 0;
#pragma unroll
    for (int e = 0; e < 4; ++e) lo |= (uint32_t)(arg[e] & 0xFF) << (8 * e);
#pragma unroll
    for (int e = 0; e < 4; ++e) hi |= (uint32_t)(arg[4 + e] & 0xFF) << (8 * e);
    *reinterpret_cast<uint2*>(idx + o) = make_uint2(lo, hi);
  }
}

// 3×3 / stride-2 windows (the ResNet stem pool): all nine 16-B window loads of a thread are issued
// before the first compare (branch-free: an out-of-image tap reads the window's centre and is masked),
// where the generic loop above kept one load in flight — 3.8 TB/s on the 112² stem pool.
template <typename IT, typename T = bf16_t>
__global__ void __launch_bounds__(256) k_maxpool_fwd_k3s2(const T* __restrict__ x, T* __restrict__ y,
                                                          int8_t* __restrict__ idx, PoolGeom g) {
  const int CG = g.C >> 3;
  const IT total = (IT)g.N * g.P * g.Q * CG;
  for (IT t = blockIdx.x * (IT)blockDim.x + threadIdx.x; t < total; t += (IT)gridDim.x * blockDim.x) {
    const int cg = (int)(t % CG);
    IT pix = t / CG;
    const int q = (int)(pix % g.Q);
    pix /= g.Q;
    const int p = (int)(pix % g.P);
    const int n = (int)(pix / g.P);
    const int h0 = p * 2 - g.ph, w0 = q * 2 - g.pw;
    // the window's centre is inside the image for any pad ≤ 1 and P, Q from the usual formulas;
    // clamp it anyway so a masked tap never addresses outside the tensor
    const int hc = min(max(h0 + 1, 0), g.H - 1), wc = min(max(w0 + 1, 0), g.W - 1);
    float v[9][8];
    bool ok[9];
#pragma unroll
    for (int i = 0; i < 3; ++i)
#pragma unroll
      for (int j = 0; j < 3; ++j) {
        const int h = h0 + i, w = w0 + j;
        ok[3 * i + j] = (unsigned)h < (unsigned)g.H && (unsigned)w < (unsigned)g.W;
        const int hh = ok[3 * i + j] ? h : hc, ww = ok[3 * i + j] ? w : wc;
        pld8(x + (((size_t)n * g.H + hh) * g.W + ww) * g.C + cg * 8, v[3 * i + j]);
      }
    float best[8];
    int arg[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) { best[e] = -INFINITY; arg[e] = 0; }
#pragma unroll
    for (int k = 0; k < 9; ++k)
#pragma unroll
      for (int e = 0; e < 8; ++e)
        if (ok[k] && (v[k][e] > best[e] || v[k][e] != v[k][e])) {  // NaN propagates like torch
          best[e] = v[k][e];
          arg[e] = k;
        }
    const size_t o = (((size_t)n * g.P + p) * g.Q + q) * g.C + cg * 8;
    pst8(y + o, best);
    if (!idx) continue;
    uint32_t lo = 0, hi = 0;
#pragma unroll
    for (int e = 0; e < 4; ++e) lo |= (uint32_t)(arg[e] & 0xFF) << (8 * e);
#pragma unroll
    for (int e = 0; e < 4; ++e) hi |= (uint32_t)(arg[4 + e] & 0xFF) << (8 * e);
    *reinterpret_cast<uint2*>(idx + o) = make_uint2(lo, hi);
  }
}

template <typename IT, typename T = bf16_t>
__global__ void __launch_bounds__(256) k_maxpool_bwd(const T* __restrict__ gy, const int8_t* __restrict__ idx,
                                                     T* __restrict__ gx, PoolGeom g) {
  const int CG = g.C >> 3;
  const IT total = (IT)g.N * g.H * g.W * CG;
  for (IT t = blockIdx.x * (IT)blockDim.x + threadIdx.x; t < total; t += (IT)gridDim.x * blockDim.x) {
    const int cg = (int)(t % CG);
    IT pix = t / CG;
    const int w = (int)(pix % g.W);
    pix /= g.W;
    const int h = (int)(pix % g.H);
    const int n = (int)(pix / g.H);
    float acc[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) acc[e] = 0.f;
    // output rows p with p·sh − ph ≤ h ≤ p·sh − ph + kh − 1
    const int hp = h + g.ph, wp = w + g.pw;
    int p_lo = hp - g.kh + 1;
    p_lo = p_lo <= 0 ? 0 : (p_lo + g.sh - 1) / g.sh;
    int p_hi = hp / g.sh;
    if (p_hi > g.P - 1) p_hi = g.P - 1;
    int q_lo = wp - g.kw + 1;
    q_lo = q_lo <= 0 ? 0 : (q_lo + g.sw - 1) / g.sw;
    int q_hi = wp / g.sw;
    if (q_hi > g.Q - 1) q_hi = g.Q - 1;
    for (int p = p_lo; p <= p_hi; ++p) {
      const int i = hp - p * g.sh;
      for (int q = q_lo; q <= q_hi; ++q) {
        const int j = wp - q * g.sw;
        const int8_t me = (int8_t)(i * g.kw + j);
        const size_t o = (((size_t)n * g.P + p) * g.Q + q) * g.C + cg * 8;
        const uint2 a = *reinterpret_cast<const uint2*>(idx + o);
        float gv[8];
        pld8(gy + o, gv);
        const uint32_t aw[2] = {a.x, a.y};
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const int8_t ae = (int8_t)((aw[e >> 2] >> (8 * (e & 3))) & 0xFF);
          if (ae == me) acc[e] += gv[e];
        }
      }
    }
    pst8(gx + (((size_t)n * g.H + h) * g.W + w) * g.C + cg * 8, acc);
  }
}

// 3×3 / stride-2 backward: an input pixel lies in at most 2 × 2 windows; all of their argmax and
// gradient chunks are requested before the first is used (masked, address-clamped when absent).
template <typename IT, typename T = bf16_t>
__global__ void __launch_bounds__(256) k_maxpool_bwd_k3s2(const T* __restrict__ gy, const int8_t* __restrict__ idx,
                                                          T* __restrict__ gx, PoolGeom g) {
  const int CG = g.C >> 3;
  const IT total = (IT)g.N * g.H * g.W * CG;
  for (IT t = blockIdx.x * (IT)blockDim.x + threadIdx.x; t < total; t += (IT)gridDim.x * blockDim.x) {
    const int cg = (int)(t % CG);
    IT pix = t / CG;
    const int w = (int)(pix % g.W);
    pix /= g.W;
    const int h = (int)(pix % g.H);
    const int n = (int)(pix / g.H);
    const int hp = h + g.ph, wp = w + g.pw;
    // windows p with 2p ≤ hp ≤ 2p + 2: p ∈ {hp/2 − 1, hp/2} (clipped to [0, P))
    const int pa = hp / 2 - 1, qa = wp / 2 - 1;
    uint2 a[4];
    float gv[4][8];
    bool ok[4];
    int8_t me[4];
#pragma unroll
    for (int u = 0; u < 2; ++u)
#pragma unroll
      for (int v2 = 0; v2 < 2; ++v2) {
        const int p = pa + u, q = qa + v2, k = 2 * u + v2;
        const int i = hp - 2 * p, j = wp - 2 * q;
        ok[k] = p >= 0 && p < g.P && q >= 0 && q < g.Q && i <= 2 && j <= 2;
        me[k] = (int8_t)(i * 3 + j);
        const int pp = ok[k] ? p : 0, qq = ok[k] ? q : 0;
        const size_t o = (((size_t)n * g.P + pp) * g.Q + qq) * g.C + cg * 8;
        a[k] = *reinterpret_cast<const uint2*>(idx + o);
        pld8(gy + o, gv[k]);
      }
    float acc[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) acc[e] = 0.f;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const uint32_t aw[2] = {a[k].x, a[k].y};
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const int8_t ae = (int8_t)((aw[e >> 2] >> (8 * (e & 3))) & 0xFF);
        if (ok[k] && ae == me[k]) acc[e] += gv[k][e];
      }
    }
    pst8(gx + (((size_t)n * g.H + h) * g.W + w) * g.C + cg * 8, acc);
  }
}

// Channel counts that are not a multiple of 8 (LeNet's 6 / 12 maps): one thread per element, same
// int8 window-offset argmax and gather backward as the vector kernels above.
__device__ __forceinline__ float pld1(const bf16_t* p) { return bf2f(*p); }
__device__ __forceinline__ float pld1(const float* p) { return *p; }
__device__ __forceinline__ void pst1(bf16_t* p, float v) { *p = f2bf(v); }
__device__ __forceinline__ void pst1(float* p, float v) { *p = v; }

template <typename T = bf16_t>
__global__ void __launch_bounds__(256) k_maxpool_fwd_c1(const T* __restrict__ x, T* __restrict__ y,
                                                        int8_t* __restrict__ idx, PoolGeom g, long long total) {
  for (long long t = blockIdx.x * (long long)blockDim.x + threadIdx.x; t < total; t += (long long)gridDim.x * blockDim.x) {
    const int c = (int)(t % g.C);
    long long pix = t / g.C;
    const int q = (int)(pix % g.Q);
    pix /= g.Q;
    const int p = (int)(pix % g.P);
    const int n = (int)(pix / g.P);
    float best = -INFINITY;
    int arg = 0;
    const int h0 = p * g.sh - g.ph, w0 = q * g.sw - g.pw;
    for (int i = 0; i < g.kh; ++i) {
      const int h = h0 + i;
      if ((unsigned)h >= (unsigned)g.H) continue;
      for (int j = 0; j < g.kw; ++j) {
        const int w = w0 + j;
        if ((unsigned)w >= (unsigned)g.W) continue;
        const float v = pld1(x + (((size_t)n * g.H + h) * g.W + w) * g.C + c);
        if (v > best || v != v) {
          best = v;
          arg = i * g.kw + j;
        }
      }
    }
    pst1(y + t, best);
    if (idx) idx[t] = (int8_t)arg;
  }
}

// Inference max-pool (no argmax): a thread produces MP_ROWS vertically adjacent outputs of one
// 8-channel chunk and walks the union of their input rows once — each input row's kw-wide maximum
// is computed once and folded into every output whose window covers it (a 3×3 stride-1 pool loads
// 6 rows for 4 outputs instead of 12).
constexpr int MP_ROWS = 4;

// IDX: the flat thread index type — 32-bit whenever the index space fits (the three index
// divisions per output chunk were 64-bit before: ~4× the integer instructions of the 32-bit form,
// and this kernel was 21 % of Inception-v1 inference, profiles/r2_cfg_inception_v4_profile.txt)
template <typename IDX>
__global__ void __launch_bounds__(256) k_maxpool_fwd_rows(const bf16_t* __restrict__ x, bf16_t* __restrict__ y,
                                                          PoolGeom g) {
  const IDX CG = (IDX)(g.C >> 3);
  const IDX PB = (IDX)((g.P + MP_ROWS - 1) / MP_ROWS);
  const IDX Q = (IDX)g.Q;
  const IDX total = (IDX)g.N * PB * Q * CG;
  for (IDX t = (IDX)blockIdx.x * 256 + threadIdx.x; t < total; t += (IDX)gridDim.x * 256) {
    IDX pix = t / CG;
    const int cg = (int)(t - pix * CG);
    IDX pq = pix / Q;
    const int q = (int)(pix - pq * Q);
    const IDX nn = pq / PB;
    const int pb = (int)(pq - nn * PB);
    const int n = (int)nn;
    const int p0 = pb * MP_ROWS;
    const int np = min(MP_ROWS, g.P - p0);
    float best[MP_ROWS][8];
#pragma unroll
    for (int j = 0; j < MP_ROWS; ++j)
#pragma unroll
      for (int e = 0; e < 8; ++e) best[j][e] = -INFINITY;
    const int w0 = q * g.sw - g.pw;
    const int hlo = p0 * g.sh - g.ph, hhi = (p0 + np - 1) * g.sh - g.ph + g.kh;  // [hlo, hhi)
    for (int h = max(hlo, 0); h < min(hhi, g.H); ++h) {
      float rm[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) rm[e] = -INFINITY;
      for (int j = 0; j < g.kw; ++j) {
        const int w = w0 + j;
        if ((unsigned)w >= (unsigned)g.W) continue;
        float v[8];
        load8(x + (((size_t)n * g.H + h) * g.W + w) * g.C + cg * 8, v);
#pragma unroll
        for (int e = 0; e < 8; ++e) rm[e] = (v[e] > rm[e] || v[e] != v[e]) ? v[e] : rm[e];
      }
#pragma unroll
      for (int j = 0; j < MP_ROWS; ++j) {
        const int top = (p0 + j) * g.sh - g.ph;
        if (j < np && h >= top && h < top + g.kh) {
#pragma unroll
          for (int e = 0; e < 8; ++e) best[j][e] = (rm[e] > best[j][e] || rm[e] != rm[e]) ? rm[e] : best[j][e];
        }
      }
    }
#pragma unroll
    for (int j = 0; j < MP_ROWS; ++j)
      if (j < np) store8(y + (((size_t)n * g.P + p0 + j) * g.Q + q) * g.C + cg * 8, best[j]);
  }
}

template <typename T = bf16_t>
__global__ void __launch_bounds__(256) k_maxpool_bwd_c1(const T* __restrict__ gy, const int8_t* __restrict__ idx,
                                                        T* __restrict__ gx, PoolGeom g, long long total) {
  for (long long t = blockIdx.x * (long long)blockDim.x + threadIdx.x; t < total; t += (long long)gridDim.x * blockDim.x) {
    const int c = (int)(t % g.C);
    long long pix = t / g.C;
    const int w = (int)(pix % g.W);
    pix /= g.W;
    const int h = (int)(pix % g.H);
    const int n = (int)(pix / g.H);
    const int hp = h + g.ph, wp = w + g.pw;
    int p_lo = hp - g.kh + 1;
    p_lo = p_lo <= 0 ? 0 : (p_lo + g.sh - 1) / g.sh;
    const int p_hi = min(hp / g.sh, g.P - 1);
    int q_lo = wp - g.kw + 1;
    q_lo = q_lo <= 0 ? 0 : (q_lo + g.sw - 1) / g.sw;
    const int q_hi = min(wp / g.sw, g.Q - 1);
    float acc = 0.f;
    for (int p = p_lo; p <= p_hi; ++p)
      for (int q = q_lo; q <= q_hi; ++q) {
        const size_t o = (((size_t)n * g.P + p) * g.Q + q) * g.C + c;
        if (idx[o] == (int8_t)((hp - p * g.sh) * g.kw + (wp - q * g.sw))) acc += pld1(gy + o);
      }
    pst1(gx + t, acc);
  }
}

static PoolGeom make_geom(int N, int H, int W, int C, int P, int Q, int kh, int kw, int sh, int sw, int ph, int pw) {
  PoolGeom g;
  g.N = N; g.H = H; g.W = W; g.C = C; g.P = P; g.Q = Q;
  g.kh = kh; g.kw = kw; g.sh = sh; g.sw = sw; g.ph = ph; g.pw = pw;
  return g;
}

BIGDL_EXPORT int bigdl_maxpool_fwd(const void* x, void* y, void* idx, int N, int H, int W, int C, int P, int Q, int kh,
                                   int kw, int sh, int sw, int ph, int pw, hipStream_t s) {
  if (kh * kw > 127 || N <= 0 || P <= 0 || Q <= 0 || C <= 0) return (int)hipErrorInvalidValue;
  PoolGeom g = make_geom(N, H, W, C, P, Q, kh, kw, sh, sw, ph, pw);
  if (C % 8) {
    const long long te = (long long)N * P * Q * C;
    hipLaunchKernelGGL(k_maxpool_fwd_c1<bf16_t>, dim3(bigdl_grid(te, 256, 16384)), dim3(256), 0, s, (const bf16_t*)x, (bf16_t*)y,
                       (int8_t*)idx, g, te);
    BIGDL_CHECK_LAUNCH();
  }
  const bool k3s2 = kh == 3 && kw == 3 && sh == 2 && sw == 2 && ph <= 1 && pw <= 1;
  if (!idx && k3s2 && (long long)N * P * Q * (C / 8) < 0x7fffffffLL) {
    // inference 3x3 / stride-2 pools (the Inception / ResNet stems): every window load in flight
    // (the row-sharing kernel below streamed the 112² Inception pool at ~2 TB/s)
    const long long total = (long long)N * P * Q * (C / 8);
    hipLaunchKernelGGL(k_maxpool_fwd_k3s2<uint32_t>, dim3(bigdl_grid(total, 256, 16384)), dim3(256), 0, s,
                       (const bf16_t*)x, (bf16_t*)y, (int8_t*)nullptr, g);
    BIGDL_CHECK_LAUNCH();
  }
  if (!idx) {
    const long long rows = (long long)N * ((P + MP_ROWS - 1) / MP_ROWS) * Q * (C / 8);
    if (rows < 0x7fffffffLL - 65536LL * 256)
      hipLaunchKernelGGL(k_maxpool_fwd_rows<uint32_t>, dim3(bigdl_grid(rows, 256, 16384)), dim3(256), 0, s,
                         (const bf16_t*)x, (bf16_t*)y, g);
    else
      hipLaunchKernelGGL(k_maxpool_fwd_rows<long long>, dim3(bigdl_grid(rows, 256, 16384)), dim3(256), 0, s,
                         (const bf16_t*)x, (bf16_t*)y, g);
    BIGDL_CHECK_LAUNCH();
  }
  const long long total = (long long)N * P * Q * (C / 8);
  const int grid = bigdl_grid(total, 256, 16384);
  if (total < 0x7fffffffLL) {
    if (k3s2) hipLaunchKernelGGL(k_maxpool_fwd_k3s2<uint32_t>, dim3(grid), dim3(256), 0, s, (const bf16_t*)x, (bf16_t*)y, (int8_t*)idx, g);
    else hipLaunchKernelGGL(k_maxpool_fwd<uint32_t>, dim3(grid), dim3(256), 0, s, (const bf16_t*)x, (bf16_t*)y, (int8_t*)idx, g);
  } else {
    hipLaunchKernelGGL(k_maxpool_fwd<long long>, dim3(grid), dim3(256), 0, s, (const bf16_t*)x, (bf16_t*)y, (int8_t*)idx, g);
  }
  BIGDL_CHECK_LAUNCH();
}

BIGDL_EXPORT int bigdl_maxpool_bwd(const void* gy, const void* idx, void* gx, int N, int H, int W, int C, int P, int Q,
                                   int kh, int kw, int sh, int sw, int ph, int pw, hipStream_t s) {
  if (kh * kw > 127 || N <= 0 || C <= 0) return (int)hipErrorInvalidValue;
  PoolGeom g = make_geom(N, H, W, C, P, Q, kh, kw, sh, sw, ph, pw);
  if (C % 8) {
    const long long te = (long long)N * H * W * C;
    hipLaunchKernelGGL(k_maxpool_bwd_c1<bf16_t>, dim3(bigdl_grid(te, 256, 16384)), dim3(256), 0, s, (const bf16_t*)gy,
                       (const int8_t*)idx, (bf16_t*)gx, g, te);
    BIGDL_CHECK_LAUNCH();
  }
  const long long total = (long long)N * H * W * (C / 8);
  const int grid = bigdl_grid(total, 256, 16384);
  const bool k3s2 = kh == 3 && kw == 3 && sh == 2 && sw == 2 && ph <= 1 && pw <= 1;
  if (total < 0x7fffffffLL && k3s2)
    hipLaunchKernelGGL(k_maxpool_bwd_k3s2<uint32_t>, dim3(grid), dim3(256), 0, s, (const bf16_t*)gy, (const int8_t*)idx,
                       (bf16_t*)gx, g);
  else if (total < 0x7fffffffLL)
    hipLaunchKernelGGL(k_maxpool_bwd<uint32_t>, dim3(grid), dim3(256), 0, s, (const bf16_t*)gy, (const int8_t*)idx,
                       (bf16_t*)gx, g);
  else
    hipLaunchKernelGGL(k_maxpool_bwd<long long>, dim3(grid), dim3(256), 0, s, (const bf16_t*)gy, (const int8_t*)idx,
                       (bf16_t*)gx, g);
  BIGDL_CHECK_LAUNCH();
}

// ------------------------------------------------------------------------------------------------
// K11: average pooling, NHWC bf16 (SpatialAveragePooling.updateOutput / updateGradInput,
// DL/nn/SpatialAveragePooling.scala:115-700).  Divisor semantics are torch's avg_pool2d ones (the
// reference path): count_include_pad counts the padded window clipped to the padded extent
// (ceil-mode overhang excluded); otherwise the in-image tap count; `divisor` > 0 overrides both.
// Forward: one thread per (output pixel, 8 channels).  Backward: a gather — each input pixel sums
// gy / count over the windows that cover it, so gx is written once with no zero-fill or atomics.
// ------------------------------------------------------------------------------------------------
__device__ __forceinline__ float avg_count(const PoolGeom& g, int p, int q, int cip, int divisor) {
  if (divisor > 0) return (float)divisor;
  int hs = p * g.sh - g.ph, ws = q * g.sw - g.pw;
  int he = min(hs + g.kh, g.H + g.ph), we = min(ws + g.kw, g.W + g.pw);
  if (cip) return (float)((he - hs) * (we - ws));
  hs = max(hs, 0); ws = max(ws, 0);
  he = min(he, g.H); we = min(we, g.W);
  return (float)((he - hs) * (we - ws));
}

template <typename IT, typename T = bf16_t>
__global__ void __launch_bounds__(256) k_avgpool_fwd(const T* __restrict__ x, T* __restrict__ y, PoolGeom g,
                                                     int cip, int divisor) {
  const int CG = g.C >> 3;
  const IT total = (IT)g.N * g.P * g.Q * CG;
  for (IT t = blockIdx.x * (IT)blockDim.x + threadIdx.x; t < total; t += (IT)gridDim.x * blockDim.x) {
    const int cg = (int)(t % CG);
    IT pix = t / CG;
    const int q = (int)(pix % g.Q);
    pix /= g.Q;
    const int p = (int)(pix % g.P);
    const int n = (int)(pix / g.P);
    float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    const int h0 = p * g.sh - g.ph, w0 = q * g.sw - g.pw;
    const int hb = max(h0, 0), he = min(h0 + g.kh, g.H), wb = max(w0, 0), we = min(w0 + g.kw, g.W);
    for (int h = hb; h < he; ++h)
      for (int w = wb; w < we; ++w) {
        float v[8];
        pld8(x + (((size_t)n * g.H + h) * g.W + w) * g.C + cg * 8, v);
#pragma unroll
        for (int e = 0; e < 8; ++e) acc[e] += v[e];
      }
    const float inv = 1.f / fmaxf(avg_count(g, p, q, cip, divisor), 1.f);
#pragma unroll
    for (int e = 0; e < 8; ++e) acc[e] *= inv;
    pst8(y + (((size_t)n * g.P + p) * g.Q + q) * g.C + cg * 8, acc);
  }
}

template <typename IT, typename T = bf16_t>
__global__ void __launch_bounds__(256) k_avgpool_bwd(const T* __restrict__ gy, T* __restrict__ gx, PoolGeom g,
                                                     int cip, int divisor) {
  const int CG = g.C >> 3;
  const IT total = (IT)g.N * g.H * g.W * CG;
  for (IT t = blockIdx.x * (IT)blockDim.x + threadIdx.x; t < total; t += (IT)gridDim.x * blockDim.x) {
    const int cg = (int)(t % CG);
    IT pix = t / CG;
    const int w = (int)(pix % g.W);
    pix /= g.W;
    const int h = (int)(pix % g.H);
    const int n = (int)(pix / g.H);
    // output windows p with p·sh − ph ≤ h < p·sh − ph + kh
    const int hp = h + g.ph, wp = w + g.pw;
    const int p_lo = hp < g.kh ? 0 : (hp - g.kh) / g.sh + 1, p_hi = min(hp / g.sh, g.P - 1);
    const int q_lo = wp < g.kw ? 0 : (wp - g.kw) / g.sw + 1, q_hi = min(wp / g.sw, g.Q - 1);
    float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    for (int p = p_lo; p <= p_hi; ++p)
      for (int q = q_lo; q <= q_hi; ++q) {
        float v[8];
        pld8(gy + (((size_t)n * g.P + p) * g.Q + q) * g.C + cg * 8, v);
        const float inv = 1.f / fmaxf(avg_count(g, p, q, cip, divisor), 1.f);
#pragma unroll
        for (int e = 0; e < 8; ++e) acc[e] = fmaf(v[e], inv, acc[e]);
      }
    pst8(gx + (((size_t)n * g.H + h) * g.W + w) * g.C + cg * 8, acc);
  }
}

BIGDL_EXPORT int bigdl_avgpool_fwd(const void* x, void* y, int N, int H, int W, int C, int P, int Q, int kh, int kw,
                                   int sh, int sw, int ph, int pw, int count_include_pad, int divisor, hipStream_t s) {
  if (C % 8 || N <= 0 || P <= 0 || Q <= 0 || kh <= 0 || kw <= 0 || sh <= 0 || sw <= 0) return (int)hipErrorInvalidValue;
  if (2 * ph > kh || 2 * pw > kw) return (int)hipErrorInvalidValue;
  if (((uintptr_t)x & 15) || ((uintptr_t)y & 15)) return (int)hipErrorInvalidValue;
  PoolGeom g = make_geom(N, H, W, C, P, Q, kh, kw, sh, sw, ph, pw);
  const long long total = (long long)N * P * Q * (C / 8);
  const int grid = bigdl_grid(total, 256, 16384);
  if (total < 0x7fffffffLL)
    hipLaunchKernelGGL(k_avgpool_fwd<uint32_t>, dim3(grid), dim3(256), 0, s, (const bf16_t*)x, (bf16_t*)y, g,
                       count_include_pad, divisor);
  else
    hipLaunchKernelGGL(k_avgpool_fwd<long long>, dim3(grid), dim3(256), 0, s, (const bf16_t*)x, (bf16_t*)y, g,
                       count_include_pad, divisor);
  BIGDL_CHECK_LAUNCH();
}

BIGDL_EXPORT int bigdl_avgpool_bwd(const void* gy, void* gx, int N, int H, int W, int C, int P, int Q, int kh, int kw,
                                   int sh, int sw, int ph, int pw, int count_include_pad, int divisor, hipStream_t s) {
  if (C % 8 || N <= 0 || P <= 0 || Q <= 0 || kh <= 0 || kw <= 0 || sh <= 0 || sw <= 0) return (int)hipErrorInvalidValue;
  if (2 * ph > kh || 2 * pw > kw) return (int)hipErrorInvalidValue;
  if (((uintptr_t)gy & 15) || ((uintptr_t)gx & 15)) return (int)hipErrorInvalidValue;
  PoolGeom g = make_geom(N, H, W, C, P, Q, kh, kw, sh, sw, ph, pw);
  const long long total = (long long)N * H * W * (C / 8);
  const int grid = bigdl_grid(total, 256, 16384);
  if (total < 0x7fffffffLL)
    hipLaunchKernelGGL(k_avgpool_bwd<uint32_t>, dim3(grid), dim3(256), 0, s, (const bf16_t*)gy, (bf16_t*)gx, g,
                       count_include_pad, divisor);
  else
    hipLaunchKernelGGL(k_avgpool_bwd<long long>, dim3(grid), dim3(256), 0, s, (const bf16_t*)gy, (bf16_t*)gx, g,
                       count_include_pad, divisor);
  BIGDL_CHECK_LAUNCH();
}

// ---- fp32 NHWC (bigdl.compute.dtype=fp32): same kernels, fp32 elements; 16-B aligned when C % 8 == 0,
// the per-element kernels otherwise (LeNet's 6 / 12 maps) ----
static bool pool32_ok(const void* a, const void* b, int C) {
  return C % 8 == 0 && ((uintptr_t)a & 15) == 0 && ((uintptr_t)b & 15) == 0;
}

BIGDL_EXPORT int bigdl_maxpool32_fwd(const float* x, float* y, void* idx, int N, int H, int W, int C, int P, int Q,
                                     int kh, int kw, int sh, int sw, int ph, int pw, hipStream_t s) {
  if (kh * kw > 127 || N <= 0 || P <= 0 || Q <= 0 || C <= 0) return (int)hipErrorInvalidValue;
  PoolGeom g = make_geom(N, H, W, C, P, Q, kh, kw, sh, sw, ph, pw);
  if (!pool32_ok(x, y, C)) {
    const long long te = (long long)N * P * Q * C;
    hipLaunchKernelGGL((k_maxpool_fwd_c1<float>), dim3(bigdl_grid(te, 256, 16384)), dim3(256), 0, s, x, y,
                       (int8_t*)idx, g, te);
    BIGDL_CHECK_LAUNCH();
  }
  const long long total = (long long)N * P * Q * (C / 8);
  const int grid = bigdl_grid(total, 256, 16384);
  const bool k3s2 = kh == 3 && kw == 3 && sh == 2 && sw == 2 && ph <= 1 && pw <= 1;
  if (total < 0x7fffffffLL && k3s2)
    hipLaunchKernelGGL((k_maxpool_fwd_k3s2<uint32_t, float>), dim3(grid), dim3(256), 0, s, x, y, (int8_t*)idx, g);
  else if (total < 0x7fffffffLL)
    hipLaunchKernelGGL((k_maxpool_fwd<uint32_t, float>), dim3(grid), dim3(256), 0, s, x, y, (int8_t*)idx, g);
  else
    hipLaunchKernelGGL((k_maxpool_fwd<long long, float>), dim3(grid), dim3(256), 0, s, x, y, (int8_t*)idx, g);
  BIGDL_CHECK_LAUNCH();
}

BIGDL_EXPORT int bigdl_maxpool32_bwd(const float* gy, const void* idx, float* gx, int N, int H, int W, int C, int P,
                                     int Q, int kh, int kw, int sh, int sw, int ph, int pw, hipStream_t s) {
  if (kh * kw > 127 || N <= 0 || C <= 0 || !idx) return (int)hipErrorInvalidValue;
  PoolGeom g = make_geom(N, H, W, C, P, Q, kh, kw, sh, sw, ph, pw);
  if (!pool32_ok(gy, gx, C)) {
    const long long te = (long long)N * H * W * C;
    hipLaunchKernelGGL((k_maxpool_bwd_c1<float>), dim3(bigdl_grid(te, 256, 16384)), dim3(256), 0, s, gy,
                       (const int8_t*)idx, gx, g, te);
    BIGDL_CHECK_LAUNCH();
  }
  const long long total = (long long)N * H * W * (C / 8);
  const int grid = bigdl_grid(total, 256, 16384);
  const bool k3s2 = kh == 3 && kw == 3 && sh == 2 && sw == 2 && ph <= 1 && pw <= 1;
  if (total < 0x7fffffffLL && k3s2)
    hipLaunchKernelGGL((k_maxpool_bwd_k3s2<uint32_t, float>), dim3(grid), dim3(256), 0, s, gy, (const int8_t*)idx, gx, g);
  else if (total < 0x7fffffffLL)
    hipLaunchKernelGGL((k_maxpool_bwd<uint32_t, float>), dim3(grid), dim3(256), 0, s, gy, (const int8_t*)idx, gx, g);
  else
    hipLaunchKernelGGL((k_maxpool_bwd<long long, float>), dim3(grid), dim3(256), 0, s, gy, (const int8_t*)idx, gx, g);
  BIGDL_CHECK_LAUNCH();
}

BIGDL_EXPORT int bigdl_avgpool32_fwd(const float* x, float* y, int N, int H, int W, int C, int P, int Q, int kh, int kw,
                                     int sh, int sw, int ph, int pw, int count_include_pad, int divisor, hipStream_t s) {
  if (N <= 0 || P <= 0 || Q <= 0 || kh <= 0 || kw <= 0 || sh <= 0 || sw <= 0 || !pool32_ok(x, y, C))
    return (int)hipErrorInvalidValue;
  if (2 * ph > kh || 2 * pw > kw) return (int)hipErrorInvalidValue;
  PoolGeom g = make_geom(N, H, W, C, P, Q, kh, kw, sh, sw, ph, pw);
  const long long total = (long long)N * P * Q * (C / 8);
  const int grid = bigdl_grid(total, 256, 16384);
  if (total < 0x7fffffffLL)
    hipLaunchKernelGGL((k_avgpool_fwd<uint32_t, float>), dim3(grid), dim3(256), 0, s, x, y, g, count_include_pad, divisor);
  else
    hipLaunchKernelGGL((k_avgpool_fwd<long long, float>), dim3(grid), dim3(256), 0, s, x, y, g, count_include_pad, divisor);
  BIGDL_CHECK_LAUNCH();
}

BIGDL_EXPORT int bigdl_avgpool32_bwd(const float* gy, float* gx, int N, int H, int W, int C, int P, int Q, int kh, int kw,
                                     int sh, int sw, int ph, int pw, int count_include_pad, int divisor, hipStream_t s) {
  if (N <= 0 || P <= 0 || Q <= 0 || kh <= 0 || kw <= 0 || sh <= 0 || sw <= 0 || !pool32_ok(gy, gx, C))
    return (int)hipErrorInvalidValue;
  if (2 * ph > kh || 2 * pw > kw) return (int)hipErrorInvalidValue;
  PoolGeom g = make_geom(N, H, W, C, P, Q, kh, kw, sh, sw, ph, pw);
  const long long total = (long long)N * H * W * (C / 8);
  const int grid = bigdl_grid(total, 256, 16384);
  if (total < 0x7fffffffLL)
    hipLaunchKernelGGL((k_avgpool_bwd<uint32_t, float>), dim3(grid), dim3(256), 0, s, gy, gx, g, count_include_pad, divisor);
  else
    hipLaunchKernelGGL((k_avgpool_bwd<long long, float>), dim3(grid), dim3(256), 0, s, gy, gx, g, count_include_pad, divisor);
  BIGDL_CHECK_LAUNCH();
}
