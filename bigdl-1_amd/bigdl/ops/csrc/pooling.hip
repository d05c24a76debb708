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

template <typename IT>
__global__ void __launch_bounds__(256) k_maxpool_fwd(const bf16_t* __restrict__ x, bf16_t* __restrict__ y,
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
        load8(x + (((size_t)n * g.H + h) * g.W + w) * g.C + cg * 8, v);
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
    store8(y + o, best);
    uint32_t lo = 0, hi = 0;
#pragma unroll
    for (int e = 0; e < 4; ++e) lo |= (uint32_t)(arg[e] & 0xFF) << (8 * e);
#pragma unroll
    for (int e = 0; e < 4; ++e) hi |= (uint32_t)(arg[4 + e] & 0xFF) << (8 * e);
    *reinterpret_cast<uint2*>(idx + o) = make_uint2(lo, hi);
  }
}

template <typename IT>
__global__ void __launch_bounds__(256) k_maxpool_bwd(const bf16_t* __restrict__ gy, const int8_t* __restrict__ idx,
                                                     bf16_t* __restrict__ gx, PoolGeom g) {
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
        load8(gy + o, gv);
        const uint32_t aw[2] = {a.x, a.y};
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const int8_t ae = (int8_t)((aw[e >> 2] >> (8 * (e & 3))) & 0xFF);
          if (ae == me) acc[e] += gv[e];
        }
      }
    }
    store8(gx + (((size_t)n * g.H + h) * g.W + w) * g.C + cg * 8, acc);
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
  if (C % 8 || kh * kw > 127 || N <= 0 || P <= 0 || Q <= 0) return (int)hipErrorInvalidValue;
  PoolGeom g = make_geom(N, H, W, C, P, Q, kh, kw, sh, sw, ph, pw);
  const long long total = (long long)N * P * Q * (C / 8);
  const int grid = bigdl_grid(total, 256, 16384);
  if (total < 0x7fffffffLL)
    hipLaunchKernelGGL(k_maxpool_fwd<uint32_t>, dim3(grid), dim3(256), 0, s, (const bf16_t*)x, (bf16_t*)y, (int8_t*)idx, g);
  else
    hipLaunchKernelGGL(k_maxpool_fwd<long long>, dim3(grid), dim3(256), 0, s, (const bf16_t*)x, (bf16_t*)y, (int8_t*)idx, g);
  BIGDL_CHECK_LAUNCH();
}

BIGDL_EXPORT int bigdl_maxpool_bwd(const void* gy, const void* idx, void* gx, int N, int H, int W, int C, int P, int Q,
                                   int kh, int kw, int sh, int sw, int ph, int pw, hipStream_t s) {
  if (C % 8 || kh * kw > 127 || N <= 0) return (int)hipErrorInvalidValue;
  PoolGeom g = make_geom(N, H, W, C, P, Q, kh, kw, sh, sw, ph, pw);
  const long long total = (long long)N * H * W * (C / 8);
  const int grid = bigdl_grid(total, 256, 16384);
  if (total < 0x7fffffffLL)
    hipLaunchKernelGGL(k_maxpool_bwd<uint32_t>, dim3(grid), dim3(256), 0, s, (const bf16_t*)gy, (const int8_t*)idx,
                       (bf16_t*)gx, g);
  else
    hipLaunchKernelGGL(k_maxpool_bwd<long long>, dim3(grid), dim3(256), 0, s, (const bf16_t*)gy, (const int8_t*)idx,
                       (bf16_t*)gx, g);
  BIGDL_CHECK_LAUNCH();
}
