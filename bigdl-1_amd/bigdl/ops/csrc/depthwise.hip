// Depthwise convolution (groups == C == K; SpatialSeparableConvolution's first stage and TF
// DepthwiseConv2D, reference nn/SpatialSeparableConvolution.scala, nn/ops/DepthwiseConv2D*.scala).
//
// A depthwise conv has no channel reduction, so there is nothing for the matrix cores: it is a
// memory-bound stencil.  NHWC bf16 activations, each thread owns 8 consecutive channels of one
// output pixel (16-B loads / stores), fp32 accumulation, weights pre-transposed to [R][S][C] so a
// tap's 8 channels are one 32-B fp32 load.  Backward-data is the same stencil walked from the input
// side (stride-aware); backward-weight reduces over pixels per (channel chunk, tap) in registers and
// adds each block's partial with one no-return fp32 atomic per weight (deterministic mode: one
// block per channel chunk).
#include "common.h"

struct DwGeom {
  int N, H, W, C, P, Q, R, S, sh, sw, ph, pw, dh, dw;
};

__global__ void __launch_bounds__(256) k_dw_fwd(const bf16_t* __restrict__ x, const float* __restrict__ wt,
                                                const float* __restrict__ bias, bf16_t* __restrict__ y, DwGeom g,
                                                int relu) {
  const int CG = g.C / 8;
  const long long total = (long long)g.N * g.P * g.Q * CG;
  for (long long i = blockIdx.x * 256ll + threadIdx.x; i < total; i += (long long)gridDim.x * 256) {
    const int cg = (int)(i % CG);
    long long pix = i / CG;
    const int q = (int)(pix % g.Q);
    pix /= g.Q;
    const int p = (int)(pix % g.P);
    const int n = (int)(pix / g.P);
    float acc[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) acc[e] = bias ? bias[cg * 8 + e] : 0.f;
    for (int r = 0; r < g.R; ++r) {
      const int h = p * g.sh - g.ph + r * g.dh;
      if ((unsigned)h >= (unsigned)g.H) continue;
      for (int s = 0; s < g.S; ++s) {
        const int w = q * g.sw - g.pw + s * g.dw;
        if ((unsigned)w >= (unsigned)g.W) continue;
        float v[8];
        load8(x + (((size_t)n * g.H + h) * g.W + w) * g.C + cg * 8, v);
        const float4* wp = reinterpret_cast<const float4*>(wt + ((size_t)(r * g.S + s) * g.C + cg * 8));
        const float4 w0 = wp[0], w1 = wp[1];
        acc[0] = fmaf(v[0], w0.x, acc[0]);
        acc[1] = fmaf(v[1], w0.y, acc[1]);
        acc[2] = fmaf(v[2], w0.z, acc[2]);
        acc[3] = fmaf(v[3], w0.w, acc[3]);
        acc[4] = fmaf(v[4], w1.x, acc[4]);
        acc[5] = fmaf(v[5], w1.y, acc[5]);
        acc[6] = fmaf(v[6], w1.z, acc[6]);
        acc[7] = fmaf(v[7], w1.w, acc[7]);
      }
    }
    if (relu) {
#pragma unroll
      for (int e = 0; e < 8; ++e) acc[e] = fmaxf(acc[e], 0.f);
    }
    store8(y + (((size_t)n * g.P + p) * g.Q + q) * g.C + cg * 8, acc);
  }
}

// gx[n,h,w,c] = Σ_{r,s: (h + ph − r·dh) = p·sh, (w + pw − s·dw) = q·sw} gy[n,p,q,c] · W[r][s][c]
__global__ void __launch_bounds__(256) k_dw_dgrad(const bf16_t* __restrict__ gy, const float* __restrict__ wt,
                                                  bf16_t* __restrict__ gx, DwGeom g) {
  const int CG = g.C / 8;
  const long long total = (long long)g.N * g.H * g.W * CG;
  for (long long i = blockIdx.x * 256ll + threadIdx.x; i < total; i += (long long)gridDim.x * 256) {
    const int cg = (int)(i % CG);
    long long pix = i / CG;
    const int w = (int)(pix % g.W);
    pix /= g.W;
    const int h = (int)(pix % g.H);
    const int n = (int)(pix / g.H);
    float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    for (int r = 0; r < g.R; ++r) {
      const int ph = h + g.ph - r * g.dh;
      if (ph < 0 || ph % g.sh) continue;
      const int p = ph / g.sh;
      if (p >= g.P) continue;
      for (int s = 0; s < g.S; ++s) {
        const int pw = w + g.pw - s * g.dw;
        if (pw < 0 || pw % g.sw) continue;
        const int q = pw / g.sw;
        if (q >= g.Q) continue;
        float v[8];
        load8(gy + (((size_t)n * g.P + p) * g.Q + q) * g.C + cg * 8, v);
        const float4* wp = reinterpret_cast<const float4*>(wt + ((size_t)(r * g.S + s) * g.C + cg * 8));
        const float4 w0 = wp[0], w1 = wp[1];
        acc[0] = fmaf(v[0], w0.x, acc[0]);
        acc[1] = fmaf(v[1], w0.y, acc[1]);
        acc[2] = fmaf(v[2], w0.z, acc[2]);
        acc[3] = fmaf(v[3], w0.w, acc[3]);
        acc[4] = fmaf(v[4], w1.x, acc[4]);
        acc[5] = fmaf(v[5], w1.y, acc[5]);
        acc[6] = fmaf(v[6], w1.z, acc[6]);
        acc[7] = fmaf(v[7], w1.w, acc[7]);
      }
    }
    store8(gx + (((size_t)n * g.H + h) * g.W + w) * g.C + cg * 8, acc);
  }
}

constexpr int DW_MAX_TAPS = 25;  // up to 5×5 filters in the weight-gradient kernel

// gw[r][s][c] += scale · Σ_pixels gy[n,p,q,c] · x[n, p·sh − ph + r·dh, q·sw − pw + s·dw, c]
// block = 256 threads = 32 channel chunks (a warp-contiguous 256-channel strip: lanes of the
// same pixel read consecutive 16-B chunks) × 8 pixel lanes; grid.x = channel strips, grid.y =
// pixel splits.
template <int MAXT>
__global__ void __launch_bounds__(256) k_dw_wgrad(const bf16_t* __restrict__ x, const bf16_t* __restrict__ gy,
                                                  float* __restrict__ gw, DwGeom g, float scale, long long per_split) {
  const int CG = g.C / 8;
  const int cgl = threadIdx.x & 31, pl = threadIdx.x >> 5;
  const int cg = blockIdx.x * 32 + cgl;
  const long long M = (long long)g.N * g.P * g.Q;
  const long long m0 = blockIdx.y * per_split;
  long long m1 = m0 + per_split;
  if (m1 > M) m1 = M;
  const int taps = g.R * g.S;
  float acc[MAXT][8];
#pragma unroll
  for (int t = 0; t < MAXT; ++t)
#pragma unroll
    for (int e = 0; e < 8; ++e) acc[t][e] = 0.f;
  if (cg < CG) {
    for (long long m = m0 + pl; m < m1; m += 8) {
      const int q = (int)(m % g.Q);
      const long long t1 = m / g.Q;
      const int p = (int)(t1 % g.P);
      const int n = (int)(t1 / g.P);
      float gv[8];
      load8(gy + (size_t)m * g.C + cg * 8, gv);
#pragma unroll
      for (int t = 0; t < MAXT; ++t) {
        if (t >= taps) break;
        const int r = t / g.S, s = t - (t / g.S) * g.S;
        const int h = p * g.sh - g.ph + r * g.dh, w = q * g.sw - g.pw + s * g.dw;
        if ((unsigned)h >= (unsigned)g.H || (unsigned)w >= (unsigned)g.W) continue;
        float v[8];
        load8(x + (((size_t)n * g.H + h) * g.W + w) * g.C + cg * 8, v);
#pragma unroll
        for (int e = 0; e < 8; ++e) acc[t][e] = fmaf(gv[e], v[e], acc[t][e]);
      }
    }
  }
  // fold the 8 pixel lanes through LDS, then one atomic per weight element of this block
  __shared__ float red[8][32 * 8 + 4];
#pragma unroll
  for (int t = 0; t < MAXT; ++t) {
    if (t >= taps) break;
#pragma unroll
    for (int e = 0; e < 8; ++e) red[pl][cgl * 8 + e] = acc[t][e];
    __syncthreads();
    const int c = threadIdx.x;  // 256 threads = 32 chunks × 8 channels
    float v = 0.f;
#pragma unroll
    for (int k = 0; k < 8; ++k) v += red[k][c];
    const int ch = blockIdx.x * 256 + c;
    if (ch < g.C) atomicAdd(gw + (size_t)t * g.C + ch, scale * v);
    __syncthreads();
  }
}

static bool dw_geom_ok(const DwGeom& g) {
  return g.N > 0 && g.C > 0 && g.C % 8 == 0 && g.P > 0 && g.Q > 0 && g.R > 0 && g.S > 0 && g.sh > 0 && g.sw > 0 &&
         g.dh > 0 && g.dw > 0;
}

// wt: fp32 [R][S][C]; x/y NHWC bf16, 16-B aligned
BIGDL_EXPORT int bigdl_dw_fwd(const void* x, const float* wt, const float* bias, void* y, int N, int H, int W, int C,
                              int P, int Q, int R, int S, int sh, int sw, int ph, int pw, int dh, int dw, int relu,
                              hipStream_t s) {
  const DwGeom g{N, H, W, C, P, Q, R, S, sh, sw, ph, pw, dh, dw};
  if (!dw_geom_ok(g)) return (int)hipErrorInvalidValue;
  const long long work = (long long)N * P * Q * (C / 8);
  hipLaunchKernelGGL(k_dw_fwd, dim3(bigdl_grid(work, 256, 65536)), dim3(256), 0, s, (const bf16_t*)x, wt, bias,
                     (bf16_t*)y, g, relu);
  BIGDL_CHECK_LAUNCH();
}

BIGDL_EXPORT int bigdl_dw_dgrad(const void* gy, const float* wt, void* gx, int N, int H, int W, int C, int P, int Q,
                                int R, int S, int sh, int sw, int ph, int pw, int dh, int dw, hipStream_t s) {
  const DwGeom g{N, H, W, C, P, Q, R, S, sh, sw, ph, pw, dh, dw};
  if (!dw_geom_ok(g)) return (int)hipErrorInvalidValue;
  const long long work = (long long)N * H * W * (C / 8);
  hipLaunchKernelGGL(k_dw_dgrad, dim3(bigdl_grid(work, 256, 65536)), dim3(256), 0, s, (const bf16_t*)gy, wt,
                     (bf16_t*)gx, g);
  BIGDL_CHECK_LAUNCH();
}

// gw: fp32 [R][S][C], accumulated
BIGDL_EXPORT int bigdl_dw_wgrad(const void* x, const void* gy, float* gw, float scale, int N, int H, int W, int C,
                                int P, int Q, int R, int S, int sh, int sw, int ph, int pw, int dh, int dw,
                                hipStream_t s) {
  const DwGeom g{N, H, W, C, P, Q, R, S, sh, sw, ph, pw, dh, dw};
  if (!dw_geom_ok(g) || R * S > DW_MAX_TAPS) return (int)hipErrorInvalidValue;
  const long long M = (long long)N * P * Q;
  const int strips = (C + 255) / 256;
  int splits = g_bigdl_deterministic ? 1 : (int)((1024 + strips - 1) / strips);
  const long long min_rows = 256;
  if ((long long)splits * min_rows > M) splits = (int)((M + min_rows - 1) / min_rows);
  if (splits < 1) splits = 1;
  if (splits > 65535) splits = 65535;
  const long long per = (M + splits - 1) / splits;
  if (R * S <= 9)
    hipLaunchKernelGGL(k_dw_wgrad<9>, dim3(strips, splits), dim3(256), 0, s, (const bf16_t*)x, (const bf16_t*)gy, gw,
                       g, scale, per);
  else
    hipLaunchKernelGGL(k_dw_wgrad<DW_MAX_TAPS>, dim3(strips, splits), dim3(256), 0, s, (const bf16_t*)x,
                       (const bf16_t*)gy, gw, g, scale, per);
  BIGDL_CHECK_LAUNCH();
}
