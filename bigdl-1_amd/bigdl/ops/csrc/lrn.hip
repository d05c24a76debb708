// K18: cross-channel local response normalisation, NHWC bf16 or fp32 (SpatialCrossMapLRN.updateOutput /
// updateGradInput, DL/nn/SpatialCrossMapLRN.scala:96-200; mkldnn LRN).
//
//   s_c = k + α/size · Σ_{c' ∈ [c-h, c+h]} x_c'²        (odd size = 2h+1, zero outside [0, C))
//   y_c = x_c · s_c^-β
//   gx_c = gy_c · s_c^-β − (2αβ/size) · x_c · Σ_{c' ∈ [c-h, c+h]} gy_c' · x_c' · s_c'^(-β-1)
//
// One thread per (pixel, 8-channel group).  In NHWC a pixel's channels are contiguous, so the
// ±h window of a group lives in the previous, own and next 16-B chunk of the same row: three
// coalesced 16-B loads per thread (the neighbours' chunks are L1/L2 hits for the adjacent lanes),
// no LDS, no cross-lane traffic.  Forward covers h ≤ 8, backward h ≤ 4 (the gradient window of
// a channel reaches 2h); Inception/AlexNet use size 5.  Nothing is saved for backward: s is
// recomputed from x, which costs less HBM traffic than writing and re-reading it.
#include "common.h"

// element access: bf16 (one 16-B load per 8 channels) or fp32 (two; the reference's precision)
__device__ __forceinline__ void ld8(const bf16_t* p, float* o) { load8(p, o); }
__device__ __forceinline__ void ld8(const float* p, float* o) {
  const float4 a = *reinterpret_cast<const float4*>(p), b = *reinterpret_cast<const float4*>(p + 4);
  o[0] = a.x; o[1] = a.y; o[2] = a.z; o[3] = a.w; o[4] = b.x; o[5] = b.y; o[6] = b.z; o[7] = b.w;
}
__device__ __forceinline__ void st8(bf16_t* p, const float* o) { store8(p, o); }
__device__ __forceinline__ void st8(float* p, const float* o) {
  *reinterpret_cast<float4*>(p) = make_float4(o[0], o[1], o[2], o[3]);
  *reinterpret_cast<float4*>(p + 4) = make_float4(o[4], o[5], o[6], o[7]);
}

template <typename T>
__device__ __forceinline__ void load8_or_zero(const T* row, int cg, int CG, float* o) {
  if (cg >= 0 && cg < CG) {
    ld8(row + cg * 8, o);
  } else {
#pragma unroll
    for (int e = 0; e < 8; ++e) o[e] = 0.f;
  }
}

__device__ __forceinline__ float pow_neg(float s, float b) { return exp2f(-b * __log2f(s)); }

// the half-window HH is a template parameter: every register-array index below is then a
// compile-time constant (a runtime index would spill the arrays to scratch)
template <int HH, typename T>
__global__ void __launch_bounds__(256) k_lrn_fwd(const T* __restrict__ x, T* __restrict__ y,
                                                 long long pixels, int C, float alpha_n, float beta, float k) {
  const int CG = C >> 3;
  const long long total = pixels * CG;
  for (long long t = blockIdx.x * (long long)blockDim.x + threadIdx.x; t < total;
       t += (long long)gridDim.x * blockDim.x) {
    const int cg = (int)(t % CG);
    const T* row = x + (t / CG) * C;
    float v[24];
    load8_or_zero(row, cg - 1, CG, v);
    load8_or_zero(row, cg, CG, v + 8);
    load8_or_zero(row, cg + 1, CG, v + 16);
    float sq[24];
#pragma unroll
    for (int i = 0; i < 24; ++i) sq[i] = v[i] * v[i];
    float out[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      float acc = 0.f;
#pragma unroll
      for (int d = -HH; d <= HH; ++d) acc += sq[8 + e + d];
      out[e] = v[8 + e] * pow_neg(k + alpha_n * acc, beta);
    }
    st8(y + (t / CG) * C + cg * 8, out);
  }
}

template <int HH, typename T>
__global__ void __launch_bounds__(256) k_lrn_bwd(const T* __restrict__ x, const T* __restrict__ gy,
                                                 T* __restrict__ gx, long long pixels, int C, float alpha_n,
                                                 float beta, float k) {
  const int CG = C >> 3;
  const long long total = pixels * CG;
  const float coef = 2.f * alpha_n * beta;
  for (long long t = blockIdx.x * (long long)blockDim.x + threadIdx.x; t < total;
       t += (long long)gridDim.x * blockDim.x) {
    const int cg = (int)(t % CG);
    const size_t base = (size_t)(t / CG) * C;
    float v[24], g[24];
    load8_or_zero(x + base, cg - 1, CG, v);
    load8_or_zero(x + base, cg, CG, v + 8);
    load8_or_zero(x + base, cg + 1, CG, v + 16);
    load8_or_zero(gy + base, cg - 1, CG, g);
    load8_or_zero(gy + base, cg, CG, g + 8);
    load8_or_zero(gy + base, cg + 1, CG, g + 16);
    float sq[24];
#pragma unroll
    for (int i = 0; i < 24; ++i) sq[i] = v[i] * v[i];
    // r_j = gy_j · x_j · s_j^(-β-1) and s_j^-β for j ∈ [8-h, 15+h] (needs sq over [8-2h, 15+2h])
    float r[24], sb[24];
#pragma unroll
    for (int j = 8 - HH; j < 16 + HH; ++j) {
      float acc = 0.f;
#pragma unroll
      for (int d = -HH; d <= HH; ++d) acc += sq[j + d];
      const float s = k + alpha_n * acc;
      const float pb = pow_neg(s, beta);
      sb[j] = pb;
      r[j] = g[j] * v[j] * pb / s;
    }
    float out[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const int j = 8 + e;
      float acc = 0.f;
#pragma unroll
      for (int d = -HH; d <= HH; ++d) acc += r[j + d];
      out[e] = g[j] * sb[j] - coef * v[j] * acc;
    }
    st8(gx + base + cg * 8, out);
  }
}

// Requirements (checked): C % 8 == 0, odd size, size ≤ 17 forward / ≤ 9 backward, 16-B aligned.
template <typename T>
static int lrn_fwd(const void* x, void* y, long long pixels, int C, int size, float alpha, float beta, float k,
                   hipStream_t s) {
  if (C % 8 || !(size & 1) || size > 17 || pixels <= 0 || ((uintptr_t)x & 15) || ((uintptr_t)y & 15))
    return (int)hipErrorInvalidValue;
  const long long work = pixels * (C / 8);
  const dim3 g(bigdl_grid(work, 256, 8192)), b(256);
  const T* xp = (const T*)x;
  T* yp = (T*)y;
  const float an = alpha / size;
  switch (size / 2) {
    case 0: hipLaunchKernelGGL((k_lrn_fwd<0, T>), g, b, 0, s, xp, yp, pixels, C, an, beta, k); break;
    case 1: hipLaunchKernelGGL((k_lrn_fwd<1, T>), g, b, 0, s, xp, yp, pixels, C, an, beta, k); break;
    case 2: hipLaunchKernelGGL((k_lrn_fwd<2, T>), g, b, 0, s, xp, yp, pixels, C, an, beta, k); break;
    case 3: hipLaunchKernelGGL((k_lrn_fwd<3, T>), g, b, 0, s, xp, yp, pixels, C, an, beta, k); break;
    case 4: hipLaunchKernelGGL((k_lrn_fwd<4, T>), g, b, 0, s, xp, yp, pixels, C, an, beta, k); break;
    case 5: hipLaunchKernelGGL((k_lrn_fwd<5, T>), g, b, 0, s, xp, yp, pixels, C, an, beta, k); break;
    case 6: hipLaunchKernelGGL((k_lrn_fwd<6, T>), g, b, 0, s, xp, yp, pixels, C, an, beta, k); break;
    case 7: hipLaunchKernelGGL((k_lrn_fwd<7, T>), g, b, 0, s, xp, yp, pixels, C, an, beta, k); break;
    default: hipLaunchKernelGGL((k_lrn_fwd<8, T>), g, b, 0, s, xp, yp, pixels, C, an, beta, k); break;
  }
  BIGDL_CHECK_LAUNCH();
}

template <typename T>
static int lrn_bwd(const void* x, const void* gy, void* gx, long long pixels, int C, int size, float alpha, float beta,
                   float k, hipStream_t s) {
  if (C % 8 || !(size & 1) || size > 9 || pixels <= 0 || ((uintptr_t)x & 15) || ((uintptr_t)gy & 15) ||
      ((uintptr_t)gx & 15))
    return (int)hipErrorInvalidValue;
  const long long work = pixels * (C / 8);
  const dim3 g(bigdl_grid(work, 256, 8192)), b(256);
  const T* xp = (const T*)x;
  const T* gp = (const T*)gy;
  T* op = (T*)gx;
  const float an = alpha / size;
  switch (size / 2) {
    case 0: hipLaunchKernelGGL((k_lrn_bwd<0, T>), g, b, 0, s, xp, gp, op, pixels, C, an, beta, k); break;
    case 1: hipLaunchKernelGGL((k_lrn_bwd<1, T>), g, b, 0, s, xp, gp, op, pixels, C, an, beta, k); break;
    case 2: hipLaunchKernelGGL((k_lrn_bwd<2, T>), g, b, 0, s, xp, gp, op, pixels, C, an, beta, k); break;
    case 3: hipLaunchKernelGGL((k_lrn_bwd<3, T>), g, b, 0, s, xp, gp, op, pixels, C, an, beta, k); break;
    default: hipLaunchKernelGGL((k_lrn_bwd<4, T>), g, b, 0, s, xp, gp, op, pixels, C, an, beta, k); break;
  }
  BIGDL_CHECK_LAUNCH();
}

BIGDL_EXPORT int bigdl_lrn_fwd(const void* x, void* y, long long pixels, int C, int size, float alpha, float beta,
                               float k, hipStream_t s) {
  return lrn_fwd<bf16_t>(x, y, pixels, C, size, alpha, beta, k, s);
}
BIGDL_EXPORT int bigdl_lrn_bwd(const void* x, const void* gy, void* gx, long long pixels, int C, int size, float alpha,
                               float beta, float k, hipStream_t s) {
  return lrn_bwd<bf16_t>(x, gy, gx, pixels, C, size, alpha, beta, k, s);
}
BIGDL_EXPORT int bigdl_lrn_fwd_f32(const void* x, void* y, long long pixels, int C, int size, float alpha, float beta,
                                   float k, hipStream_t s) {
  return lrn_fwd<float>(x, y, pixels, C, size, alpha, beta, k, s);
}
BIGDL_EXPORT int bigdl_lrn_bwd_f32(const void* x, const void* gy, void* gx, long long pixels, int C, int size,
                                   float alpha, float beta, float k, hipStream_t s) {
  return lrn_bwd<float>(x, gy, gx, pixels, C, size, alpha, beta, k, s);
}
