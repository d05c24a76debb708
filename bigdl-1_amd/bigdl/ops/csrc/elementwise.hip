// Elementwise kernels: dtype casts, ReLU/Threshold fwd+bwd (K8), fused optimizer updates (K22).
// All are HBM-bound streaming kernels: 16 B per lane per access, grid-stride, grid capped at
// 2048 blocks of 256 (cdna_hip_programming.md Guideline 11).
#include "common.h"

// ------------------------------------------------------------------------------------------------
// casts
// ------------------------------------------------------------------------------------------------
__global__ void k_f32_to_bf16(const float* __restrict__ src, bf16_t* __restrict__ dst, long long n) {
  long long n8 = n >> 3;
  long long stride = (long long)gridDim.x * blockDim.x;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n8; i += stride) {
    float4 a = reinterpret_cast<const float4*>(src)[2 * i];
    float4 b = reinterpret_cast<const float4*>(src)[2 * i + 1];
    float v[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
    store8(dst + 8 * i, v);
  }
  for (long long i = (n8 << 3) + (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride)
    dst[i] = f2bf(src[i]);
}

__global__ void k_bf16_to_f32(const bf16_t* __restrict__ src, float* __restrict__ dst, long long n) {
  long long n8 = n >> 3;
  long long stride = (long long)gridDim.x * blockDim.x;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n8; i += stride) {
    float v[8];
    load8(src + 8 * i, v);
    reinterpret_cast<float4*>(dst)[2 * i] = make_float4(v[0], v[1], v[2], v[3]);
    reinterpret_cast<float4*>(dst)[2 * i + 1] = make_float4(v[4], v[5], v[6], v[7]);
  }
  for (long long i = (n8 << 3) + (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride)
    dst[i] = bf2f(src[i]);
}

// 32-bit fill (the per-step gradient-arena clear): 16-B vector stores, grid-stride, scalar tail
__global__ void k_fill32(uint32_t* __restrict__ dst, long long n, uint32_t v) {
  const long long n4 = n >> 2;
  const long long stride = (long long)gridDim.x * blockDim.x;
  const uint4 q = make_uint4(v, v, v, v);
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += stride)
    reinterpret_cast<uint4*>(dst)[i] = q;
  for (long long i = (n4 << 2) + (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) dst[i] = v;
}

// n 32-bit words of dst (16-B aligned, checked on the host) set to the bit pattern v
BIGDL_EXPORT int bigdl_fill32(void* dst, long long n, uint32_t v, hipStream_t s) {
  if (n <= 0) return 0;
  const int grid = bigdl_grid((n + 3) / 4, 256);
  hipLaunchKernelGGL(k_fill32, dim3(grid), dim3(256), 0, s, (uint32_t*)dst, n, v);
  BIGDL_CHECK_LAUNCH();
}

// conv weight rows [K][taps][C] (bf16, KRSC) → [K][ldw] with every tap's channels zero-padded to cp
// and the row zero-padded to ldw (the narrow-channel conv operand: the RGB stem's C4 gather, C % 8
// inputs); one pass, every destination element written once
__global__ void k_pad_taps_bf16(const bf16_t* __restrict__ src, bf16_t* __restrict__ dst, int K, int taps, int C,
                                int cp, int ldw) {
  const long long n = (long long)K * ldw;
  const long long stride = (long long)gridDim.x * blockDim.x;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    const int k = (int)(i / ldw), j = (int)(i - (long long)k * ldw);
    const int t = j / cp, c = j - t * cp;
    dst[i] = (t < taps && c < C) ? src[((long long)k * taps + t) * C + c] : (bf16_t)0;
  }
}

BIGDL_EXPORT int bigdl_pad_taps_bf16(const void* src, void* dst, int K, int taps, int C, int cp, int ldw,
                                     hipStream_t s) {
  if (K <= 0 || taps <= 0 || C <= 0 || cp < C || ldw < taps * cp) return (int)hipErrorInvalidValue;
  const int grid = bigdl_grid((long long)K * ldw, 256);
  hipLaunchKernelGGL(k_pad_taps_bf16, dim3(grid), dim3(256), 0, s, (const bf16_t*)src, (bf16_t*)dst, K, taps, C, cp,
                     ldw);
  BIGDL_CHECK_LAUNCH();
}

// mode 0: f32->bf16, 1: bf16->f32.  Pointers must be 16-B aligned (checked on the host).
BIGDL_EXPORT int bigdl_cast(const void* src, void* dst, long long n, int mode, hipStream_t s) {
  if (n <= 0) return 0;
  int grid = bigdl_grid((n + 7) / 8, 256);
  if (mode == 0)
    hipLaunchKernelGGL(k_f32_to_bf16, dim3(grid), dim3(256), 0, s, (const float*)src, (bf16_t*)dst, n);
  else
    hipLaunchKernelGGL(k_bf16_to_f32, dim3(grid), dim3(256), 0, s, (const bf16_t*)src, (float*)dst, n);
  BIGDL_CHECK_LAUNCH();
}

// ------------------------------------------------------------------------------------------------
// ReLU / Threshold (bf16): y = x > th ? x : v ; backward gx = gy * (ref > th)
// ------------------------------------------------------------------------------------------------
__global__ void k_threshold_fwd_bf16(const bf16_t* __restrict__ x, bf16_t* __restrict__ y, long long n8, float th,
                                     float val) {
  long long stride = (long long)gridDim.x * blockDim.x;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n8; i += stride) {
    float v[8];
    load8(x + 8 * i, v);
#pragma unroll
    for (int k = 0; k < 8; ++k) v[k] = v[k] > th ? v[k] : val;
    store8(y + 8 * i, v);
  }
}

__global__ void k_threshold_bwd_bf16(const bf16_t* __restrict__ gy, const bf16_t* __restrict__ ref,
                                     bf16_t* __restrict__ gx, long long n8, float th) {
  long long stride = (long long)gridDim.x * blockDim.x;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n8; i += stride) {
    float g[8], r[8];
    load8(gy + 8 * i, g);
    load8(ref + 8 * i, r);
#pragma unroll
    for (int k = 0; k < 8; ++k) g[k] = r[k] > th ? g[k] : 0.f;
    store8(gx + 8 * i, g);
  }
}

BIGDL_EXPORT int bigdl_threshold_fwd_bf16(const void* x, void* y, long long n, float th, float val, hipStream_t s) {
  if (n <= 0) return 0;
  if (n % 8) return (int)hipErrorInvalidValue;
  long long n8 = n / 8;
  hipLaunchKernelGGL(k_threshold_fwd_bf16, dim3(bigdl_grid(n8, 256)), dim3(256), 0, s, (const bf16_t*)x, (bf16_t*)y,
                     n8, th, val);
  BIGDL_CHECK_LAUNCH();
}

BIGDL_EXPORT int bigdl_threshold_bwd_bf16(const void* gy, const void* ref, void* gx, long long n, float th,
                                          hipStream_t s) {
  if (n <= 0) return 0;
  if (n % 8) return (int)hipErrorInvalidValue;
  long long n8 = n / 8;
  hipLaunchKernelGGL(k_threshold_bwd_bf16, dim3(bigdl_grid(n8, 256)), dim3(256), 0, s, (const bf16_t*)gy,
                     (const bf16_t*)ref, (bf16_t*)gx, n8, th);
  BIGDL_CHECK_LAUNCH();
}

// fp32 variants (the reference's precision, DL/nn/Threshold.scala:46-421): 16 B per lane, a scalar
// tail for n % 4.  Backward takes the forward's INPUT (in-place forward: its output, which is > th
// exactly where the input was, since the replacement value v ≤ th is the only other output).
__global__ void k_threshold_fwd_f32(const float* __restrict__ x, float* __restrict__ y, long long n, float th,
                                    float val) {
  const long long n4 = n >> 2, stride = (long long)gridDim.x * blockDim.x;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += stride) {
    float4 v = reinterpret_cast<const float4*>(x)[i];
    v.x = v.x > th ? v.x : val;
    v.y = v.y > th ? v.y : val;
    v.z = v.z > th ? v.z : val;
    v.w = v.w > th ? v.w : val;
    reinterpret_cast<float4*>(y)[i] = v;
  }
  for (long long i = (n4 << 2) + (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride)
    y[i] = x[i] > th ? x[i] : val;
}

__global__ void k_threshold_bwd_f32(const float* __restrict__ gy, const float* __restrict__ ref,
                                    float* __restrict__ gx, long long n, float th) {
  const long long n4 = n >> 2, stride = (long long)gridDim.x * blockDim.x;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += stride) {
    float4 g = reinterpret_cast<const float4*>(gy)[i];
    const float4 r = reinterpret_cast<const float4*>(ref)[i];
    g.x = r.x > th ? g.x : 0.f;
    g.y = r.y > th ? g.y : 0.f;
    g.z = r.z > th ? g.z : 0.f;
    g.w = r.w > th ? g.w : 0.f;
    reinterpret_cast<float4*>(gx)[i] = g;
  }
  for (long long i = (n4 << 2) + (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride)
    gx[i] = ref[i] > th ? gy[i] : 0.f;
}

BIGDL_EXPORT int bigdl_threshold_fwd_f32(const void* x, void* y, long long n, float th, float val, hipStream_t s) {
  if (n <= 0) return 0;
  hipLaunchKernelGGL(k_threshold_fwd_f32, dim3(bigdl_grid((n + 3) / 4, 256)), dim3(256), 0, s, (const float*)x,
                     (float*)y, n, th, val);
  BIGDL_CHECK_LAUNCH();
}

BIGDL_EXPORT int bigdl_threshold_bwd_f32(const void* gy, const void* ref, void* gx, long long n, float th,
                                         hipStream_t s) {
  if (n <= 0) return 0;
  hipLaunchKernelGGL(k_threshold_bwd_f32, dim3(bigdl_grid((n + 3) / 4, 256)), dim3(256), 0, s, (const float*)gy,
                     (const float*)ref, (float*)gx, n, th);
  BIGDL_CHECK_LAUNCH();
}

// ------------------------------------------------------------------------------------------------
// fused SGD (DL/optim/SGD.scala:61-124) over a flat fp32 buffer:
//   g' = g*scale (+ wd * wds * w) ; v = first ? g' : mom*v + (1-damp)*g' ;
//   d = nesterov ? g' + mom*v : v (or g' when mom == 0) ; w -= lr * (lrs ? lrs*d : d) ;
//   shadow = bf16(w)
// ------------------------------------------------------------------------------------------------
// gradient loads: fp32, or the bf16 reduce-scatter output of the bf16 wire format (read
// directly — no separate unpack pass over the shard)
__device__ __forceinline__ float g_at(const float* g, long long e) { return g[e]; }
__device__ __forceinline__ float g_at(const bf16_t* g, long long e) { return bf2f(g[e]); }
__device__ __forceinline__ void g_load4(const float* g, long long i, float* o) {
  float4 G = reinterpret_cast<const float4*>(g)[i];
  o[0] = G.x; o[1] = G.y; o[2] = G.z; o[3] = G.w;
}
__device__ __forceinline__ void g_load4(const bf16_t* g, long long i, float* o) {
  uint2 G = reinterpret_cast<const uint2*>(g)[i];
  o[0] = __uint_as_float(G.x << 16); o[1] = __uint_as_float(G.x & 0xffff0000u);
  o[2] = __uint_as_float(G.y << 16); o[3] = __uint_as_float(G.y & 0xffff0000u);
}

template <typename GT, bool MOM, bool NEST, bool FIRST, bool SHADOW, bool PERELEM>
__global__ void k_sgd(float* __restrict__ w, const GT* __restrict__ g, float* __restrict__ buf,
                      bf16_t* __restrict__ shadow, const float* __restrict__ lrs, const float* __restrict__ wds,
                      long long n4, float lr, float mom, float damp, float wd, float scale, int tail,
                      const float* __restrict__ first_dev) {
  long long stride = (long long)gridDim.x * blockDim.x;
  // first-iteration rule (v = g) from the template or, in HIP-graph mode, from a device flag the
  // captured step clears after the update (so a replayed graph can start a fresh trajectory)
  const bool first = FIRST || (first_dev != nullptr && *first_dev != 0.f);
  if (blockIdx.x == 0 && threadIdx.x < tail) {
    // the n % 4 trailing elements (scalar; the arena slice need not be a multiple of 4)
    const long long e = n4 * 4 + threadIdx.x;
    const float wv = w[e];
    const float gg = g_at(g, e) * scale + wd * (PERELEM && wds ? wds[e] : 1.f) * wv;
    float d = gg;
    if (MOM) {
      const float b = first ? gg : mom * buf[e] + (1.f - damp) * gg;
      buf[e] = b;
      d = NEST ? gg + mom * b : b;
    }
    const float nw = wv - lr * (PERELEM && lrs ? lrs[e] : 1.f) * d;
    w[e] = nw;
    if (SHADOW) shadow[e] = f2bf(nw);
  }
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += stride) {
    float4 W = reinterpret_cast<float4*>(w)[i];
    float wv[4] = {W.x, W.y, W.z, W.w};
    float gv[4];
    g_load4(g, i, gv);
    float wdv[4] = {1.f, 1.f, 1.f, 1.f};
    float lrv[4] = {1.f, 1.f, 1.f, 1.f};
    if (PERELEM) {
      if (wds) {
        float4 t = reinterpret_cast<const float4*>(wds)[i];
        wdv[0] = t.x; wdv[1] = t.y; wdv[2] = t.z; wdv[3] = t.w;
      }
      if (lrs) {
        float4 t = reinterpret_cast<const float4*>(lrs)[i];
        lrv[0] = t.x; lrv[1] = t.y; lrv[2] = t.z; lrv[3] = t.w;
      }
    }
    float bv[4] = {0.f, 0.f, 0.f, 0.f};
    if (MOM && !first) {
      float4 B = reinterpret_cast<float4*>(buf)[i];
      bv[0] = B.x; bv[1] = B.y; bv[2] = B.z; bv[3] = B.w;
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      float gg = gv[k] * scale + wd * wdv[k] * wv[k];
      float d = gg;
      if (MOM) {
        bv[k] = first ? gg : mom * bv[k] + (1.f - damp) * gg;
        d = NEST ? gg + mom * bv[k] : bv[k];
      }
      wv[k] -= lr * lrv[k] * d;
    }
    reinterpret_cast<float4*>(w)[i] = make_float4(wv[0], wv[1], wv[2], wv[3]);
    if (MOM) reinterpret_cast<float4*>(buf)[i] = make_float4(bv[0], bv[1], bv[2], bv[3]);
    if (SHADOW) {
      uint32_t lo = (uint32_t)f2bf(wv[0]) | ((uint32_t)f2bf(wv[1]) << 16);
      uint32_t hi = (uint32_t)f2bf(wv[2]) | ((uint32_t)f2bf(wv[3]) << 16);
      reinterpret_cast<uint2*>(shadow)[i] = make_uint2(lo, hi);
    }
  }
}

#define SGD_LAUNCH(M, NS, F, SH, PE)                                                                    \
  hipLaunchKernelGGL((k_sgd<GT, M, NS, F, SH, PE>), dim3(grid), dim3(256), 0, s, w, g, buf, shadow, lrs, wds, n4, \
                     lr, mom, damp, wd, scale, tail, first_dev)

template <typename GT>
static int sgd_impl(float* w, const GT* g, float* buf, bf16_t* shadow, const float* lrs, const float* wds,
                    long long n, float lr, float mom, float damp, float wd, int nesterov, int first, float scale,
                    const float* first_dev, hipStream_t s) {
  if (n <= 0) return 0;
  const long long n4 = n / 4;
  const int tail = (int)(n & 3);
  int grid = bigdl_grid(n4 > 0 ? n4 : 1, 256);
  bool M = mom != 0.f, NS = nesterov != 0, F = first != 0, SH = shadow != nullptr, PE = (lrs || wds);
  // dispatch the common combinations without per-element branches
  if (!PE) {
    if (M && NS && !F && SH) SGD_LAUNCH(true, true, false, true, false);
    else if (M && NS && !F && !SH) SGD_LAUNCH(true, true, false, false, false);
    else if (M && !NS && !F && SH) SGD_LAUNCH(true, false, false, true, false);
    else if (M && !NS && !F && !SH) SGD_LAUNCH(true, false, false, false, false);
    else if (M && NS && F && SH) SGD_LAUNCH(true, true, true, true, false);
    else if (M && NS && F && !SH) SGD_LAUNCH(true, true, true, false, false);
    else if (M && !NS && F && SH) SGD_LAUNCH(true, false, true, true, false);
    else if (M && !NS && F && !SH) SGD_LAUNCH(true, false, true, false, false);
    else if (!M && SH) SGD_LAUNCH(false, false, false, true, false);
    else SGD_LAUNCH(false, false, false, false, false);
  } else {
    // the shadow flag must follow the pointer: a sharded fp32-wire update passes no shadow
    if (SH) {
      if (M && NS && F) SGD_LAUNCH(true, true, true, true, true);
      else if (M && NS) SGD_LAUNCH(true, true, false, true, true);
      else if (M && F) SGD_LAUNCH(true, false, true, true, true);
      else if (M) SGD_LAUNCH(true, false, false, true, true);
      else SGD_LAUNCH(false, false, false, true, true);
    } else {
      if (M && NS && F) SGD_LAUNCH(true, true, true, false, true);
      else if (M && NS) SGD_LAUNCH(true, true, false, false, true);
      else if (M && F) SGD_LAUNCH(true, false, true, false, true);
      else if (M) SGD_LAUNCH(true, false, false, false, true);
      else SGD_LAUNCH(false, false, false, false, true);
    }
  }
  BIGDL_CHECK_LAUNCH();
}


// all pointers 16-B aligned (host-checked); the n % 4 tail is handled by block 0.
// first_dev: optional device flag (graph mode), non-zero = apply the first-iteration rule
BIGDL_EXPORT int bigdl_sgd(float* w, const float* g, float* buf, bf16_t* shadow, const float* lrs, const float* wds,
                           long long n, float lr, float mom, float damp, float wd, int nesterov, int first,
                           float scale, const float* first_dev, hipStream_t s) {
  return sgd_impl<float>(w, g, buf, shadow, lrs, wds, n, lr, mom, damp, wd, nesterov, first, scale, first_dev, s);
}

// same update with a bf16 gradient (the bf16-wire reduce-scatter output); g 8-B aligned
BIGDL_EXPORT int bigdl_sgd_g16(float* w, const bf16_t* g, float* buf, bf16_t* shadow, const float* lrs,
                               const float* wds, long long n, float lr, float mom, float damp, float wd, int nesterov,
                               int first, float scale, const float* first_dev, hipStream_t s) {
  return sgd_impl<bf16_t>(w, g, buf, shadow, lrs, wds, n, lr, mom, damp, wd, nesterov, first, scale, first_dev, s);
}

// ------------------------------------------------------------------------------------------------
// fused Adam (DL/optim/Adam.scala): m = b1 m + (1-b1) g ; v = b2 v + (1-b2) g² ;
// w -= step_size * m / (sqrt(v) + eps), step_size = lr * sqrt(1-b2^t) / (1-b1^t)
// ------------------------------------------------------------------------------------------------
__global__ void k_adam(float* __restrict__ w, const float* __restrict__ g, float* __restrict__ m,
                       float* __restrict__ v, bf16_t* __restrict__ shadow, long long n4, float step_size, float b1,
                       float b2, float eps, float wd, float scale, int tail, const float* __restrict__ dev_n,
                       float lr, float lr_decay) {
  long long stride = (long long)gridDim.x * blockDim.x;
  if (dev_n) {
    // replay-safe form (HIP graphs): the iteration count n lives on the device, so the decayed
    // rate and the bias corrections are formed here instead of baked in as a host scalar
    const float n = dev_n[0], t = n + 1.f;
    step_size = lr / (1.f + n * lr_decay) * sqrtf(1.f - powf(b2, t)) / (1.f - powf(b1, t));
  }
  if (blockIdx.x == 0 && threadIdx.x < tail) {
    const long long e = n4 * 4 + threadIdx.x;
    const float gg = g[e] * scale + wd * w[e];
    const float mm = b1 * m[e] + (1.f - b1) * gg, vv = b2 * v[e] + (1.f - b2) * gg * gg;
    m[e] = mm;
    v[e] = vv;
    const float nw = w[e] - step_size * mm / (sqrtf(vv) + eps);
    w[e] = nw;
    if (shadow) shadow[e] = f2bf(nw);
  }
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += stride) {
    float4 W = reinterpret_cast<float4*>(w)[i];
    float4 G = reinterpret_cast<const float4*>(g)[i];
    float4 M = reinterpret_cast<float4*>(m)[i];
    float4 V = reinterpret_cast<float4*>(v)[i];
    float wv[4] = {W.x, W.y, W.z, W.w}, gv[4] = {G.x, G.y, G.z, G.w};
    float mv[4] = {M.x, M.y, M.z, M.w}, vv[4] = {V.x, V.y, V.z, V.w};
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      float gg = gv[k] * scale + wd * wv[k];
      mv[k] = b1 * mv[k] + (1.f - b1) * gg;
      vv[k] = b2 * vv[k] + (1.f - b2) * gg * gg;
      wv[k] -= step_size * mv[k] / (sqrtf(vv[k]) + eps);
    }
    reinterpret_cast<float4*>(w)[i] = make_float4(wv[0], wv[1], wv[2], wv[3]);
    reinterpret_cast<float4*>(m)[i] = make_float4(mv[0], mv[1], mv[2], mv[3]);
    reinterpret_cast<float4*>(v)[i] = make_float4(vv[0], vv[1], vv[2], vv[3]);
    if (shadow) {
      uint32_t lo = (uint32_t)f2bf(wv[0]) | ((uint32_t)f2bf(wv[1]) << 16);
      uint32_t hi = (uint32_t)f2bf(wv[2]) | ((uint32_t)f2bf(wv[3]) << 16);
      reinterpret_cast<uint2*>(shadow)[i] = make_uint2(lo, hi);
    }
  }
}

BIGDL_EXPORT int bigdl_adam(float* w, const float* g, float* m, float* v, bf16_t* shadow, long long n,
                            float step_size, float b1, float b2, float eps, float wd, float scale, hipStream_t s) {
  if (n <= 0) return 0;
  const long long n4 = n / 4;
  hipLaunchKernelGGL(k_adam, dim3(bigdl_grid(n4 > 0 ? n4 : 1, 256)), dim3(256), 0, s, w, g, m, v, shadow, n4,
                     step_size, b1, b2, eps, wd, scale, (int)(n & 3), (const float*)nullptr, 0.f, 0.f);
  BIGDL_CHECK_LAUNCH();
}

// dev_n: fp32 [1] iteration count before this step (the caller advances it after the launch)
BIGDL_EXPORT int bigdl_adam_dev(float* w, const float* g, float* m, float* v, bf16_t* shadow, long long n,
                                const float* dev_n, float lr, float lr_decay, float b1, float b2, float eps, float wd,
                                float scale, hipStream_t s) {
  if (n <= 0) return 0;
  const long long n4 = n / 4;
  hipLaunchKernelGGL(k_adam, dim3(bigdl_grid(n4 > 0 ? n4 : 1, 256)), dim3(256), 0, s, w, g, m, v, shadow, n4, 0.f,
                     b1, b2, eps, wd, scale, (int)(n & 3), dev_n, lr, lr_decay);
  BIGDL_CHECK_LAUNCH();
}

// ------------------------------------------------------------------------------------------------
// fused Adagrad (DL/optim/Adagrad.scala): g' = scale·g + wd·w ; s += g'² ;
// w -= clr · g' / (sqrt(s) + 1e-10),  clr = lr / (1 + n·lr_decay) — one pass over (w, g, s) plus the
// optional bf16 shadow, in place of five torch elementwise kernels.  dev_n (nullable): the
// iteration count n read on the device (replay-safe under HIP-graph capture); else clr is given.
// G = bf16: the gradient read straight from the DistriOptimizer's bf16 reduce-scatter wire shard
// (widened on load, as the SGD kernel does) — no fp32 unpack pass per bucket.
__device__ __forceinline__ float ag_ld(const float* g, long long e) { return g[e]; }
__device__ __forceinline__ float ag_ld(const bf16_t* g, long long e) { return bf2f(g[e]); }
__device__ __forceinline__ void ag_ld4(const float* g, long long i, float (&o)[4]) {
  const float4 G = reinterpret_cast<const float4*>(g)[i];
  o[0] = G.x; o[1] = G.y; o[2] = G.z; o[3] = G.w;
}
__device__ __forceinline__ void ag_ld4(const bf16_t* g, long long i, float (&o)[4]) {
  const uint2 u = reinterpret_cast<const uint2*>(g)[i];
  o[0] = __uint_as_float(u.x << 16); o[1] = __uint_as_float(u.x & 0xFFFF0000u);
  o[2] = __uint_as_float(u.y << 16); o[3] = __uint_as_float(u.y & 0xFFFF0000u);
}

template <typename G>
__global__ void k_adagrad(float* __restrict__ w, const G* __restrict__ g, float* __restrict__ sv,
                          bf16_t* __restrict__ shadow, long long n4, float clr, float wd, float scale, int tail,
                          const float* __restrict__ dev_n, float lr, float lr_decay) {
  if (dev_n) clr = lr / (1.f + dev_n[0] * lr_decay);
  const long long stride = (long long)gridDim.x * blockDim.x;
  if (blockIdx.x == 0 && threadIdx.x < tail) {
    const long long e = n4 * 4 + threadIdx.x;
    const float gg = ag_ld(g, e) * scale + wd * w[e];
    const float ss = sv[e] + gg * gg;
    sv[e] = ss;
    const float nw = w[e] - clr * gg / (sqrtf(ss) + 1e-10f);
    w[e] = nw;
    if (shadow) shadow[e] = f2bf(nw);
  }
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += stride) {
    const float4 W = reinterpret_cast<float4*>(w)[i];
    const float4 S = reinterpret_cast<float4*>(sv)[i];
    float wv[4] = {W.x, W.y, W.z, W.w}, gv[4], sq[4] = {S.x, S.y, S.z, S.w};
    ag_ld4(g, i, gv);
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const float gg = gv[k] * scale + wd * wv[k];
      sq[k] += gg * gg;
      wv[k] -= clr * gg / (sqrtf(sq[k]) + 1e-10f);
    }
    reinterpret_cast<float4*>(w)[i] = make_float4(wv[0], wv[1], wv[2], wv[3]);
    reinterpret_cast<float4*>(sv)[i] = make_float4(sq[0], sq[1], sq[2], sq[3]);
    if (shadow) {
      const uint32_t lo = (uint32_t)f2bf(wv[0]) | ((uint32_t)f2bf(wv[1]) << 16);
      const uint32_t hi = (uint32_t)f2bf(wv[2]) | ((uint32_t)f2bf(wv[3]) << 16);
      reinterpret_cast<uint2*>(shadow)[i] = make_uint2(lo, hi);
    }
  }
}

BIGDL_EXPORT int bigdl_adagrad(float* w, const float* g, float* sv, bf16_t* shadow, long long n, float clr,
                               const float* dev_n, float lr, float lr_decay, float wd, float scale, hipStream_t s) {
  if (n <= 0) return 0;
  const long long n4 = n / 4;
  hipLaunchKernelGGL(k_adagrad<float>, dim3(bigdl_grid(n4 > 0 ? n4 : 1, 256)), dim3(256), 0, s, w, g, sv, shadow, n4,
                     clr, wd, scale, (int)(n & 3), dev_n, lr, lr_decay);
  BIGDL_CHECK_LAUNCH();
}

// the same update with a bf16 gradient (8-B aligned: the host checks)
BIGDL_EXPORT int bigdl_adagrad_g16(float* w, const bf16_t* g, float* sv, bf16_t* shadow, long long n, float clr,
                                   const float* dev_n, float lr, float lr_decay, float wd, float scale, hipStream_t s) {
  if (n <= 0) return 0;
  const long long n4 = n / 4;
  hipLaunchKernelGGL(k_adagrad<bf16_t>, dim3(bigdl_grid(n4 > 0 ? n4 : 1, 256)), dim3(256), 0, s, w, g, sv, shadow, n4,
                     clr, wd, scale, (int)(n & 3), dev_n, lr, lr_decay);
  BIGDL_CHECK_LAUNCH();
}

// ------------------------------------------------------------------------------------------------
// Reference wire format (K23, FP16CompressedTensor.scala:43-277): fp32 → bf16 by truncation (the
// top 16 bits, no rounding), written straight into the reduce-scatter wire buffer — one pass in
// place of the int32 view / shift / narrow temporaries of the torch formulation.
__global__ void __launch_bounds__(256) k_trunc_bf16(const uint32_t* __restrict__ src, bf16_t* __restrict__ dst,
                                                    long long n) {
  const long long n4 = n >> 2;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n4; i += (long long)gridDim.x * blockDim.x) {
    const uint4 u = reinterpret_cast<const uint4*>(src)[i];
    reinterpret_cast<uint2*>(dst)[i] = make_uint2((u.x >> 16) | (u.y & 0xFFFF0000u), (u.z >> 16) | (u.w & 0xFFFF0000u));
  }
  for (long long i = n4 * 4 + blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n;
       i += (long long)gridDim.x * blockDim.x)
    dst[i] = (bf16_t)(src[i] >> 16);
}

BIGDL_EXPORT int bigdl_trunc_bf16(const float* src, void* dst, long long n, hipStream_t s) {
  if (n <= 0 || ((uintptr_t)src & 15) || ((uintptr_t)dst & 7)) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(k_trunc_bf16, dim3(bigdl_grid((n + 3) / 4, 256, 8192)), dim3(256), 0, s, (const uint32_t*)src,
                     (bf16_t*)dst, n);
  BIGDL_CHECK_LAUNCH();
}

// ------------------------------------------------------------------------------------------------
// NCHW (fp32 or bf16) → NHWC bf16 in one pass (K24: the host-layout → device-layout boundary,
// a cast plus a channels-last copy otherwise).  A block transposes a 32-channel × 64-pixel tile
// through LDS: reads coalesced along pixels, writes 64-B runs along channels.
template <typename T>
__global__ void __launch_bounds__(256) k_nchw_to_nhwc(const T* __restrict__ x, bf16_t* __restrict__ y, int C,
                                                      long long HW) {
  __shared__ float tile[32][65];
  const int n = blockIdx.z;
  const int c0 = blockIdx.y * 32;
  const long long p0 = (long long)blockIdx.x * 64;
  const T* xs = x + (long long)n * C * HW;
  for (int i = threadIdx.x; i < 32 * 64; i += 256) {
    const int cl = i >> 6, pl = i & 63;
    const int c = c0 + cl;
    const long long p = p0 + pl;
    float v = 0.f;
    if (c < C && p < HW) {
      if constexpr (sizeof(T) == 4) v = xs[(long long)c * HW + p];
      else v = bf2f(xs[(long long)c * HW + p]);
    }
    tile[cl][pl] = v;
  }
  __syncthreads();
  bf16_t* ys = y + (long long)n * HW * C;
  for (int i = threadIdx.x; i < 32 * 64; i += 256) {
    const int pl = i >> 5, cl = i & 31;
    const int c = c0 + cl;
    const long long p = p0 + pl;
    if (c < C && p < HW) ys[p * C + c] = f2bf(tile[cl][pl]);
  }
}

// Few-channel images (the RGB model input): one thread per pixel reads its C planes (coalesced along
// pixels) and writes the Cp-channel zero-padded NHWC row as ONE 8-B (Cp 4) or 16-B (Cp 8) store —
// the stem conv's channel-padded operand directly, no tile transpose and no separate pad pass.
template <typename T>
__device__ __forceinline__ float ld_as_f32(const T* p) {
  if constexpr (sizeof(T) == 4) return *p;
  else return bf2f(*p);
}

template <typename T, int CP>
__global__ void __launch_bounds__(256) k_nchw_to_nhwc_pad(const T* __restrict__ x, bf16_t* __restrict__ y, int C,
                                                          long long HW, long long total) {
  for (long long t = blockIdx.x * 256LL + threadIdx.x; t < total; t += (long long)gridDim.x * 256) {
    const long long n = t / HW, p = t - n * HW;
    const T* xs = x + n * C * HW + p;
    uint32_t w[CP / 2];
#pragma unroll
    for (int e = 0; e < CP / 2; ++e) {
      float v0 = 0.f, v1 = 0.f;
      if (2 * e < C) v0 = ld_as_f32(xs + (2 * e) * HW);
      if (2 * e + 1 < C) v1 = ld_as_f32(xs + (2 * e + 1) * HW);
      w[e] = (uint32_t)f2bf(v0) | ((uint32_t)f2bf(v1) << 16);
    }
    if constexpr (CP == 4) *reinterpret_cast<uint2*>(y + t * 4) = make_uint2(w[0], w[1]);
    else *reinterpret_cast<uint4*>(y + t * 8) = make_uint4(w[0], w[1], w[2], w[3]);
  }
}

BIGDL_EXPORT int bigdl_nchw_to_nhwc_pad_bf16(const void* x, int dtype, void* y, int N, int C, long long HW, int Cp,
                                             hipStream_t s) {
  if (!x || !y || N <= 0 || HW <= 0 || C <= 0 || C > Cp || (Cp != 4 && Cp != 8) || ((uintptr_t)y & (2 * Cp - 1)))
    return (int)hipErrorInvalidValue;
  const long long total = (long long)N * HW;
  const dim3 g((unsigned)bigdl_grid(total, 256, 65536));
  if (dtype == 0) {
    if (Cp == 4) hipLaunchKernelGGL((k_nchw_to_nhwc_pad<float, 4>), g, dim3(256), 0, s, (const float*)x, (bf16_t*)y, C, HW, total);
    else hipLaunchKernelGGL((k_nchw_to_nhwc_pad<float, 8>), g, dim3(256), 0, s, (const float*)x, (bf16_t*)y, C, HW, total);
  } else {
    if (Cp == 4) hipLaunchKernelGGL((k_nchw_to_nhwc_pad<bf16_t, 4>), g, dim3(256), 0, s, (const bf16_t*)x, (bf16_t*)y, C, HW, total);
    else hipLaunchKernelGGL((k_nchw_to_nhwc_pad<bf16_t, 8>), g, dim3(256), 0, s, (const bf16_t*)x, (bf16_t*)y, C, HW, total);
  }
  BIGDL_CHECK_LAUNCH();
}

// dtype: 0 = fp32 input, 1 = bf16 input
BIGDL_EXPORT int bigdl_nchw_to_nhwc_bf16(const void* x, int dtype, void* y, int N, int C, long long HW,
                                         hipStream_t s) {
  if (N <= 0 || C <= 0 || HW <= 0 || N > 65535 || (C + 31) / 32 > 65535) return (int)hipErrorInvalidValue;
  const long long gx = (HW + 63) / 64;
  if (gx > 0x7fffffffLL) return (int)hipErrorInvalidValue;
  const dim3 g((unsigned)gx, (unsigned)((C + 31) / 32), (unsigned)N);
  if (dtype == 0)
    hipLaunchKernelGGL((k_nchw_to_nhwc<float>), g, dim3(256), 0, s, (const float*)x, (bf16_t*)y, C, HW);
  else
    hipLaunchKernelGGL((k_nchw_to_nhwc<bf16_t>), g, dim3(256), 0, s, (const bf16_t*)x, (bf16_t*)y, C, HW);
  BIGDL_CHECK_LAUNCH();
}
