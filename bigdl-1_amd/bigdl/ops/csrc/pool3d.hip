// 3-D max / average pooling (VolumetricMaxPooling.scala, VolumetricAveragePooling.scala) on NDHWC
// bf16: one thread per (output voxel, 8-channel chunk) — 16-B loads along the channel-contiguous
// layout.  Max pooling keeps the window-linear argmax per channel (uint8, window ≤ 255) for the
// backward; both backwards scatter into an fp32 input-gradient buffer with atomics (windows may
// overlap), which the caller zeroes and casts.
#include "common.h"

struct Pool3P {
  const bf16_t* x;
  bf16_t* y;
  uint8_t* idx;
  const bf16_t* gy;
  float* gx;
  int N, T, H, W, C, OT, OH, OW;
  int kt, kh, kw, st, sh, sw, pt, ph, pw;
  int count_include_pad;
};

__device__ __forceinline__ void decode(long long i, const Pool3P& p, int& n, int& ot, int& oh, int& ow, int& cg) {
  const int CG = p.C >> 3;
  cg = (int)(i % CG);
  long long r = i / CG;
  ow = (int)(r % p.OW);
  r /= p.OW;
  oh = (int)(r % p.OH);
  r /= p.OH;
  ot = (int)(r % p.OT);
  n = (int)(r / p.OT);
}

__device__ __forceinline__ long long out_off(const Pool3P& p, int n, int ot, int oh, int ow, int cg) {
  return ((((long long)n * p.OT + ot) * p.OH + oh) * p.OW + ow) * p.C + cg * 8;
}

__device__ __forceinline__ long long in_off(const Pool3P& p, int n, int t, int h, int w, int cg) {
  return ((((long long)n * p.T + t) * p.H + h) * p.W + w) * p.C + cg * 8;
}

// average divisor: the window clipped to the padded extent (count_include_pad) or to the input
__device__ __forceinline__ float avg_div(const Pool3P& p, int t0, int h0, int w0) {
  if (p.count_include_pad) {
    const int t1 = min(t0 + p.kt, p.T + p.pt), h1 = min(h0 + p.kh, p.H + p.ph), w1 = min(w0 + p.kw, p.W + p.pw);
    return (float)((t1 - t0) * (h1 - h0) * (w1 - w0));
  }
  const int ta = max(t0, 0), ha = max(h0, 0), wa = max(w0, 0);
  const int tb = min(t0 + p.kt, p.T), hb = min(h0 + p.kh, p.H), wb = min(w0 + p.kw, p.W);
  return (float)(max(tb - ta, 0) * max(hb - ha, 0) * max(wb - wa, 0));
}

template <bool MAX>
__global__ void __launch_bounds__(256) k_pool3d_fwd(Pool3P p) {
  const long long total = (long long)p.N * p.OT * p.OH * p.OW * (p.C >> 3);
  for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < total; i += (long long)gridDim.x * 256) {
    int n, ot, oh, ow, cg;
    decode(i, p, n, ot, oh, ow, cg);
    const int t0 = ot * p.st - p.pt, h0 = oh * p.sh - p.ph, w0 = ow * p.sw - p.pw;
    float acc[8];
    int arg[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      acc[k] = MAX ? -INFINITY : 0.f;
      arg[k] = 0;
    }
    for (int a = 0; a < p.kt; ++a) {
      const int t = t0 + a;
      if ((unsigned)t >= (unsigned)p.T) continue;
      for (int b = 0; b < p.kh; ++b) {
        const int h = h0 + b;
        if ((unsigned)h >= (unsigned)p.H) continue;
        for (int c = 0; c < p.kw; ++c) {
          const int w = w0 + c;
          if ((unsigned)w >= (unsigned)p.W) continue;
          float v[8];
          load8(p.x + in_off(p, n, t, h, w, cg), v);
          const int widx = (a * p.kh + b) * p.kw + c;
#pragma unroll
          for (int k = 0; k < 8; ++k) {
            if (MAX) {
              if (v[k] > acc[k] || (v[k] != v[k])) {  // NaN propagates, as max_pool
                acc[k] = v[k];
                arg[k] = widx;
              }
            } else {
              acc[k] += v[k];
            }
          }
        }
      }
    }
    const long long o = out_off(p, n, ot, oh, ow, cg);
    if (MAX) {
      uint32_t lo = 0, hi = 0;
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        lo |= (uint32_t)(arg[k] & 0xFF) << (8 * k);
        hi |= (uint32_t)(arg[k + 4] & 0xFF) << (8 * k);
      }
      *reinterpret_cast<uint2*>(p.idx + o) = make_uint2(lo, hi);
    } else {
      const float d = avg_div(p, t0, h0, w0);
      const float r = d > 0.f ? 1.f / d : 0.f;
#pragma unroll
      for (int k = 0; k < 8; ++k) acc[k] *= r;
    }
    store8(p.y + o, acc);
  }
}

template <bool MAX>
__global__ void __launch_bounds__(256) k_pool3d_bwd(Pool3P p) {
  const long long total = (long long)p.N * p.OT * p.OH * p.OW * (p.C >> 3);
  for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < total; i += (long long)gridDim.x * 256) {
    int n, ot, oh, ow, cg;
    decode(i, p, n, ot, oh, ow, cg);
    const int t0 = ot * p.st - p.pt, h0 = oh * p.sh - p.ph, w0 = ow * p.sw - p.pw;
    const long long o = out_off(p, n, ot, oh, ow, cg);
    float g[8];
    load8(p.gy + o, g);
    if (MAX) {
      const uint2 ab = *reinterpret_cast<const uint2*>(p.idx + o);
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const int widx = (int)(((k < 4 ? ab.x : ab.y) >> (8 * (k & 3))) & 0xFF);
        const int c = widx % p.kw, b = (widx / p.kw) % p.kh, a = widx / (p.kw * p.kh);
        const int t = t0 + a, h = h0 + b, w = w0 + c;
        if ((unsigned)t < (unsigned)p.T && (unsigned)h < (unsigned)p.H && (unsigned)w < (unsigned)p.W)
          atomicAdd(p.gx + in_off(p, n, t, h, w, cg) + k, g[k]);
      }
    } else {
      const float d = avg_div(p, t0, h0, w0);
      const float r = d > 0.f ? 1.f / d : 0.f;
      for (int a = 0; a < p.kt; ++a) {
        const int t = t0 + a;
        if ((unsigned)t >= (unsigned)p.T) continue;
        for (int b = 0; b < p.kh; ++b) {
          const int h = h0 + b;
          if ((unsigned)h >= (unsigned)p.H) continue;
          for (int c = 0; c < p.kw; ++c) {
            const int w = w0 + c;
            if ((unsigned)w >= (unsigned)p.W) continue;
            float* q = p.gx + in_off(p, n, t, h, w, cg);
#pragma unroll
            for (int k = 0; k < 8; ++k) atomicAdd(q + k, g[k] * r);
          }
        }
      }
    }
  }
}

static int pool3_grid(long long total) {
  long long b = (total + 255) / 256;
  if (b > 8192) b = 8192;
  return (int)(b < 1 ? 1 : b);
}

static bool pool3_ok(int N, int T, int H, int W, int C, int OT, int OH, int OW, int kt, int kh, int kw, int st, int sh,
                     int sw) {
  return N > 0 && T > 0 && H > 0 && W > 0 && C > 0 && C % 8 == 0 && OT > 0 && OH > 0 && OW > 0 && kt > 0 &&
         kh > 0 && kw > 0 && st > 0 && sh > 0 && sw > 0 && kt * kh * kw <= 255;
}

// mode 0 = max (idx: uint8 [N][OT][OH][OW][C]), 1 = average.  x [N][T][H][W][C] bf16 → y.
BIGDL_EXPORT int bigdl_pool3d_fwd(int mode, const void* x, void* y, void* idx, int N, int T, int H, int W, int C,
                                  int OT, int OH, int OW, int kt, int kh, int kw, int st, int sh, int sw, int pt,
                                  int ph, int pw, int count_include_pad, hipStream_t s) {
  if (!pool3_ok(N, T, H, W, C, OT, OH, OW, kt, kh, kw, st, sh, sw) || (mode == 0 && !idx)) return (int)hipErrorInvalidValue;
  if (((uintptr_t)x & 15) || ((uintptr_t)y & 15) || ((uintptr_t)idx & 7)) return (int)hipErrorInvalidValue;
  Pool3P p{};
  p.x = (const bf16_t*)x; p.y = (bf16_t*)y; p.idx = (uint8_t*)idx;
  p.N = N; p.T = T; p.H = H; p.W = W; p.C = C; p.OT = OT; p.OH = OH; p.OW = OW;
  p.kt = kt; p.kh = kh; p.kw = kw; p.st = st; p.sh = sh; p.sw = sw; p.pt = pt; p.ph = ph; p.pw = pw;
  p.count_include_pad = count_include_pad;
  const dim3 g(pool3_grid((long long)N * OT * OH * OW * (C / 8)));
  if (mode == 0) hipLaunchKernelGGL(k_pool3d_fwd<true>, g, dim3(256), 0, s, p);
  else hipLaunchKernelGGL(k_pool3d_fwd<false>, g, dim3(256), 0, s, p);
  BIGDL_CHECK_LAUNCH();
}

// gx32 [N][T][H][W][C] fp32 (zeroed by the caller) += pooling backward of gy.
BIGDL_EXPORT int bigdl_pool3d_bwd(int mode, const void* gy, const void* idx, float* gx32, int N, int T, int H, int W,
                                  int C, int OT, int OH, int OW, int kt, int kh, int kw, int st, int sh, int sw, int pt,
                                  int ph, int pw, int count_include_pad, hipStream_t s) {
  if (!pool3_ok(N, T, H, W, C, OT, OH, OW, kt, kh, kw, st, sh, sw) || (mode == 0 && !idx)) return (int)hipErrorInvalidValue;
  if (((uintptr_t)gy & 15) || ((uintptr_t)gx32 & 15) || ((uintptr_t)idx & 7)) return (int)hipErrorInvalidValue;
  Pool3P p{};
  p.gy = (const bf16_t*)gy; p.idx = (uint8_t*)idx; p.gx = gx32;
  p.N = N; p.T = T; p.H = H; p.W = W; p.C = C; p.OT = OT; p.OH = OH; p.OW = OW;
  p.kt = kt; p.kh = kh; p.kw = kw; p.st = st; p.sh = sh; p.sw = sw; p.pt = pt; p.ph = ph; p.pw = pw;
  p.count_include_pad = count_include_pad;
  const dim3 g(pool3_grid((long long)N * OT * OH * OW * (C / 8)));
  if (mode == 0) hipLaunchKernelGGL(k_pool3d_bwd<true>, g, dim3(256), 0, s, p);
  else hipLaunchKernelGGL(k_pool3d_bwd<false>, g, dim3(256), 0, s, p);
  BIGDL_CHECK_LAUNCH();
}
