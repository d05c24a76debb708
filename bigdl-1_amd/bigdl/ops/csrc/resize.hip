// Bilinear resize with the reference's TensorFlow-style sampling (nn/ResizeBilinear.scala:266-284,
// 406-412): source coordinate = dst · scale with scale = in/out (or (in−1)/(out−1) with
// alignCorners), lower = ⌊src⌋, upper = min(lower + 1, in − 1), lerp = src − lower — NO half-pixel
// offset.  NHWC bf16, 8 channels (one 16-B chunk) per thread; the backward scatters each output
// gradient into its four source pixels with fp32 atomics (gx32, zeroed by the caller).
#include "common.h"

struct ResizeP {
  const bf16_t* x;
  bf16_t* y;
  const bf16_t* gy;
  float* gx;
  int N, H, W, C, OH, OW;
  float sh, sw;
};

__device__ __forceinline__ void src_coord(int o, float scale, int in, int& lo, int& hi, float& l) {
  const float s = (float)o * scale;
  lo = (int)s;  // s ≥ 0: truncation = floor, as the reference's toInt
  if (lo > in - 1) lo = in - 1;
  hi = lo + 1 < in ? lo + 1 : in - 1;
  l = s - (float)lo;
}

__global__ void __launch_bounds__(256) k_resize_bilinear_fwd(ResizeP p) {
  const int CG = p.C >> 3;
  const long long total = (long long)p.N * p.OH * p.OW * CG;
  for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < total; i += (long long)gridDim.x * 256) {
    const int cg = (int)(i % CG);
    long long r = i / CG;
    const int ox = (int)(r % p.OW);
    r /= p.OW;
    const int oy = (int)(r % p.OH);
    const int n = (int)(r / p.OH);
    int y0, y1, x0, x1;
    float ly, lx;
    src_coord(oy, p.sh, p.H, y0, y1, ly);
    src_coord(ox, p.sw, p.W, x0, x1, lx);
    const bf16_t* base = p.x + (long long)n * p.H * p.W * p.C + cg * 8;
    float tl[8], tr[8], bl[8], br[8], o[8];
    load8(base + ((long long)y0 * p.W + x0) * p.C, tl);
    load8(base + ((long long)y0 * p.W + x1) * p.C, tr);
    load8(base + ((long long)y1 * p.W + x0) * p.C, bl);
    load8(base + ((long long)y1 * p.W + x1) * p.C, br);
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const float top = tl[k] + (tr[k] - tl[k]) * lx;
      const float bot = bl[k] + (br[k] - bl[k]) * lx;
      o[k] = top + (bot - top) * ly;
    }
    store8(p.y + (((long long)n * p.OH + oy) * p.OW + ox) * p.C + cg * 8, o);
  }
}

__global__ void __launch_bounds__(256) k_resize_bilinear_bwd(ResizeP p) {
  const int CG = p.C >> 3;
  const long long total = (long long)p.N * p.OH * p.OW * CG;
  for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < total; i += (long long)gridDim.x * 256) {
    const int cg = (int)(i % CG);
    long long r = i / CG;
    const int ox = (int)(r % p.OW);
    r /= p.OW;
    const int oy = (int)(r % p.OH);
    const int n = (int)(r / p.OH);
    int y0, y1, x0, x1;
    float ly, lx;
    src_coord(oy, p.sh, p.H, y0, y1, ly);
    src_coord(ox, p.sw, p.W, x0, x1, lx);
    float g[8];
    load8(p.gy + (((long long)n * p.OH + oy) * p.OW + ox) * p.C + cg * 8, g);
    float* base = p.gx + (long long)n * p.H * p.W * p.C + cg * 8;
    const float w00 = (1.f - ly) * (1.f - lx), w01 = (1.f - ly) * lx, w10 = ly * (1.f - lx), w11 = ly * lx;
    float* q00 = base + ((long long)y0 * p.W + x0) * p.C;
    float* q01 = base + ((long long)y0 * p.W + x1) * p.C;
    float* q10 = base + ((long long)y1 * p.W + x0) * p.C;
    float* q11 = base + ((long long)y1 * p.W + x1) * p.C;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      atomicAdd(q00 + k, g[k] * w00);
      atomicAdd(q01 + k, g[k] * w01);
      atomicAdd(q10 + k, g[k] * w10);
      atomicAdd(q11 + k, g[k] * w11);
    }
  }
}

static float resize_scale(int in, int out, int align) {
  return (align && out > 1) ? (float)(in - 1) / (float)(out - 1) : (float)in / (float)out;
}

static int resize_grid(long long total) {
  long long b = (total + 255) / 256;
  if (b > 4096) b = 4096;
  return (int)(b < 1 ? 1 : b);
}

// x [N][H][W][C] bf16 → y [N][OH][OW][C] bf16.  C % 8 == 0, 16-B aligned.
BIGDL_EXPORT int bigdl_resize_bilinear_fwd(const void* x, void* y, int N, int H, int W, int C, int OH, int OW,
                                           int align, hipStream_t s) {
  if (N <= 0 || H <= 0 || W <= 0 || C <= 0 || C % 8 || OH <= 0 || OW <= 0) return (int)hipErrorInvalidValue;
  if (((uintptr_t)x & 15) || ((uintptr_t)y & 15)) return (int)hipErrorInvalidValue;
  ResizeP p{};
  p.x = (const bf16_t*)x; p.y = (bf16_t*)y; p.N = N; p.H = H; p.W = W; p.C = C; p.OH = OH; p.OW = OW;
  p.sh = resize_scale(H, OH, align); p.sw = resize_scale(W, OW, align);
  hipLaunchKernelGGL(k_resize_bilinear_fwd, dim3(resize_grid((long long)N * OH * OW * (C / 8))), dim3(256), 0, s, p);
  BIGDL_CHECK_LAUNCH();
}

// gx32 [N][H][W][C] fp32 (zeroed by the caller) += resize backward of gy [N][OH][OW][C] bf16.
BIGDL_EXPORT int bigdl_resize_bilinear_bwd(const void* gy, float* gx32, int N, int H, int W, int C, int OH, int OW,
                                           int align, hipStream_t s) {
  if (N <= 0 || H <= 0 || W <= 0 || C <= 0 || C % 8 || OH <= 0 || OW <= 0) return (int)hipErrorInvalidValue;
  if (((uintptr_t)gy & 15) || ((uintptr_t)gx32 & 15)) return (int)hipErrorInvalidValue;
  ResizeP p{};
  p.gy = (const bf16_t*)gy; p.gx = gx32; p.N = N; p.H = H; p.W = W; p.C = C; p.OH = OH; p.OW = OW;
  p.sh = resize_scale(H, OH, align); p.sw = resize_scale(W, OW, align);
  hipLaunchKernelGGL(k_resize_bilinear_bwd, dim3(resize_grid((long long)N * OH * OW * (C / 8))), dim3(256), 0, s, p);
  BIGDL_CHECK_LAUNCH();
}
