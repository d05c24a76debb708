// fp32-accurate products on the bf16 MFMA pipes ("bf16x3").  The reference computes in fp32 (MKL
// sgemm / MKL-DNN fp32 primitives, DL/tensor/DenseTensorBLAS.scala:70-112,
// DL/nn/SpatialConvolution.scala:253-362).  CDNA4's fp32 MFMA (v_mfma_f32_16x16x4_f32) runs at
// 1/16 of the bf16 rate, so the fp32 compute mode instead splits every fp32 operand v into
//   hi = bf16(v), lo = bf16(v − hi)          (|v − hi − lo| ≤ 2^-16 |v|)
// and evaluates a·b ≈ a_hi·b_hi + a_hi·b_lo + a_lo·b_hi (the dropped a_lo·b_lo term is ≤ 2^-16
// relative) with fp32 accumulation — three bf16 MFMAs per product, 5.3× the fp32-MFMA rate.
// The three products become ONE GEMM / implicit-GEMM conv by concatenating the parts along the
// reduction dimension: A' = [a_hi | a_hi | a_lo], B' = [b_hi | b_lo | b_hi], Σ_k' A'·B' = the sum
// above.  This file holds the split; the GEMM (gemm.hip, fp32 C) and the conv kernels
// (conv_igemm.hip, ConvParams::y32 fp32 output; conv_wgrad.hip, fp32 accumulation) do the rest.
#include "common.h"

typedef float f4v __attribute__((ext_vector_type(4)));

// src: `rows` rows of C fp32 values, row stride ld (elements).  dst: the three parts, each Cp ≥ C
// wide (zero beyond C), either side by side in one row (stacked = 0: dst row r = [p0 | p1 | p2],
// 3·Cp elements) or stacked along rows (stacked = 1: part q is rows [q·rows, (q+1)·rows)).  Bit q
// of `code` selects lo (1) or hi (0) for part q.  A block covers 256 / tpr rows per trip, tpr
// threads per row one 8-channel chunk each (no per-element index division; streaming-bound).
__global__ void __launch_bounds__(256) k_split_bf16x3(const float* __restrict__ src, long long rows, int C, long long ld,
                                                      int Cp, bf16_t* __restrict__ dst, int code, int stacked,
                                                      int vec4, int nparts) {
  const int chunks = Cp / 8;
  const int tpr = chunks < 256 ? chunks : 256;
  const int rpi = 256 / tpr;
  const int tl = threadIdx.x % tpr, rl = threadIdx.x / tpr;
  if (rl >= rpi) return;
  const long long rstep = (long long)gridDim.x * rpi;
  for (long long r = (long long)blockIdx.x * rpi + rl; r < rows; r += rstep) {
    for (int ch = tl; ch < chunks; ch += tpr) {
      const int c0 = ch * 8;
      const float* sp = src + r * ld + c0;
      float v[8];
      if (vec4 && c0 + 8 <= C) {
        const f4v a = __builtin_nontemporal_load(reinterpret_cast<const f4v*>(sp));
        const f4v b = __builtin_nontemporal_load(reinterpret_cast<const f4v*>(sp + 4));
#pragma unroll
        for (int e = 0; e < 4; ++e) { v[e] = a[e]; v[4 + e] = b[e]; }
      } else {
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] = c0 + e < C ? sp[e] : 0.f;
      }
      uint32_t hw[4], lw[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const bf16_t h0 = f2bf(v[2 * e]), h1 = f2bf(v[2 * e + 1]);
        const bf16_t l0 = f2bf(v[2 * e] - bf2f(h0)), l1 = f2bf(v[2 * e + 1] - bf2f(h1));
        hw[e] = (uint32_t)h0 | ((uint32_t)h1 << 16);
        lw[e] = (uint32_t)l0 | ((uint32_t)l1 << 16);
      }
      const uint4 H = make_uint4(hw[0], hw[1], hw[2], hw[3]), L = make_uint4(lw[0], lw[1], lw[2], lw[3]);
#pragma unroll
      for (int q = 0; q < 3; ++q) {
        if (q >= nparts) break;
        const size_t off = stacked ? ((size_t)(q * rows + r) * Cp + c0) : ((size_t)r * nparts * Cp + (size_t)q * Cp + c0);
        *reinterpret_cast<uint4*>(dst + off) = ((code >> q) & 1) ? L : H;
      }
    }
  }
}

BIGDL_EXPORT int bigdl_split_bf16x3(const float* src, long long rows, int C, long long ld, int Cp, void* dst, int code,
                                    int stacked, hipStream_t s) {
  if (rows <= 0 || C <= 0 || Cp < C || Cp % 8 || ld < C || code < 0 || code > 7 || ((uintptr_t)dst & 15))
    return (int)hipErrorInvalidValue;
  const int vec4 = (ld % 4 == 0 && ((uintptr_t)src & 15) == 0) ? 1 : 0;
  const int chunks = Cp / 8, tpr = chunks < 256 ? chunks : 256, rpi = 256 / tpr;
  long long grid = (rows + rpi - 1) / rpi;
  if (grid > 2048) grid = 2048;
  hipLaunchKernelGGL(k_split_bf16x3, dim3((unsigned)grid), dim3(256), 0, s, src, rows, C, ld, Cp, (bf16_t*)dst, code,
                     stacked, vec4, 3);
  BIGDL_CHECK_LAUNCH();
}

// The two-part activation split [hi | lo] side by side ([rows][2·Cp]): the conv kernels read it as
// [hi | hi | lo] (ConvParams::cdup) and the weight-gradient kernels take hi / lo channel slices, so the
// duplicated hi part is never written (4 instead of 6 bytes out per element).
BIGDL_EXPORT int bigdl_split_bf16x2(const float* src, long long rows, int C, long long ld, int Cp, void* dst,
                                    hipStream_t s) {
  if (rows <= 0 || C <= 0 || Cp < C || Cp % 8 || ld < C || ((uintptr_t)dst & 15)) return (int)hipErrorInvalidValue;
  const int vec4 = (ld % 4 == 0 && ((uintptr_t)src & 15) == 0) ? 1 : 0;
  const int chunks = Cp / 8, tpr = chunks < 256 ? chunks : 256, rpi = 256 / tpr;
  long long grid = (rows + rpi - 1) / rpi;
  if (grid > 2048) grid = 2048;
  hipLaunchKernelGGL(k_split_bf16x3, dim3((unsigned)grid), dim3(256), 0, s, src, rows, C, ld, Cp, (bf16_t*)dst, 0b10, 0,
                     vec4, 2);
  BIGDL_CHECK_LAUNCH();
}

// Space-to-depth of a stride-2 convolution's input (the fp32 RGB stem on the direct kernels,
// csrc/conv_x3.hip, which need C % 32 == 0): x (any strides, element (n, c, h, w) at
// x + n·sn + c·sc + h·sh + w·sw) padded by (ph, pw) at the top / left and by zeros beyond, split into 2×2
// blocks: out[n][h2][w2][c·4 + bh·2 + bw] = xpad[n][c][2·h2 + bh][2·w2 + bw] for c < C, zero for the
// channels up to Cp (% 4 == 0).  A stride-2 R×S conv of x is then a stride-1 ⌈R/2⌉×⌈S/2⌉ conv of `out`
// with the filter rearranged the same way (ops/fp32x3.py _stem_weights).  One thread per output pixel.
__global__ void __launch_bounds__(256) k_s2d_f32(const float* __restrict__ x, long long sn, long long sc, long long sh,
                                                 long long sw, int N, int C, int H, int W, int ph, int pw, int H2,
                                                 int W2, int Cp, float* __restrict__ out) {
  // one thread per (output pixel, 4-channel group): consecutive lanes store consecutive 16 B
  const int G = Cp >> 2;
  const long long total = (long long)N * H2 * W2 * G;
  for (long long t = blockIdx.x * (long long)blockDim.x + threadIdx.x; t < total; t += (long long)gridDim.x * blockDim.x) {
    const int g = (int)(t % G);
    const long long pix = t / G;
    const int w2 = (int)(pix % W2);
    const long long r = pix / W2;
    const int h2 = (int)(r % H2);
    const int n = (int)(r / H2);
    float v[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int cc = 4 * g + e, c = cc >> 2, bh = (cc >> 1) & 1, bw = cc & 1;
      const int h = 2 * h2 + bh - ph, w = 2 * w2 + bw - pw;
      v[e] = (c < C && (unsigned)h < (unsigned)H && (unsigned)w < (unsigned)W)
                 ? x[n * sn + c * sc + h * sh + w * sw] : 0.f;
    }
    *reinterpret_cast<float4*>(out + t * 4) = make_float4(v[0], v[1], v[2], v[3]);
  }
}

// The RGB stem input for the C4 x3 / fp32 wgrad gathers: any-stride fp32 [N][C ≤ 4][H][W] → NHWC
// [N][H][W][4] fp32 (channels ≥ C zero): one 16-B store per pixel (the 7×7 stem then reduces over 49 taps
// × 4 channels = 196 → 224 indices instead of the s2d image's 16 taps × 32 padded channels = 512).
__global__ void __launch_bounds__(256) k_pad4_f32(const float* __restrict__ x, long long sn, long long sc,
                                                  long long sh, long long sw, int N, int C, int H, int W,
                                                  float* __restrict__ out) {
  const long long total = (long long)N * H * W;
  for (long long t = blockIdx.x * (long long)blockDim.x + threadIdx.x; t < total; t += (long long)gridDim.x * blockDim.x) {
    const int w = (int)(t % W);
    const long long r = t / W;
    const int h = (int)(r % H);
    const int n = (int)(r / H);
    const float* px = x + n * sn + h * sh + w * sw;
    float v[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) v[e] = e < C ? px[e * sc] : 0.f;
    *reinterpret_cast<float4*>(out + t * 4) = make_float4(v[0], v[1], v[2], v[3]);
  }
}

BIGDL_EXPORT int bigdl_pad4_f32(const float* x, long long sn, long long sc, long long sh, long long sw, int N, int C,
                                int H, int W, float* out, hipStream_t s) {
  if (!x || !out || N <= 0 || C <= 0 || C > 4 || H <= 0 || W <= 0 || ((uintptr_t)out & 15))
    return (int)hipErrorInvalidValue;
  const long long total = (long long)N * H * W;
  hipLaunchKernelGGL(k_pad4_f32, dim3(bigdl_grid(total, 256, 32768)), dim3(256), 0, s, x, sn, sc, sh, sw, N, C, H, W,
                     out);
  BIGDL_CHECK_LAUNCH();
}

BIGDL_EXPORT int bigdl_s2d_f32(const float* x, long long sn, long long sc, long long sh, long long sw, int N, int C,
                               int H, int W, int ph, int pw, int H2, int W2, int Cp, float* out, hipStream_t s) {
  if (!x || !out || N <= 0 || C <= 0 || H2 <= 0 || W2 <= 0 || Cp % 4 || 4 * C > Cp || ((uintptr_t)out & 15))
    return (int)hipErrorInvalidValue;
  const long long total = (long long)N * H2 * W2 * (Cp / 4);
  hipLaunchKernelGGL(k_s2d_f32, dim3(bigdl_grid(total, 256, 32768)), dim3(256), 0, s, x, sn, sc, sh, sw, N, C, H, W, ph,
                     pw, H2, W2, Cp, out);
  BIGDL_CHECK_LAUNCH();
}
