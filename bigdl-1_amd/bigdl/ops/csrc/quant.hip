// int8 inference path (K26): per-window symmetric quantisation + int8 MFMA GEMM with fused
// dequantisation — the MI355X equivalent of BigQuant's FCDataInit/ConvDataInit + MixPrecisionGEMM
// (DL/nn/quantized/{Linear,SpatialConvolution}.scala, Quantization.scala:26-180).
//
// Quantisation (Quantization.quantize): q = round(v / max(|max|, |min|) · 127) with Java's
// Math.round (half-up), one scale per window = row of the GEMM operand (an FC input row, a conv
// im2col window, a weight output channel).  Rows are zero-padded to Kp (multiple of 64).
//
// GEMM: C[m][n] = (Σ_k A[m][k]·B[n][k]) · sa[m] · sb[n] + bias[n], A/B int8 K-contiguous,
// accumulated exactly in int32 by v_mfma_i32_16x16x64_i8 (2× the bf16 MFMA rate).  Tile 128×128×128,
// 4 waves (2×2) of 4×4 16×16 tiles, LDS rows of 128 B with the 16-B-chunk XOR swizzle used by the
// conv kernels, double-buffered, one barrier per k-tile, XCD-aware tile order.
#include "common.h"

typedef int v4i __attribute__((ext_vector_type(4)));

__device__ __forceinline__ float round_half_up(float x) { return floorf(x + 0.5f); }

// one wave per row: amax reduction, then quantise; T = float or bf16
template <typename T>
__device__ __forceinline__ float ld(const T* p, long long i);
template <>
__device__ __forceinline__ float ld<float>(const float* p, long long i) { return p[i]; }
template <>
__device__ __forceinline__ float ld<bf16_t>(const bf16_t* p, long long i) { return bf2f(p[i]); }

template <typename T>
__global__ void __launch_bounds__(256) k_quant_rows(const T* __restrict__ src, long long M, int K, long long ld_src,
                                                    int8_t* __restrict__ dst, int Kp, float* __restrict__ scale) {
  const int lane = threadIdx.x & 63;
  const long long row = (long long)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= M) return;
  const T* s = src + row * ld_src;
  float mx = -INFINITY, mn = INFINITY;
  for (int k = lane; k < K; k += 64) {
    float v = ld<T>(s, k);
    mx = fmaxf(mx, v);
    mn = fminf(mn, v);
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    mx = fmaxf(mx, __shfl_xor(mx, o, 64));
    mn = fminf(mn, __shfl_xor(mn, o, 64));
  }
  const float amax = fmaxf(fabsf(mx), fabsf(mn));
  const float inv = amax > 0.f ? 127.f / amax : 0.f;
  int8_t* d = dst + row * (long long)Kp;
  for (int k = lane; k < Kp; k += 64) {
    float q = k < K ? round_half_up(ld<T>(s, k) * inv) : 0.f;
    q = fminf(fmaxf(q, -127.f), 127.f);
    d[k] = (int8_t)q;
  }
  if (lane == 0) scale[row] = amax / 127.f;
}

constexpr int QBM = 128, QBN = 128, QBK = 128;

__device__ __forceinline__ int qswz(int row, int chunk) { return row * QBK + ((chunk ^ (row & 7)) << 4); }

__device__ __forceinline__ int q_xcd_remap(int bid, int nwg) {
  const int xcd = bid & 7, q = nwg >> 3, r = nwg & 7;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (bid >> 3);
}

// Epilogue of the int8 GEMM (direct or after the split-K sum): v = acc·sa[m]·sb[n] + bias[n] (sa == null:
// the uniform activation scale sa0 of a statically quantised input), ReLU, then fp32 / bf16 out, or —
// out_q > 0 — the next quantised layer's int8 input at scale out_q (signed, or the offset unsigned code
// of a ReLU'd output when out_u8; round half up as quant_static).
struct QEpi {
  const float* sa;
  float sa0;
  const float* sb;
  const float* bias;
  void* out;
  int out_bf16, relu;
  float out_q;
  int out_u8;
};

__device__ __forceinline__ void q_epi_store(const QEpi& e, int m, int n, int N, int acc) {
  float v = (float)acc * (e.sa ? e.sa[m] : e.sa0) * e.sb[n] + (e.bias ? e.bias[n] : 0.f);
  if (e.relu) v = fmaxf(v, 0.f);
  const size_t o = (size_t)m * N + n;
  if (e.out_q > 0.f) {
    float q = round_half_up(v / e.out_q);
    if (e.out_u8) {
      q = fminf(fmaxf(q, 0.f), 255.f) - 128.f;
    } else {
      q = fminf(fmaxf(q, -127.f), 127.f);
    }
    reinterpret_cast<int8_t*>(e.out)[o] = (int8_t)q;
  } else if (e.out_bf16) {
    reinterpret_cast<bf16_t*>(e.out)[o] = f2bf(v);
  } else {
    reinterpret_cast<float*>(e.out)[o] = v;
  }
}

// partial: null = direct epilogue; else split-K (gridDim.y splits of kt_split k-tiles each), the raw
// int32 sums of split blockIdx.y land in partial[split][M][N] (summed exactly by k_gemm_i8_epi)
__global__ void __launch_bounds__(256, 2)
k_gemm_i8(const int8_t* __restrict__ A, const int8_t* __restrict__ B, int M, int N, int Kp, QEpi ep, int tiles_n,
          int kt_split, int* __restrict__ partial) {
  __shared__ __attribute__((aligned(16))) int8_t lds[2][(QBM + QBN) * QBK];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wave_m = wid & 1, wave_n = wid >> 1;
  const int tile = q_xcd_remap(blockIdx.x, gridDim.x);
  const int tm = tile / tiles_n, tn = tile - tm * tiles_n;
  const int m0 = tm * QBM, n0 = tn * QBN;
  const int col = tid & 7;  // 16-B chunk in a 128-B k row
  uint4 ra[4], rb[4];
  const int KTall = Kp / QBK + (Kp % QBK ? 1 : 0);
  const int kt0 = blockIdx.y * kt_split;
  const int KT = (KTall - kt0) < kt_split ? (KTall - kt0) : kt_split;
  A += (size_t)kt0 * QBK;
  B += (size_t)kt0 * QBK;
  const int Kl = Kp - kt0 * QBK;  // k extent left from this split's start

  auto load = [&](int kt) {
    const int k = kt * QBK + col * 16;
    const bool kin = k < Kl;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int r = (tid >> 3) + 32 * i;
      const int m = m0 + r, n = n0 + r;
      ra[i] = (kin && m < M) ? *reinterpret_cast<const uint4*>(A + (size_t)m * Kp + k) : make_uint4(0, 0, 0, 0);
      rb[i] = (kin && n < N) ? *reinterpret_cast<const uint4*>(B + (size_t)n * Kp + k) : make_uint4(0, 0, 0, 0);
    }
  };
  auto store = [&](int buf) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int r = (tid >> 3) + 32 * i;
      *reinterpret_cast<uint4*>(&lds[buf][qswz(r, col)]) = ra[i];
      *reinterpret_cast<uint4*>(&lds[buf][qswz(QBM + r, col)]) = rb[i];
    }
  };

  v4i acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = v4i{0, 0, 0, 0};

  load(0);
  store(0);
  __syncthreads();
  const int fr = lane & 15, fq = lane >> 4;
  for (int kt = 0; kt < KT; ++kt) {
    const int buf = kt & 1;
    if (kt + 1 < KT) load(kt + 1);
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      const int chunk = kk * 4 + fq;  // lane holds k = 64·kk + 16·fq + [0, 16)
      v4i af[4], bfr[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) af[i] = *reinterpret_cast<const v4i*>(&lds[buf][qswz(QBM + wave_n * 64 + i * 16 + fr, chunk)]);
#pragma unroll
      for (int j = 0; j < 4; ++j) bfr[j] = *reinterpret_cast<const v4i*>(&lds[buf][qswz(wave_m * 64 + j * 16 + fr, chunk)]);
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = __builtin_amdgcn_mfma_i32_16x16x64_i8(af[i], bfr[j], acc[i][j], 0, 0, 0);
    }
    if (kt + 1 < KT) store(buf ^ 1);
    __syncthreads();
  }
  // acc[i][j][e]: row (of the weight operand) = n, col = m; D layout row=(lane>>4)*4+e, col=lane&15
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int nb = n0 + wave_n * 64 + i * 16 + fq * 4;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int m = m0 + wave_m * 64 + j * 16 + fr;
      if (m >= M) continue;
      if (partial) {
        int* pr = partial + ((size_t)blockIdx.y * M + m) * N;
        if (nb + 3 < N && (N & 3) == 0) {
          *reinterpret_cast<v4i*>(pr + nb) = acc[i][j];
        } else {
#pragma unroll
          for (int e = 0; e < 4; ++e)
            if (nb + e < N) pr[nb + e] = acc[i][j][e];
        }
        continue;
      }
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int n = nb + e;
        if (n < N) q_epi_store(ep, m, n, N, acc[i][j][e]);
      }
    }
  }
}

// split-K epilogue: exact int32 sum of the splits' partial slabs, then the GEMM epilogue
__global__ void __launch_bounds__(256) k_gemm_i8_epi(const int* __restrict__ partial, int splits, int M, int N,
                                                     QEpi ep) {
  const long long i = (long long)blockIdx.x * 256 + threadIdx.x;
  if (i >= (long long)M * N) return;
  const size_t MN = (size_t)M * N;
  int acc = 0;
  for (int sp = 0; sp < splits; ++sp) acc += partial[sp * MN + i];
  q_epi_store(ep, (int)(i / N), (int)(i % N), N, acc);
}

BIGDL_EXPORT int bigdl_quant_rows(const void* src, int src_bf16, long long M, int K, long long ld_src, void* dst,
                                  int Kp, float* scale, hipStream_t s) {
  if (M <= 0 || K <= 0 || Kp < K || Kp % 16) return (int)hipErrorInvalidValue;
  const long long blocks = (M + 3) / 4;
  if (blocks > 0x7fffffffLL) return (int)hipErrorInvalidValue;
  if (src_bf16)
    hipLaunchKernelGGL(k_quant_rows<bf16_t>, dim3((unsigned)blocks), dim3(256), 0, s, (const bf16_t*)src, M, K, ld_src,
                       (int8_t*)dst, Kp, scale);
  else
    hipLaunchKernelGGL(k_quant_rows<float>, dim3((unsigned)blocks), dim3(256), 0, s, (const float*)src, M, K, ld_src,
                       (int8_t*)dst, Kp, scale);
  BIGDL_CHECK_LAUNCH();
}

// A: [M][Kp] int8 (activations, row scales sa), B: [N][Kp] int8 (weights, row scales sb).
BIGDL_EXPORT int bigdl_gemm_i8(const void* A, const void* B, int M, int N, int Kp, const float* sa, const float* sb,
                               const float* bias, void* out, int out_bf16, int relu, hipStream_t s) {
  if (M <= 0 || N <= 0 || Kp <= 0 || Kp % 16 || !sa) return (int)hipErrorInvalidValue;
  const int tiles_n = (N + QBN - 1) / QBN;
  const long long tiles = (long long)((M + QBM - 1) / QBM) * tiles_n;
  if (tiles > 0x7fffffffLL) return (int)hipErrorInvalidValue;
  QEpi ep{sa, 0.f, sb, bias, out, out_bf16, relu, 0.f, 0};
  const int KT = (Kp + QBK - 1) / QBK;
  hipLaunchKernelGGL(k_gemm_i8, dim3((unsigned)tiles), dim3(256), 0, s, (const int8_t*)A, (const int8_t*)B, M, N, Kp,
                     ep, tiles_n, KT, (int*)nullptr);
  BIGDL_CHECK_LAUNCH();
}

// The classifier-head form: sa == null → every row has the activation scale sa0 (a statically
// quantised input); out_q > 0 → int8 output for the next quantised layer (out_u8: offset unsigned
// code); splits > 1 → split-K over `splits` slabs of `work` ([splits][M][N] int32; small-M, long-K
// products such as VGG16 fc6, which on whole-K tiles would run 32 workgroups on 256 CUs).
BIGDL_EXPORT int bigdl_gemm_i8_ex(const void* A, const void* B, int M, int N, int Kp, const float* sa, float sa0,
                                  const float* sb, const float* bias, void* out, int out_bf16, int relu, float out_q,
                                  int out_u8, int splits, void* work, hipStream_t s) {
  if (M <= 0 || N <= 0 || Kp <= 0 || Kp % 16 || (!sa && !(sa0 > 0.f)) || splits < 1 || (splits > 1 && !work))
    return (int)hipErrorInvalidValue;
  const int tiles_n = (N + QBN - 1) / QBN;
  const long long tiles = (long long)((M + QBM - 1) / QBM) * tiles_n;
  if (tiles > 0x7fffffffLL) return (int)hipErrorInvalidValue;
  QEpi ep{sa, sa0, sb, bias, out, out_bf16, relu, out_q, out_u8};
  const int KT = (Kp + QBK - 1) / QBK;
  if (splits > KT) splits = KT;
  const int kts = (KT + splits - 1) / splits;
  splits = (KT + kts - 1) / kts;  // every split has at least one k-tile
  if (splits == 1) {
    hipLaunchKernelGGL(k_gemm_i8, dim3((unsigned)tiles), dim3(256), 0, s, (const int8_t*)A, (const int8_t*)B, M, N, Kp,
                       ep, tiles_n, KT, (int*)nullptr);
    BIGDL_CHECK_LAUNCH();
  }
  hipLaunchKernelGGL(k_gemm_i8, dim3((unsigned)tiles, splits), dim3(256), 0, s, (const int8_t*)A, (const int8_t*)B, M,
                     N, Kp, ep, tiles_n, kts, (int*)work);
  const long long n = (long long)M * N;
  hipLaunchKernelGGL(k_gemm_i8_epi, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, (const int*)work, splits, M, N,
                     ep);
  BIGDL_CHECK_LAUNCH();
}
