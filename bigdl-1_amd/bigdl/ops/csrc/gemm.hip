// Dense GEMM on MFMA (K4) with fused epilogues, plus the small helpers a Linear layer needs
// (weight transpose for backward-data, column sums for the bias gradient).
// Reference: Linear.updateOutput / updateGradInput (DL/nn/Linear.scala:108-158) and the MKL
// gemm wrappers (DL/tensor/DenseTensorBLAS.scala:70-112).
//
//   C[m][n] = act( alpha · Σ_k A[m][k] · B[n][k] + bias[n] + D[m][n] ) (+ beta · C[m][n], fp32 out)
//
// Both operands are k-contiguous rows ("NT"): A = activations [M][K] (row stride lda), B =
// weights [N][K] (ldb) — exactly Linear's x·Wᵀ.  Backward-data (gy·W) runs the same kernel on a
// transposed weight copy (k_transpose below, weights are small); the weight gradient gyᵀ·x is the
// 1×1 case of the convolution wgrad kernel (conv_wgrad.hip, transposed LDS reads + split-K).
//
// Tiling follows conv_igemm.hip: 256 threads = 4 waves (2 × 2), wave tile (BM/2) × (BN/2) of
// mfma_f32_16x16x32_bf16, operands staged global → registers → XOR-swizzled LDS, register sets
// two k-tiles ahead, one barrier per k-tile, XCD-contiguous block remap.  The MFMA "A" side is the
// weight row, so each lane's accumulator holds 4 CONSECUTIVE output columns of one row → 8-B bf16
// / 16-B fp32 stores straight from registers (no LDS round trip in the epilogue).
#include "common.h"

typedef short v8s __attribute__((ext_vector_type(8)));
typedef float v4f __attribute__((ext_vector_type(4)));

struct GemmParams {
  const bf16_t* a;
  const bf16_t* b;
  const float* bias;  // [N] or null
  const bf16_t* d;    // optional addend [M][N] (row stride ldd)
  void* c;
  long long lda, ldb, ldc, ldd;
  int M, N, K;
  int tiles_n;
  int act;      // 0 none, 1 relu, 2 sigmoid, 3 tanh
  int out_f32;  // 0: bf16 C, 1: fp32 C
  float alpha, beta;
  uint32_t a_bytes, b_bytes;
  // split-K (slab != null): block row blockIdx.y reduces K range [y·kchunk, (y+1)·kchunk) and stores
  // its raw fp32 partial tile into slab[y][M][N]; k_gemm_splitk_epi sums the slabs and applies the
  // epilogue.  For the small-M, long-K GEMMs (a classifier head: batch × 25088 · 4096) whose 64×64
  // tile grid alone fills half the CUs at most, each block walking all of K.
  float* slab;
  int kchunk;
};

template <int BK>
__device__ __forceinline__ int gswz(int row, int chunk) {
  if constexpr (BK == 64) return row * BK + ((chunk ^ (row & 7)) << 3);
  else return row * BK + ((chunk ^ ((row >> 2) & 2)) << 3);  // conflict-free for the b128 lane groups
}

__device__ __forceinline__ int gxcd_remap(int bid, int nwg) {
  const int xcd = bid & 7, q = nwg >> 3, r = nwg & 7;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (bid >> 3);
}

__device__ __forceinline__ float apply_act(float v, int act) {
  if (act == 1) return fmaxf(v, 0.f);
  if (act == 2) return 1.f / (1.f + __expf(-v));
  if (act == 3) return tanhf(v);
  return v;
}

template <int BM, int BN, int BK>
__global__ void __launch_bounds__(256, 2) k_gemm(GemmParams p) {
  constexpr int CPK = BK / 8;
  constexpr int RPS = 256 / CPK;
  constexpr int TN = BN / 32, TM = BM / 32;
  constexpr int A_CHUNKS = BM * BK / 8 / 256;
  constexpr int B_CHUNKS = BN * BK / 8 / 256;
  constexpr int STAGE = (BM + BN) * BK;
  __shared__ __attribute__((aligned(16))) bf16_t lds[2 * STAGE];

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wave_m = wid & 1, wave_n = wid >> 1;
  const int tile = gxcd_remap(blockIdx.x, gridDim.x);
  const int tm = tile / p.tiles_n, tn = tile - tm * p.tiles_n;
  const int m0 = tm * BM, n0 = tn * BN;
  const int col8 = tid & (CPK - 1);

  const __amdgpu_buffer_rsrc_t ar = __builtin_amdgcn_make_buffer_rsrc((void*)p.a, 0, (int)p.a_bytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t br = __builtin_amdgcn_make_buffer_rsrc((void*)p.b, 0, (int)p.b_bytes, 0x00020000);
  constexpr uint32_t OOB = 0x80000000u;

  uint32_t a_row[A_CHUNKS], b_row[B_CHUNKS];
#pragma unroll
  for (int i = 0; i < A_CHUNKS; ++i) {
    const int m = m0 + tid / CPK + RPS * i;
    a_row[i] = m < p.M ? (uint32_t)((long long)m * p.lda * 2) : OOB;
  }
#pragma unroll
  for (int i = 0; i < B_CHUNKS; ++i) {
    const int n = n0 + tid / CPK + RPS * i;
    b_row[i] = n < p.N ? (uint32_t)((long long)n * p.ldb * 2) : OOB;
  }
  const int kbeg = p.slab ? (int)blockIdx.y * p.kchunk : 0;
  const int kend = p.slab ? min(p.K, kbeg + p.kchunk) : p.K;
  const int KT = (kend - kbeg + BK - 1) / BK;

  // every load is issued (dead ones with an out-of-range offset that returns zero) so hipcc's
  // vmcnt accounting stays exact; the K tail inside a row is masked per 16-B chunk (K % 8 == 0)
  auto load_tile = [&](int kt, bool live, uint4 (&ra)[A_CHUNKS], uint4 (&rb)[B_CHUNKS]) {
    const int k = kbeg + kt * BK + col8 * 8;
    const bool kin = live && k < kend;
    const uint32_t kb = (uint32_t)k * 2u;
#pragma unroll
    for (int i = 0; i < A_CHUNKS; ++i) {
      const uint32_t off = (kin && a_row[i] != OOB) ? a_row[i] + kb : OOB;
      ra[i] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(ar, off, 0, 0));
    }
#pragma unroll
    for (int i = 0; i < B_CHUNKS; ++i) {
      const uint32_t off = (kin && b_row[i] != OOB) ? b_row[i] + kb : OOB;
      rb[i] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(br, off, 0, 0));
    }
  };
  auto store_tile = [&](int buf, const uint4 (&ra)[A_CHUNKS], const uint4 (&rb)[B_CHUNKS]) {
#pragma unroll
    for (int i = 0; i < A_CHUNKS; ++i)
      *reinterpret_cast<uint4*>(&lds[buf * STAGE + gswz<BK>(tid / CPK + RPS * i, col8)]) = ra[i];
#pragma unroll
    for (int i = 0; i < B_CHUNKS; ++i)
      *reinterpret_cast<uint4*>(&lds[buf * STAGE + gswz<BK>(BM + tid / CPK + RPS * i, col8)]) = rb[i];
  };

  v4f acc[TN][TM];
#pragma unroll
  for (int i = 0; i < TN; ++i)
#pragma unroll
    for (int j = 0; j < TM; ++j) acc[i][j] = v4f{0.f, 0.f, 0.f, 0.f};

  const int fr = lane & 15, fq = lane >> 4;
  auto compute = [&](int buf) {
#pragma unroll
    for (int kk = 0; kk < BK / 32; ++kk) {
      const int chunk = kk * 4 + fq;
      v8s af[TN], bfr[TM];
#pragma unroll
      for (int i = 0; i < TN; ++i)
        af[i] = *reinterpret_cast<const v8s*>(&lds[buf * STAGE + gswz<BK>(BM + wave_n * (BN / 2) + i * 16 + fr, chunk)]);
#pragma unroll
      for (int j = 0; j < TM; ++j)
        bfr[j] = *reinterpret_cast<const v8s*>(&lds[buf * STAGE + gswz<BK>(wave_m * (BM / 2) + j * 16 + fr, chunk)]);
#pragma unroll
      for (int i = 0; i < TN; ++i)
#pragma unroll
        for (int j = 0; j < TM; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
    }
  };

  uint4 ra0[A_CHUNKS], rb0[B_CHUNKS], ra1[A_CHUNKS], rb1[B_CHUNKS];
  load_tile(0, true, ra0, rb0);
  load_tile(1, KT > 1, ra1, rb1);
  store_tile(0, ra0, rb0);
  __syncthreads();
  int kt = 0;
  for (; kt + 2 <= KT; kt += 2) {
    load_tile(kt + 2, kt + 2 < KT, ra0, rb0);
    compute(0);
    store_tile(1, ra1, rb1);
    __syncthreads();
    load_tile(kt + 3, kt + 3 < KT, ra1, rb1);
    compute(1);
    if (kt + 2 < KT) store_tile(0, ra0, rb0);
    __syncthreads();
  }
  if (kt < KT) compute(0);

  // epilogue straight from the accumulators: lane → (row m, 4 consecutive columns n..n+3)
  if (p.slab) {  // split-K partial: raw fp32 sums, the epilogue runs after all slices
    float* sl = p.slab + (size_t)blockIdx.y * p.M * p.N;
#pragma unroll
    for (int i = 0; i < TN; ++i) {
      const int n = n0 + wave_n * (BN / 2) + i * 16 + fq * 4;
      if (n >= p.N) continue;
#pragma unroll
      for (int j = 0; j < TM; ++j) {
        const int m = m0 + wave_m * (BM / 2) + j * 16 + fr;
        if (m < p.M)
          *reinterpret_cast<float4*>(sl + (size_t)m * p.N + n) =
              make_float4(acc[i][j][0], acc[i][j][1], acc[i][j][2], acc[i][j][3]);
      }
    }
    return;
  }
#pragma unroll
  for (int i = 0; i < TN; ++i) {
    const int n = n0 + wave_n * (BN / 2) + i * 16 + fq * 4;
    if (n >= p.N) continue;  // N % 4 == 0: a column quad is all in or all out
    float b4[4] = {0.f, 0.f, 0.f, 0.f};
    if (p.bias) {
      const float4 bb = *reinterpret_cast<const float4*>(p.bias + n);
      b4[0] = bb.x; b4[1] = bb.y; b4[2] = bb.z; b4[3] = bb.w;
    }
#pragma unroll
    for (int j = 0; j < TM; ++j) {
      const int m = m0 + wave_m * (BM / 2) + j * 16 + fr;
      if (m >= p.M) continue;
      float v[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) v[e] = p.alpha * acc[i][j][e] + b4[e];
      if (p.d) {
        const uint2 dd = *reinterpret_cast<const uint2*>(p.d + (long long)m * p.ldd + n);
        v[0] += __uint_as_float(dd.x << 16);
        v[1] += __uint_as_float(dd.x & 0xFFFF0000u);
        v[2] += __uint_as_float(dd.y << 16);
        v[3] += __uint_as_float(dd.y & 0xFFFF0000u);
      }
      if (p.out_f32) {
        float* cp = reinterpret_cast<float*>(p.c) + (long long)m * p.ldc + n;
        if (p.beta != 0.f) {
          const float4 o = *reinterpret_cast<const float4*>(cp);
          v[0] += p.beta * o.x; v[1] += p.beta * o.y; v[2] += p.beta * o.z; v[3] += p.beta * o.w;
        }
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] = apply_act(v[e], p.act);
        *reinterpret_cast<float4*>(cp) = make_float4(v[0], v[1], v[2], v[3]);
      } else {
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] = apply_act(v[e], p.act);
        bf16_t* cp = reinterpret_cast<bf16_t*>(p.c) + (long long)m * p.ldc + n;
        *reinterpret_cast<uint2*>(cp) = make_uint2((uint32_t)f2bf(v[0]) | ((uint32_t)f2bf(v[1]) << 16),
                                                   (uint32_t)f2bf(v[2]) | ((uint32_t)f2bf(v[3]) << 16));
      }
    }
  }
}

static bool al(const void* q, int bytes) { return ((uintptr_t)q & (uintptr_t)(bytes - 1)) == 0; }

// Σ of the S split-K slabs, then alpha, bias, addend, beta·C, activation and the output dtype
__global__ void __launch_bounds__(256) k_gemm_splitk_epi(GemmParams p, int S) {
  const long long quads = (long long)p.M * (p.N / 4);
  for (long long t = blockIdx.x * 256ll + threadIdx.x; t < quads; t += (long long)gridDim.x * 256) {
    const int m = (int)(t / (p.N / 4)), n = (int)(t - (long long)m * (p.N / 4)) * 4;
    float4 a = *reinterpret_cast<const float4*>(p.slab + (size_t)m * p.N + n);
    for (int y = 1; y < S; ++y) {
      const float4 b = *reinterpret_cast<const float4*>(p.slab + ((size_t)y * p.M + m) * p.N + n);
      a.x += b.x; a.y += b.y; a.z += b.z; a.w += b.w;
    }
    float v[4] = {p.alpha * a.x, p.alpha * a.y, p.alpha * a.z, p.alpha * a.w};
    if (p.bias) {
      const float4 bb = *reinterpret_cast<const float4*>(p.bias + n);
      v[0] += bb.x; v[1] += bb.y; v[2] += bb.z; v[3] += bb.w;
    }
    if (p.d) {
      const uint2 dd = *reinterpret_cast<const uint2*>(p.d + (long long)m * p.ldd + n);
      v[0] += __uint_as_float(dd.x << 16);
      v[1] += __uint_as_float(dd.x & 0xFFFF0000u);
      v[2] += __uint_as_float(dd.y << 16);
      v[3] += __uint_as_float(dd.y & 0xFFFF0000u);
    }
    if (p.out_f32) {
      float* cp = reinterpret_cast<float*>(p.c) + (long long)m * p.ldc + n;
      if (p.beta != 0.f) {
        const float4 o = *reinterpret_cast<const float4*>(cp);
        v[0] += p.beta * o.x; v[1] += p.beta * o.y; v[2] += p.beta * o.z; v[3] += p.beta * o.w;
      }
#pragma unroll
      for (int e = 0; e < 4; ++e) v[e] = apply_act(v[e], p.act);
      *reinterpret_cast<float4*>(cp) = make_float4(v[0], v[1], v[2], v[3]);
    } else {
#pragma unroll
      for (int e = 0; e < 4; ++e) v[e] = apply_act(v[e], p.act);
      bf16_t* cp = reinterpret_cast<bf16_t*>(p.c) + (long long)m * p.ldc + n;
      *reinterpret_cast<uint2*>(cp) = make_uint2((uint32_t)f2bf(v[0]) | ((uint32_t)f2bf(v[1]) << 16),
                                                 (uint32_t)f2bf(v[2]) | ((uint32_t)f2bf(v[3]) << 16));
    }
  }
}

// Requirements (checked): K % 8 == 0, N % 4 == 0, lda / ldb % 8 == 0, ldc / ldd % 4 == 0, a / b 16-B
// aligned, c 8-B (bf16) or 16-B (fp32) aligned, bias 16-B aligned, operands below 2 GiB.
BIGDL_EXPORT int bigdl_gemm_splitk(const void* a, long long lda, const void* b, long long ldb, const float* bias,
                                   const void* d, long long ldd, void* c, long long ldc, int M, int N, int K, int act,
                                   int out_f32, float alpha, float beta, float* slab, int S, hipStream_t s);

BIGDL_EXPORT int bigdl_gemm(const void* a, long long lda, const void* b, long long ldb, const float* bias,
                            const void* d, long long ldd, void* c, long long ldc, int M, int N, int K, int act,
                            int out_f32, float alpha, float beta, hipStream_t s) {
  return bigdl_gemm_splitk(a, lda, b, ldb, bias, d, ldd, c, ldc, M, N, K, act, out_f32, alpha, beta, nullptr, 1, s);
}

// slab: S·M·N fp32 workspace (S > 1 splits K on the 64 × 64 tiles; S ≤ 1 or slab null: no split)
BIGDL_EXPORT int bigdl_gemm_splitk(const void* a, long long lda, const void* b, long long ldb, const float* bias,
                                   const void* d, long long ldd, void* c, long long ldc, int M, int N, int K, int act,
                                   int out_f32, float alpha, float beta, float* slab, int S, hipStream_t s) {
  if (M <= 0 || N <= 0 || K <= 0 || K % 8 || N % 4) return (int)hipErrorInvalidValue;
  if (lda < K || ldb < K || ldc < N || lda % 8 || ldb % 8 || ldc % 4) return (int)hipErrorInvalidValue;
  if (d && (ldd < N || ldd % 4 || !al(d, 8))) return (int)hipErrorInvalidValue;
  if (!al(a, 16) || !al(b, 16) || !al(c, out_f32 ? 16 : 8) || (bias && !al(bias, 16))) return (int)hipErrorInvalidValue;
  if (act < 0 || act > 3) return (int)hipErrorInvalidValue;
  const unsigned long long ab = ((unsigned long long)(M - 1) * lda + K) * 2ull;
  const unsigned long long bb = ((unsigned long long)(N - 1) * ldb + K) * 2ull;
  if (ab >= 0x7fff0000ull || bb >= 0x7fff0000ull) return (int)hipErrorInvalidValue;
  GemmParams p{};
  p.a = (const bf16_t*)a; p.b = (const bf16_t*)b; p.bias = bias; p.d = (const bf16_t*)d; p.c = c;
  p.lda = lda; p.ldb = ldb; p.ldc = ldc; p.ldd = ldd;
  p.M = M; p.N = N; p.K = K; p.act = act; p.out_f32 = out_f32; p.alpha = alpha; p.beta = beta;
  p.a_bytes = (uint32_t)ab; p.b_bytes = (uint32_t)bb;
  // 128 × 128 tiles while that still gives ≥ 1 block per CU, else 64 × 64 (small-M recurrent /
  // classifier GEMMs are latency-bound: more, smaller blocks)
  const long long big = (long long)((M + 127) / 128) * ((N + 127) / 128);
  if (slab && S > 1) {
    if (!al(slab, 16) || S > 64) return (int)hipErrorInvalidValue;
    constexpr int BK = 64;
    const int KT = (K + BK - 1) / BK;
    const int per = (KT + S - 1) / S;  // k-tiles per slice
    p.kchunk = per * BK;
    const int Se = (K + p.kchunk - 1) / p.kchunk;  // slices actually used (all non-empty)
    p.slab = slab;
    p.tiles_n = (N + 63) / 64;
    const long long t = (long long)((M + 63) / 64) * p.tiles_n;
    hipLaunchKernelGGL((k_gemm<64, 64, 64>), dim3((unsigned)t, (unsigned)Se), dim3(256), 0, s, p);
    const long long quads = (long long)M * (N / 4);
    hipLaunchKernelGGL(k_gemm_splitk_epi, dim3((unsigned)bigdl_grid(quads, 256, 4096)), dim3(256), 0, s, p, Se);
    BIGDL_CHECK_LAUNCH();
  }
  if (big >= 256) {
    p.tiles_n = (N + 127) / 128;
    hipLaunchKernelGGL((k_gemm<128, 128, 64>), dim3((unsigned)big), dim3(256), 0, s, p);
  } else {
    p.tiles_n = (N + 63) / 64;
    const long long t = (long long)((M + 63) / 64) * p.tiles_n;
    hipLaunchKernelGGL((k_gemm<64, 64, 64>), dim3((unsigned)t), dim3(256), 0, s, p);
  }
  BIGDL_CHECK_LAUNCH();
}

// ------------------------------------------------------------------------------------------------
// bf16 transpose [R][C] (row stride lds_) → [C][R] through a 64 × 64 LDS tile (+1 column of pad
// against bank conflicts on the transposed read)
// ------------------------------------------------------------------------------------------------
__global__ void __launch_bounds__(256) k_transpose(const bf16_t* __restrict__ src, long long lds_, bf16_t* __restrict__ dst,
                                                   long long ldd, int R, int C) {
  __shared__ bf16_t t[64][65];
  const int r0 = blockIdx.y * 64, c0 = blockIdx.x * 64;
  for (int i = threadIdx.x; i < 64 * 64; i += 256) {
    const int rr = i >> 6, cc = i & 63;
    if (r0 + rr < R && c0 + cc < C) t[rr][cc] = src[(long long)(r0 + rr) * lds_ + c0 + cc];
  }
  __syncthreads();
  for (int i = threadIdx.x; i < 64 * 64; i += 256) {
    const int cc = i >> 6, rr = i & 63;
    if (r0 + rr < R && c0 + cc < C) dst[(long long)(c0 + cc) * ldd + r0 + rr] = t[rr][cc];
  }
}

BIGDL_EXPORT int bigdl_transpose_bf16(const void* src, long long ld_src, void* dst, long long ld_dst, int R, int C,
                                      hipStream_t s) {
  if (R <= 0 || C <= 0 || ld_src < C || ld_dst < R) return (int)hipErrorInvalidValue;
  dim3 g((unsigned)((C + 63) / 64), (unsigned)((R + 63) / 64));
  hipLaunchKernelGGL(k_transpose, g, dim3(256), 0, s, (const bf16_t*)src, ld_src, (bf16_t*)dst, ld_dst, R, C);
  BIGDL_CHECK_LAUNCH();
}

// ------------------------------------------------------------------------------------------------
// column sums (bias gradient): out[n] += scale · Σ_m x[m][n], x bf16 [M][N] (row stride ld), N % 8 == 0.
// Block = 32 column chunks (8 columns each) × 8 row groups; row splits over blockIdx.y; the 8 row
// groups are folded through LDS and each block adds its partial with one float atomic per column.
// ------------------------------------------------------------------------------------------------
__global__ void __launch_bounds__(256) k_colsum(const bf16_t* __restrict__ x, long long ld, float* __restrict__ out,
                                                int M, int N, int rows_per_split, float scale) {
  __shared__ float red[8][256 + 4];
  const int cc = threadIdx.x & 31, rg = threadIdx.x >> 5;
  const int n = blockIdx.x * 256 + cc * 8;
  const int mb = blockIdx.y * rows_per_split;
  const int me = min(M, mb + rows_per_split);
  float s8[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  if (n < N) {
    for (int m = mb + rg; m < me; m += 8) {
      float v[8];
      load8(x + (long long)m * ld + n, v);
#pragma unroll
      for (int e = 0; e < 8; ++e) s8[e] += v[e];
    }
  }
#pragma unroll
  for (int e = 0; e < 8; ++e) red[rg][cc * 8 + e] = s8[e];
  __syncthreads();
  const int c = threadIdx.x;
  if (blockIdx.x * 256 + c < N) {
    float a = 0.f;
#pragma unroll
    for (int g = 0; g < 8; ++g) a += red[g][c];
    atomicAdd(out + blockIdx.x * 256 + c, scale * a);
  }
}

BIGDL_EXPORT int bigdl_colsum_bf16(const void* x, long long ld, float* out, int M, int N, float scale, hipStream_t s) {
  if (M <= 0 || N <= 0 || N % 8 || ld < N || ld % 8 || !al(x, 16)) return (int)hipErrorInvalidValue;
  const int gx = (N + 255) / 256;
  int splits = (512 + gx - 1) / gx;
  const int max_splits = (M + 63) / 64;
  if (splits > max_splits) splits = max_splits;
  if (splits < 1 || g_bigdl_deterministic) splits = 1;
  const int rps = (M + splits - 1) / splits;
  splits = (M + rps - 1) / rps;
  hipLaunchKernelGGL(k_colsum, dim3((unsigned)gx, (unsigned)splits), dim3(256), 0, s, (const bf16_t*)x, ld, out, M, N,
                     rps, scale);
  BIGDL_CHECK_LAUNCH();
}

// fp32 rows (the fp32 compute mode's bias gradients, NHWC dY as [N·H·W][K]): 4 columns per lane,
// 64 column chunks × 4 row groups per block, N % 4 == 0.
__global__ void __launch_bounds__(256) k_colsum_f32(const float* __restrict__ x, long long ld, float* __restrict__ out,
                                                    int M, int N, int rows_per_split, float scale) {
  __shared__ float red[4][256 + 4];
  const int cc = threadIdx.x & 63, rg = threadIdx.x >> 6;
  const int n = blockIdx.x * 256 + cc * 4;
  const int mb = blockIdx.y * rows_per_split;
  const int me = min(M, mb + rows_per_split);
  float4 a = make_float4(0.f, 0.f, 0.f, 0.f);
  if (n < N) {
    for (int m = mb + rg; m < me; m += 4) {
      const float4 v = *reinterpret_cast<const float4*>(x + (long long)m * ld + n);
      a.x += v.x;
      a.y += v.y;
      a.z += v.z;
      a.w += v.w;
    }
  }
  red[rg][cc * 4 + 0] = a.x;
  red[rg][cc * 4 + 1] = a.y;
  red[rg][cc * 4 + 2] = a.z;
  red[rg][cc * 4 + 3] = a.w;
  __syncthreads();
  const int c = threadIdx.x;
  if (blockIdx.x * 256 + c < N) atomicAdd(out + blockIdx.x * 256 + c, scale * (red[0][c] + red[1][c] + red[2][c] + red[3][c]));
}

BIGDL_EXPORT int bigdl_colsum_f32(const void* x, long long ld, float* out, int M, int N, float scale, hipStream_t s) {
  if (M <= 0 || N <= 0 || N % 4 || ld < N || ld % 4 || !al(x, 16)) return (int)hipErrorInvalidValue;
  const int gx = (N + 255) / 256;
  int splits = (512 + gx - 1) / gx;
  const int max_splits = (M + 63) / 64;
  if (splits > max_splits) splits = max_splits;
  if (splits < 1 || g_bigdl_deterministic) splits = 1;
  const int rps = (M + splits - 1) / splits;
  splits = (M + rps - 1) / rps;
  hipLaunchKernelGGL(k_colsum_f32, dim3((unsigned)gx, (unsigned)splits), dim3(256), 0, s, (const float*)x, ld, out, M,
                     N, rps, scale);
  BIGDL_CHECK_LAUNCH();
}
