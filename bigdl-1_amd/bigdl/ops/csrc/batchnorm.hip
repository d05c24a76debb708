// NHWC BatchNormalization for training and inference (K5/K6/K7 + fused K8/K9 epilogues).
//
// Reference semantics: DL/nn/SpatialBatchNormalization.scala (updateOutputNCHWTrainFloat :1211,
// updateGradInputNCHWTrainFloat :1048, accGradientNCHWFloat :1970): normalise with the biased batch
// variance, update runningVar with the UNBIASED variance, momentum m: r = (1-m) r + m v.
//
// Layout: x is [M = N·H·W rows][C channels] bf16 (NHWC contiguous), C % 8 == 0.
// A thread owns one group of 8 channels (one 16-B load per row) and strides over rows; a block covers
// all channels of a contiguous row range and writes per-block partial sums; a small finalize kernel
// combines the G partials per channel in double precision.  Statistics use the SHIFTED sums
// Σ(x−K), Σ(x−K)² with K = x[row 0] per channel, so no catastrophic cancellation when |mean| ≫ std.
//
// Forward (train) = stats (read x) + finalize + apply (read x [+res], write y): 3 passes of HBM
// traffic — the minimum for a non-fused BN.  Backward = reduce (read gy, x [, y]) + finalize + apply
// (read gy, x [, y], write gx [, g_res]).
#include "common.h"

struct BnGeom {
  int C, CG, RPI, tpr;  // channels, channel groups of 8, rows per iteration, active threads
};

__device__ __forceinline__ BnGeom bn_geom(int C) {
  BnGeom g;
  g.C = C;
  g.CG = C >> 3;
  int cg_eff = g.CG < 256 ? g.CG : 256;
  g.RPI = 256 / cg_eff;
  g.tpr = cg_eff;
  return g;
}

// ------------------------------------------------------------------------------------------------ stats
// partial[b][c] = Σ_{rows of block b} (x − K_c),  partial[G + b][c] = Σ (x − K_c)²
// kshift (optional): per-channel shift K (a cross-rank SyncBN needs the SAME K on every rank — the
// running mean); default K = x[row 0]
__global__ void __launch_bounds__(256) k_bn_stats(const bf16_t* __restrict__ x, long long M, int C,
                                                  long long rows_per_block, float* __restrict__ partial, int G,
                                                  const float* __restrict__ kshift = nullptr) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  BnGeom g = bn_geom(C);
  const int t = threadIdx.x;
  const int cg_local = t % g.tpr;
  const int r_off = t / g.tpr;
  const long long r0 = (long long)blockIdx.x * rows_per_block;
  long long r1 = r0 + rows_per_block;
  if (r1 > M) r1 = M;
  float* s_sum = smem;                 // [RPI][C]
  float* s_sq = smem + g.RPI * C;      // [RPI][C]
  for (int cg = cg_local; cg < g.CG; cg += g.tpr) {
    float K[8], s[8], q[8];
    if (kshift) {
#pragma unroll
      for (int k = 0; k < 8; ++k) K[k] = kshift[cg * 8 + k];
    } else {
      load8(x + (size_t)cg * 8, K);  // row 0
    }
#pragma unroll
    for (int k = 0; k < 8; ++k) { s[k] = 0.f; q[k] = 0.f; }
    if (r_off < g.RPI) {
      for (long long r = r0 + r_off; r < r1; r += g.RPI) {
        float v[8];
        load8_nt(x + (size_t)r * C + (size_t)cg * 8, v);
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          float d = v[k] - K[k];
          s[k] += d;
          q[k] = fmaf(d, d, q[k]);
        }
      }
      #pragma unroll
      for (int k = 0; k < 8; ++k) {
        s_sum[r_off * C + cg * 8 + k] = s[k];
        s_sq[r_off * C + cg * 8 + k] = q[k];
      }
    }
  }
  __syncthreads();
  for (int c = t; c < C; c += 256) {
    float s = 0.f, q = 0.f;
    for (int i = 0; i < g.RPI; ++i) {
      s += s_sum[i * C + c];
      q += s_sq[i * C + c];
    }
    partial[(size_t)blockIdx.x * C + c] = s;
    partial[(size_t)(G + blockIdx.x) * C + c] = q;
  }
}

// Parallel reduction of the G per-block partials: a block owns 32 channels; its kFinRG row groups
// each sum G/kFinRG partials with coalesced 128-B loads (8 in flight per thread), then a LDS tree.
// Results: red[0][c] = Σ partial[0..G), red[1][c] = Σ partial[G..2G) for the block's 32 channels.
// The sums over partials are fp64: the conv epilogue's partials are unshifted 128-row Σy, Σy², so
// var = Σy²/M − mean² cancels; summing thousands of partials in double keeps that difference exact
// to the partials' own fp32 rounding (profiles: a shifted fp32 epilogue cost 11 % of conv-forward
// time, the fp64 combine costs nothing measurable).
// 256 threads = 32 channels × kFinRG row groups: small blocks, so a finalize queued behind the
// side-stream weight-gradient kernels finds a CU with room quickly (1024-thread blocks waited for a
// CU with 16 free wave slots: ~40 µs per finalize in a contended step, profiles/r3_bench_prof_a.txt)
constexpr int kFinRG = 8;

template <typename T>
__device__ __forceinline__ void reduce_partials(const T* __restrict__ partial, int G, int C, int c0,
                                                double (*lds)[2][33], double& outA, double& outB,
                                                float* rezero = nullptr) {
  const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;
  const int c = c0 + tx;
  double a = 0.0, b = 0.0;
  if (c < C) {
    int i = ty;
#pragma unroll 8
    for (; i < G; i += kFinRG) {
      a += partial[(size_t)i * C + c];
      b += partial[(size_t)(G + i) * C + c];
    }
    // replicated atomic statistics: this block owns columns c0..c0+31 — clear what it just read
    // for the next accumulation (each thread clears exactly the elements it loaded)
    asm volatile("" ::: "memory");  // the clears below alias `partial` (declared __restrict__)
    if (rezero)
      for (i = ty; i < G; i += kFinRG) {
        rezero[(size_t)i * C + c] = 0.f;
        rezero[(size_t)(G + i) * C + c] = 0.f;
      }
  }
  lds[ty][0][tx] = a;
  lds[ty][1][tx] = b;
  __syncthreads();
  for (int s = kFinRG / 2; s > 0; s >>= 1) {
    if (ty < s) {
      lds[ty][0][tx] += lds[ty + s][0][tx];
      lds[ty][1][tx] += lds[ty + s][1][tx];
    }
    __syncthreads();
  }
  outA = lds[0][0][tx];
  outB = lds[0][1][tx];
}

// Combine partials; write save_mean/save_invstd, apply coefficients scale/shift, update running stats.
// ``in_bias`` (optional) is a per-channel constant the producer did NOT add to x (a conv bias folded
// into this BN): normalisation is shift-invariant, so only the running mean sees it.
template <typename T>
__global__ void __launch_bounds__(32 * kFinRG) k_bn_finalize(const bf16_t* __restrict__ x, const float* kshift,
                                                      const T* __restrict__ partial,
                                                      int G, long long M, int C, const float* __restrict__ gamma,
                                                      const float* __restrict__ beta,
                                                      const float* __restrict__ in_bias,
                                                      float* run_mean, float* __restrict__ run_var,
                                                      float momentum, float eps, float* __restrict__ save_mean,
                                                      float* __restrict__ save_invstd, float* __restrict__ scale,
                                                      float* __restrict__ shift, const float* __restrict__ dM = nullptr,
                                                      float* rezero = nullptr) {
  // dM: the row count read from device memory (SyncBN: the all-reduced count travels in the sums
  // buffer, so the host never waits for it); else M.  rezero: clear the partials after reading them
  // (replicated atomic statistics, ConvParams::stats_atomic = R)
  __shared__ double lds[kFinRG][2][33];
  double s, q;
  reduce_partials(partial, G, C, blockIdx.x * 32, lds, s, q, rezero);
  const int c = blockIdx.x * 32 + (threadIdx.x & 31);
  if ((threadIdx.x >> 5) != 0 || c >= C) return;
  // partials are shifted by the first row (standalone stats pass), by ``kshift`` (conv epilogue
  // given the running mean — it may alias run_mean: read here, before run_mean is written below,
  // hence neither pointer is __restrict__) or unshifted
  const float K = kshift ? kshift[c] : (x ? bf2f(x[c]) : 0.f);
  const double Md = dM ? (double)*dM : (double)M;
  const double dmd = s / Md;
  const float var = (float)fmax(q / Md - dmd * dmd, 0.0);
  const float dm = (float)dmd;
  float mean = K + dm;
  float invstd = rsqrtf(var + eps);
  save_mean[c] = mean;
  save_invstd[c] = invstd;
  float gm = gamma ? gamma[c] : 1.f;
  float bt = beta ? beta[c] : 0.f;
  float sc = gm * invstd;
  scale[c] = sc;
  shift[c] = bt - mean * sc;
  if (run_mean) {
    float unb = Md > 1.0 ? (float)(var * Md / (Md - 1.0)) : var;
    float true_mean = mean + (in_bias ? in_bias[c] : 0.f);
    run_mean[c] = (1.f - momentum) * run_mean[c] + momentum * true_mean;
    run_var[c] = (1.f - momentum) * run_var[c] + momentum * unb;
  }
}

// inference coefficients from running stats (x excludes an optional folded producer bias)
__global__ void k_bn_infer_coef(int C, const float* __restrict__ gamma, const float* __restrict__ beta,
                                const float* __restrict__ run_mean, const float* __restrict__ run_var,
                                const float* __restrict__ in_bias, float eps, float* __restrict__ scale,
                                float* __restrict__ shift) {
  int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  float invstd = rsqrtf(run_var[c] + eps);
  float sc = (gamma ? gamma[c] : 1.f) * invstd;
  scale[c] = sc;
  shift[c] = (beta ? beta[c] : 0.f) - (run_mean[c] - (in_bias ? in_bias[c] : 0.f)) * sc;
}

// ------------------------------------------------------------------------------------------------ apply
// inputs are streamed with non-temporal loads (read once per pass, next use a whole step later):
// k_bn_apply<res, relu> 1.56 → 1.37 ms per ResNet-50 step, step 23.1 → 22.8 ms
// (profiles/r2_bench_v7_profile.txt)
// BITS (with RELU): also emit the ReLU mask as one byte per 8-channel chunk (bit e = output channel
// cg·8 + e is > 0) — a ResNet block tail's output mask for the backward, 1/16 of the bytes of
// re-reading the bf16 output there.
// The streaming body (scale / shift: global memory, or the block's LDS copy in the one-launch
// finalize+apply kernels below).
template <bool RES, bool RELU, bool BITS, int kApplyUnroll>
__device__ __forceinline__ void bn_apply_rows(const bf16_t* __restrict__ x, const bf16_t* __restrict__ res,
                                              bf16_t* __restrict__ y, long long M, int C, const float* scale,
                                              const float* shift, uint8_t* __restrict__ bits,
                                              const float* rcoef = nullptr) {
  BnGeom g = bn_geom(C);
  const int t = threadIdx.x;
  const int cg_local = t % g.tpr;
  const int r_off = t / g.tpr;
  if (r_off >= g.RPI) return;
  const long long rstride = (long long)gridDim.x * g.RPI;
  for (int cg = cg_local; cg < g.CG; cg += g.tpr) {
    float sc[8], sh[8], rsc[8], rsh[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      sc[k] = scale[cg * 8 + k];
      sh[k] = shift[cg * 8 + k];
      // rcoef: the residual is itself a BN input (a deferred shortcut BN): res · rscale + rshift
      rsc[k] = (RES && rcoef) ? rcoef[cg * 8 + k] : 1.f;
      rsh[k] = (RES && rcoef) ? rcoef[C + cg * 8 + k] : 0.f;
    }
    // kApplyUnroll rows per trip: all their loads are issued before the first use, so each thread
    // keeps several 16-B requests in flight (one per trip left the streaming passes latency-bound)
    long long r = (long long)blockIdx.x * g.RPI + r_off;
    for (; r < M; r += kApplyUnroll * rstride) {
      bigdl_u32x4 xv[kApplyUnroll], rvv[kApplyUnroll];
#pragma unroll
      for (int u = 0; u < kApplyUnroll; ++u) {
        const long long ru = r + u * rstride;
        const size_t off = (size_t)(ru < M ? ru : r) * C + (size_t)cg * 8;
        xv[u] = __builtin_nontemporal_load(reinterpret_cast<const bigdl_u32x4*>(x + off));
        if (RES) rvv[u] = __builtin_nontemporal_load(reinterpret_cast<const bigdl_u32x4*>(res + off));
      }
#pragma unroll
      for (int u = 0; u < kApplyUnroll; ++u) {
        const long long ru = r + u * rstride;
        if (ru >= M) break;
        const size_t off = (size_t)ru * C + (size_t)cg * 8;
        float v[8], rv[8];
        unpack8(make_uint4(xv[u][0], xv[u][1], xv[u][2], xv[u][3]), v);
        if (RES) unpack8(make_uint4(rvv[u][0], rvv[u][1], rvv[u][2], rvv[u][3]), rv);
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          float o = fmaf(v[k], sc[k], sh[k]);
          if (RES) o += fmaf(rv[k], rsc[k], rsh[k]);
          if (RELU) o = fmaxf(o, 0.f);
          v[k] = o;
        }
        store8(y + off, v);
        if (BITS) {
          // the bit must agree with the stored bf16 value (> 0 after rounding: a positive fp32 never
          // rounds to +0 in bf16, so o > 0 is exact)
          uint32_t b = 0;
#pragma unroll
          for (int k = 0; k < 8; ++k) b |= (v[k] > 0.f ? 1u : 0u) << k;
          bits[off >> 3] = (uint8_t)b;
        }
      }
    }
  }
}

template <bool RES, bool RELU, bool BITS = false, int kApplyUnroll = 4>
__global__ void __launch_bounds__(256) k_bn_apply(const bf16_t* __restrict__ x, const bf16_t* __restrict__ res,
                                                  bf16_t* __restrict__ y, long long M, int C,
                                                  const float* __restrict__ scale, const float* __restrict__ shift,
                                                  uint8_t* __restrict__ bits = nullptr,
                                                  const float* __restrict__ rcoef = nullptr) {
  bn_apply_rows<RES, RELU, BITS, kApplyUnroll>(x, res, y, M, C, scale, shift, bits, rcoef);
}

// A/B knobs (profiles/r3_bn_apply_ab.txt, r5_bn_apply_blocks_ab.txt): BIGDL_BN_APPLY_BLOCKS caps the grid (default 2048 since round 5; at 1024: 0.87-1.06
// of the best streaming copy in isolation vs 0.64-0.98 at 2048; neutral inside the ResNet step),
// BIGDL_BN_UNROLL=1 issues one row per trip instead of 4.
static int apply_cap() {
  static int cap = [] {
    const char* e = getenv("BIGDL_BN_APPLY_BLOCKS");
    const int v = e ? atoi(e) : 0;
    return v >= 64 ? v : 2048;  // round 5: 2048 20.64-20.69 vs 1024 20.69-20.73 ms (profiles/r5_bn_apply_blocks_ab.txt)
  }();
  return cap;
}
static bool apply_unroll1() {
  static bool u1 = [] {
    const char* e = getenv("BIGDL_BN_UNROLL");
    return e && e[0] == '1';
  }();
  return u1;
}

static int apply_grid(long long M, int C) {
  int CG = C / 8;
  int tpr = CG < 256 ? CG : 256;
  int rpi = 256 / tpr;
  long long blocks = (M + rpi - 1) / rpi;
  if (blocks > apply_cap()) blocks = apply_cap();
  if (blocks < 1) blocks = 1;
  return (int)blocks;
}

static void launch_apply(const void* x, const void* res, void* y, long long M, int C, const float* coef, int relu,
                         void* bits, hipStream_t s, const float* rcoef = nullptr) {
  int grid = apply_grid(M, C);
  const bf16_t* xr = (const bf16_t*)x;
  const bf16_t* rr = (const bf16_t*)res;
  bf16_t* yr = (bf16_t*)y;
  uint8_t* br = (uint8_t*)bits;
  if (apply_unroll1()) {
    if (relu && bits && res)
      hipLaunchKernelGGL((k_bn_apply<true, true, true, 1>), dim3(grid), dim3(256), 0, s, xr, rr, yr, M, C, coef, coef + C, br, rcoef);
    else if (relu && bits)
      hipLaunchKernelGGL((k_bn_apply<false, true, true, 1>), dim3(grid), dim3(256), 0, s, xr, rr, yr, M, C, coef, coef + C, br, rcoef);
    else if (res && relu) hipLaunchKernelGGL((k_bn_apply<true, true, false, 1>), dim3(grid), dim3(256), 0, s, xr, rr, yr, M, C, coef, coef + C, br, rcoef);
    else if (res) hipLaunchKernelGGL((k_bn_apply<true, false, false, 1>), dim3(grid), dim3(256), 0, s, xr, rr, yr, M, C, coef, coef + C, br, rcoef);
    else if (relu) hipLaunchKernelGGL((k_bn_apply<false, true, false, 1>), dim3(grid), dim3(256), 0, s, xr, rr, yr, M, C, coef, coef + C, br, rcoef);
    else hipLaunchKernelGGL((k_bn_apply<false, false, false, 1>), dim3(grid), dim3(256), 0, s, xr, rr, yr, M, C, coef, coef + C, br, rcoef);
    return;
  }
  if (relu && bits && res)
    hipLaunchKernelGGL((k_bn_apply<true, true, true>), dim3(grid), dim3(256), 0, s, xr, rr, yr, M, C, coef, coef + C, br, rcoef);
  else if (relu && bits)
    hipLaunchKernelGGL((k_bn_apply<false, true, true>), dim3(grid), dim3(256), 0, s, xr, rr, yr, M, C, coef, coef + C, br, rcoef);
  else if (res && relu) hipLaunchKernelGGL((k_bn_apply<true, true>), dim3(grid), dim3(256), 0, s, xr, rr, yr, M, C, coef, coef + C, br, rcoef);
  else if (res) hipLaunchKernelGGL((k_bn_apply<true, false>), dim3(grid), dim3(256), 0, s, xr, rr, yr, M, C, coef, coef + C, br, rcoef);
  else if (relu) hipLaunchKernelGGL((k_bn_apply<false, true>), dim3(grid), dim3(256), 0, s, xr, rr, yr, M, C, coef, coef + C, br, rcoef);
  else hipLaunchKernelGGL((k_bn_apply<false, false>), dim3(grid), dim3(256), 0, s, xr, rr, yr, M, C, coef, coef + C, br, rcoef);
}

// number of partial blocks used by the stats / backward-reduce kernels (mirrored in Python)
BIGDL_EXPORT int bigdl_bn_num_partials(long long M, int C) {
  int CG = C / 8;
  int tpr = CG < 256 ? CG : 256;
  int rpi = 256 / tpr;
  long long target_rows = (long long)rpi * 32;  // ≥32 rows per thread per block
  long long G = (M + target_rows - 1) / target_rows;
  if (G > 512) G = 512;
  if (G < 1) G = 1;
  return (int)G;
}

static size_t stats_smem(int C) {
  int CG = C / 8;
  int tpr = CG < 256 ? CG : 256;
  int rpi = 256 / tpr;
  return (size_t)rpi * C * 2 * sizeof(float);
}

// Training forward.  ws: partial buffer of 2·G·C floats; coef: 2·C floats (scale, shift).
// bits (optional, relu only): M·C/8 bytes receiving the output's ReLU mask (see k_bn_apply)
BIGDL_EXPORT int bigdl_bn_fwd_train(const void* x, const void* res, void* y, long long M, int C, const float* gamma,
                                    const float* beta, const float* in_bias, float* run_mean, float* run_var,
                                    float momentum, float eps, float* save_mean, float* save_invstd, float* ws,
                                    float* coef, int relu, void* bits, hipStream_t s) {
  if (bits && !relu) return (int)hipErrorInvalidValue;
  if (C % 8 || M <= 0) return (int)hipErrorInvalidValue;
  int G = bigdl_bn_num_partials(M, C);
  long long rpb = (M + G - 1) / G;
  size_t sm = stats_smem(C);
  if (sm > 64 * 1024) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(k_bn_stats, dim3(G), dim3(256), sm, s, (const bf16_t*)x, M, C, rpb, ws, G);
  hipLaunchKernelGGL(k_bn_finalize<float>, dim3((C + 31) / 32), dim3(32 * kFinRG), 0, s, (const bf16_t*)x, nullptr,
                     (const float*)ws, G,
                     M, C, gamma, beta, in_bias, run_mean, run_var, momentum, eps, save_mean, save_invstd, coef, coef + C);
  launch_apply(x, res, y, M, C, coef, relu, bits, s);
  BIGDL_CHECK_LAUNCH();
}

// Pre-fold of many per-row-tile partials (conv-epilogue statistics: G up to M/128) into S ≤ G/128
// rows, so the per-channel finalize reads a short column instead of a latency-bound 6k-long one.
// grid (ceil(C/64), S), 256 threads = 64 channels × 4 row groups; rows [sy·R, sy·R + R) per block.
__global__ void __launch_bounds__(256) k_bn_fold_partials(const float* __restrict__ partial, int G, int C, int R,
                                                          int S, double* __restrict__ out) {
  __shared__ double red[2][4][64];
  const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
  const int c = blockIdx.x * 64 + tx;
  const int g0 = blockIdx.y * R;
  int g1 = g0 + R;
  if (g1 > G) g1 = G;
  double a = 0.0, b = 0.0;
  if (c < C) {
#pragma unroll 4
    for (int g = g0 + ty; g < g1; g += 4) {
      a += partial[(size_t)g * C + c];
      b += partial[(size_t)(G + g) * C + c];
    }
  }
  red[0][ty][tx] = a;
  red[1][ty][tx] = b;
  __syncthreads();
  if (ty == 0 && c < C) {
    out[(size_t)blockIdx.y * C + c] = red[0][0][tx] + red[0][1][tx] + red[0][2][tx] + red[0][3][tx];
    out[(size_t)(S + blockIdx.y) * C + c] = red[1][0][tx] + red[1][1][tx] + red[1][2][tx] + red[1][3][tx];
  }
}

static constexpr int kFoldRows = 128;

// floats of scratch bigdl_bn_*_partials needs for G partials of C channels (0: no pre-fold); the
// folded rows are fp64 (2 floats each)
BIGDL_EXPORT long long bigdl_bn_fold_scratch(int G, int C) {
  if (G <= 512) return 0;
  const int S = (G + kFoldRows - 1) / kFoldRows;
  return 4LL * S * C;
}

// launch the finalize-type kernel on either the raw fp32 partials or their fp64 pre-fold
static bool maybe_fold(const float* partial, int& G, int C, float* scratch, hipStream_t s) {
  if (G <= 512 || !scratch) return false;
  const int S = (G + kFoldRows - 1) / kFoldRows;
  hipLaunchKernelGGL(k_bn_fold_partials, dim3((C + 63) / 64, S), dim3(256), 0, s, partial, G, C, kFoldRows, S,
                     (double*)scratch);
  G = S;
  return true;
}

// Training forward from precomputed partials (the producing conv's epilogue wrote Σy, Σy² per row
// tile, unshifted): finalize + apply only — the stats pass over x is gone.
BIGDL_EXPORT int bigdl_bn_fwd_train_partials2(const void* x, const void* res, const float* rcoef, void* y, long long M,
                                              int C, const float* gamma, const float* beta, const float* in_bias,
                                              float* run_mean, float* run_var, float momentum, float eps,
                                              float* save_mean, float* save_invstd, const float* partial, int G,
                                              const float* kshift, float* coef, int relu, float* scratch, void* bits,
                                              int rezero, hipStream_t s);

BIGDL_EXPORT int bigdl_bn_fwd_train_partials(const void* x, const void* res, void* y, long long M, int C,
                                             const float* gamma, const float* beta, const float* in_bias,
                                             float* run_mean, float* run_var, float momentum, float eps,
                                             float* save_mean, float* save_invstd, const float* partial, int G,
                                             const float* kshift, float* coef, int relu, float* scratch, void* bits,
                                             int rezero, hipStream_t s) {
  if (!y) return (int)hipErrorInvalidValue;
  return bigdl_bn_fwd_train_partials2(x, res, nullptr, y, M, C, gamma, beta, in_bias, run_mean, run_var, momentum, eps,
                                      save_mean, save_invstd, partial, G, kshift, coef, relu, scratch, bits, rezero, s);
}

// y == null: finalize only (statistics, running averages, coef) — a shortcut BN whose apply is
// deferred into the block tail's (rcoef there); rcoef (with res): the residual is res·rcoef[c] +
// rcoef[C + c], a deferred BN's input and coefficients
BIGDL_EXPORT int bigdl_bn_fwd_train_partials2(const void* x, const void* res, const float* rcoef, void* y, long long M,
                                              int C, const float* gamma, const float* beta, const float* in_bias,
                                              float* run_mean, float* run_var, float momentum, float eps,
                                              float* save_mean, float* save_invstd, const float* partial, int G,
                                              const float* kshift, float* coef, int relu, float* scratch, void* bits,
                                              int rezero, hipStream_t s) {
  if (rcoef && !res) return (int)hipErrorInvalidValue;
  if (C % 8 || M <= 0 || G <= 0 || (bits && !relu) || (rezero && G > 512)) return (int)hipErrorInvalidValue;
  if (!rezero && maybe_fold(partial, G, C, scratch, s))
    hipLaunchKernelGGL(k_bn_finalize<double>, dim3((C + 31) / 32), dim3(32 * kFinRG), 0, s, (const bf16_t*)nullptr, kshift,
                       (const double*)scratch, G, M, C, gamma, beta, in_bias, run_mean, run_var, momentum, eps, save_mean,
                       save_invstd, coef, coef + C);
  else
    hipLaunchKernelGGL(k_bn_finalize<float>, dim3((C + 31) / 32), dim3(32 * kFinRG), 0, s, (const bf16_t*)nullptr, kshift,
                       partial, G, M, C, gamma, beta, in_bias, run_mean, run_var, momentum, eps, save_mean, save_invstd,
                       coef, coef + C, nullptr, rezero ? const_cast<float*>(partial) : nullptr);
  if (y) launch_apply(x, res, y, M, C, coef, relu, bits, s, rcoef);
  BIGDL_CHECK_LAUNCH();
}

BIGDL_EXPORT int bigdl_bn_fwd_infer(const void* x, void* y, long long M, int C, const float* gamma, const float* beta,
                                    const float* run_mean, const float* run_var, const float* in_bias, float eps,
                                    float* coef, int relu, hipStream_t s) {
  if (C % 8 || M <= 0) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(k_bn_infer_coef, dim3((C + 255) / 256), dim3(256), 0, s, C, gamma, beta, run_mean, run_var,
                     in_bias, eps, coef, coef + C);
  int grid = apply_grid(M, C);
  if (relu)
    hipLaunchKernelGGL((k_bn_apply<false, true>), dim3(grid), dim3(256), 0, s, (const bf16_t*)x, nullptr, (bf16_t*)y,
                       M, C, coef, coef + C);
  else
    hipLaunchKernelGGL((k_bn_apply<false, false>), dim3(grid), dim3(256), 0, s, (const bf16_t*)x, nullptr,
                       (bf16_t*)y, M, C, coef, coef + C);
  BIGDL_CHECK_LAUNCH();
}

// ------------------------------------------------------------------------------------------------ backward
// partial[b][c] = Σ g',  partial[G+b][c] = Σ g'·(x − mean),  g' = gy · [y > 0 if RELU]
template <bool RELU>
__global__ void __launch_bounds__(256) k_bn_bwd_reduce(const bf16_t* __restrict__ gy, const bf16_t* __restrict__ x,
                                                       const bf16_t* __restrict__ y, long long M, int C,
                                                       long long rows_per_block, const float* __restrict__ mean,
                                                       float* __restrict__ partial, int G) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  BnGeom g = bn_geom(C);
  const int t = threadIdx.x;
  const int cg_local = t % g.tpr;
  const int r_off = t / g.tpr;
  const long long r0 = (long long)blockIdx.x * rows_per_block;
  long long r1 = r0 + rows_per_block;
  if (r1 > M) r1 = M;
  float* s_a = smem;
  float* s_b = smem + g.RPI * C;
  for (int cg = cg_local; cg < g.CG; cg += g.tpr) {
    if (r_off >= g.RPI) break;
    float mu[8], a[8], b[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) { mu[k] = mean[cg * 8 + k]; a[k] = 0.f; b[k] = 0.f; }
    for (long long r = r0 + r_off; r < r1; r += g.RPI) {
      size_t off = (size_t)r * C + (size_t)cg * 8;
      float gv[8], xv[8];
      load8_nt(gy + off, gv);
      load8_nt(x + off, xv);
      if (RELU) {
        float yv[8];
        load8_nt(y + off, yv);
#pragma unroll
        for (int k = 0; k < 8; ++k) gv[k] = yv[k] > 0.f ? gv[k] : 0.f;
      }
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        a[k] += gv[k];
        b[k] = fmaf(gv[k], xv[k] - mu[k], b[k]);
      }
    }
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      s_a[r_off * C + cg * 8 + k] = a[k];
      s_b[r_off * C + cg * 8 + k] = b[k];
    }
  }
  __syncthreads();
  for (int c = t; c < C; c += 256) {
    float a = 0.f, b = 0.f;
    for (int i = 0; i < g.RPI; ++i) {
      a += s_a[i * C + c];
      b += s_b[i * C + c];
    }
    partial[(size_t)blockIdx.x * C + c] = a;
    partial[(size_t)(G + blockIdx.x) * C + c] = b;
  }
}

// dβ = Σg', dγ = invstd·Σg'(x−μ); accumulate scale·dγ, scale·dβ into the fp32 grad arena;
// coefficients for gx = A·g' + B·x + Cc
// ``cbias`` (optional): gradient of a producer bias folded into this BN = Σ_rows gx, evaluated from
// the closed form A·Σg' + B·Σx + M·Cc (Σx = M·mean) and accumulated with ``cbscale``.
template <typename T>
__global__ void __launch_bounds__(32 * kFinRG) k_bn_bwd_finalize(const T* __restrict__ partial, int G, long long M,
                                                          int C, const float* __restrict__ gamma,
                                                          const float* __restrict__ mean,
                                                          const float* __restrict__ invstd,
                                                          float* __restrict__ ggamma, float* __restrict__ gbeta,
                                                          float gscale, float* __restrict__ cbias, float cbscale,
                                                          float* __restrict__ coef, const float* __restrict__ dM = nullptr,
                                                          float* rezero = nullptr) {
  __shared__ double lds[kFinRG][2][33];
  double ad, bd;
  reduce_partials(partial, G, C, blockIdx.x * 32, lds, ad, bd, rezero);
  const int c = blockIdx.x * 32 + (threadIdx.x & 31);
  if ((threadIdx.x >> 5) != 0 || c >= C) return;
  const float a = (float)ad, b = (float)bd;
  float is = invstd[c];
  float dbeta = a;
  float dgamma = b * is;
  if (ggamma) ggamma[c] += gscale * dgamma;
  if (gbeta) gbeta[c] += gscale * dbeta;
  float gm = gamma ? gamma[c] : 1.f;
  float A = gm * is;
  const float Mf = dM ? *dM : (float)M;
  float B = -gm * is * is * dgamma / Mf;
  float Cc = -gm * is * dbeta / Mf - B * mean[c];
  coef[c] = A;
  coef[C + c] = B;
  coef[2 * C + c] = Cc;
  if (cbias) cbias[c] += cbscale * (A * dbeta + B * Mf * mean[c] + Mf * Cc);
}

template <bool RELU, bool GRES, int kApplyUnroll>
__device__ __forceinline__ void bn_bwd_apply_rows(const bf16_t* __restrict__ gy, const bf16_t* __restrict__ x,
                                                  const bf16_t* __restrict__ y, bf16_t* __restrict__ gx,
                                                  bf16_t* __restrict__ gres, long long M, int C, const float* coef) {
  BnGeom g = bn_geom(C);
  const int t = threadIdx.x;
  const int cg_local = t % g.tpr;
  const int r_off = t / g.tpr;
  if (r_off >= g.RPI) return;
  const long long rstride = (long long)gridDim.x * g.RPI;
  for (int cg = cg_local; cg < g.CG; cg += g.tpr) {
    float A[8], B[8], Cc[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      A[k] = coef[cg * 8 + k];
      B[k] = coef[C + cg * 8 + k];
      Cc[k] = coef[2 * C + cg * 8 + k];
    }
    long long r = (long long)blockIdx.x * g.RPI + r_off;
    for (; r < M; r += kApplyUnroll * rstride) {  // see k_bn_apply: loads of all rows of a trip first
      bigdl_u32x4 gq[kApplyUnroll], xq[kApplyUnroll], yq[kApplyUnroll];
#pragma unroll
      for (int u = 0; u < kApplyUnroll; ++u) {
        const long long ru = r + u * rstride;
        const size_t off = (size_t)(ru < M ? ru : r) * C + (size_t)cg * 8;
        gq[u] = __builtin_nontemporal_load(reinterpret_cast<const bigdl_u32x4*>(gy + off));
        xq[u] = __builtin_nontemporal_load(reinterpret_cast<const bigdl_u32x4*>(x + off));
        if (RELU) yq[u] = __builtin_nontemporal_load(reinterpret_cast<const bigdl_u32x4*>(y + off));
      }
#pragma unroll
      for (int u = 0; u < kApplyUnroll; ++u) {
        const long long ru = r + u * rstride;
        if (ru >= M) break;
        const size_t off = (size_t)ru * C + (size_t)cg * 8;
        float gv[8], xv[8];
        unpack8(make_uint4(gq[u][0], gq[u][1], gq[u][2], gq[u][3]), gv);
        unpack8(make_uint4(xq[u][0], xq[u][1], xq[u][2], xq[u][3]), xv);
        if (RELU) {
          float yv[8];
          unpack8(make_uint4(yq[u][0], yq[u][1], yq[u][2], yq[u][3]), yv);
#pragma unroll
          for (int k = 0; k < 8; ++k) gv[k] = yv[k] > 0.f ? gv[k] : 0.f;
        }
        if (GRES) store8(gres + off, gv);
#pragma unroll
        for (int k = 0; k < 8; ++k) xv[k] = fmaf(A[k], gv[k], fmaf(B[k], xv[k], Cc[k]));
        store8(gx + off, xv);
      }
    }
  }
}

template <bool RELU, bool GRES, int kApplyUnroll = 4>
__global__ void __launch_bounds__(256) k_bn_bwd_apply(const bf16_t* __restrict__ gy, const bf16_t* __restrict__ x,
                                                      const bf16_t* __restrict__ y, bf16_t* __restrict__ gx,
                                                      bf16_t* __restrict__ gres, long long M, int C,
                                                      const float* __restrict__ coef) {
  bn_bwd_apply_rows<RELU, GRES, kApplyUnroll>(gy, x, y, gx, gres, M, C, coef);
}

// Backward.  ws: 2·G·C floats; coef: 3·C floats.  gx may be null (no input gradient needed).
// gres (optional): receives g' (the masked upstream gradient) for a fused residual branch.
BIGDL_EXPORT int bigdl_bn_bwd(const void* gy, const void* x, const void* y, void* gx, void* gres, long long M, int C,
                              const float* gamma, const float* mean, const float* invstd, float* ggamma,
                              float* gbeta, float gscale, float* cbias, float cbscale, float* ws, float* coef,
                              int relu, hipStream_t s) {
  if (C % 8 || M <= 0) return (int)hipErrorInvalidValue;
  int G = bigdl_bn_num_partials(M, C);
  long long rpb = (M + G - 1) / G;
  size_t sm = stats_smem(C);
  if (relu)
    hipLaunchKernelGGL(k_bn_bwd_reduce<true>, dim3(G), dim3(256), sm, s, (const bf16_t*)gy, (const bf16_t*)x,
                       (const bf16_t*)y, M, C, rpb, mean, ws, G);
  else
    hipLaunchKernelGGL(k_bn_bwd_reduce<false>, dim3(G), dim3(256), sm, s, (const bf16_t*)gy, (const bf16_t*)x,
                       (const bf16_t*)y, M, C, rpb, mean, ws, G);
  hipLaunchKernelGGL(k_bn_bwd_finalize<float>, dim3((C + 31) / 32), dim3(32 * kFinRG), 0, s, (const float*)ws, G, M, C, gamma,
                     mean, invstd, ggamma, gbeta, gscale, cbias, cbscale, coef);
  if (gx) {
    int grid = apply_grid(M, C);
    const bf16_t *g_ = (const bf16_t*)gy, *x_ = (const bf16_t*)x, *y_ = (const bf16_t*)y;
    bf16_t *gx_ = (bf16_t*)gx, *gr_ = (bf16_t*)gres;
    if (relu && gres) hipLaunchKernelGGL((k_bn_bwd_apply<true, true>), dim3(grid), dim3(256), 0, s, g_, x_, y_, gx_, gr_, M, C, coef);
    else if (relu) hipLaunchKernelGGL((apply_unroll1() ? k_bn_bwd_apply<true, false, 1> : k_bn_bwd_apply<true, false, 4>), dim3(grid), dim3(256), 0, s, g_, x_, y_, gx_, gr_, M, C, coef);
    else if (gres) hipLaunchKernelGGL((k_bn_bwd_apply<false, true>), dim3(grid), dim3(256), 0, s, g_, x_, y_, gx_, gr_, M, C, coef);
    else hipLaunchKernelGGL((apply_unroll1() ? k_bn_bwd_apply<false, false, 1> : k_bn_bwd_apply<false, false, 4>), dim3(grid), dim3(256), 0, s, g_, x_, y_, gx_, gr_, M, C, coef);
  }
  BIGDL_CHECK_LAUNCH();
}

// Backward from partials produced by the consuming conv's dgrad epilogue (Σg, Σg·(x − mean) of
// the already ReLU-masked gradient gm): finalize + apply only — the reduce pass over (gy, x, y)
// is gone and the apply no longer reads y.
BIGDL_EXPORT int bigdl_bn_bwd_partials(const void* gm, const void* x, void* gx, long long M, int C, const float* gamma,
                                       const float* mean, const float* invstd, float* ggamma, float* gbeta,
                                       float gscale, float* cbias, float cbscale, const float* partial, int G,
                                       float* coef, float* scratch, int rezero, hipStream_t s) {
  if (C % 8 || M <= 0 || G <= 0 || (rezero && G > 512)) return (int)hipErrorInvalidValue;
  if (!rezero && maybe_fold(partial, G, C, scratch, s))
    hipLaunchKernelGGL(k_bn_bwd_finalize<double>, dim3((C + 31) / 32), dim3(32 * kFinRG), 0, s, (const double*)scratch, G, M,
                       C, gamma, mean, invstd, ggamma, gbeta, gscale, cbias, cbscale, coef);
  else
    hipLaunchKernelGGL(k_bn_bwd_finalize<float>, dim3((C + 31) / 32), dim3(32 * kFinRG), 0, s, partial, G, M, C, gamma, mean,
                       invstd, ggamma, gbeta, gscale, cbias, cbscale, coef, nullptr,
                       rezero ? const_cast<float*>(partial) : nullptr);
  if (gx) {
    int grid = apply_grid(M, C);
    hipLaunchKernelGGL((apply_unroll1() ? k_bn_bwd_apply<false, false, 1> : k_bn_bwd_apply<false, false, 4>), dim3(grid), dim3(256), 0, s, (const bf16_t*)gm,
                       (const bf16_t*)x, (const bf16_t*)nullptr, (bf16_t*)gx, (bf16_t*)nullptr, M, C, coef);
  }
  BIGDL_CHECK_LAUNCH();
}

// Apply-only backward: gx = A·gm + B·x + Cc with precomputed coefficients (coef [3][C]) — the
// materialisation of a deferred BN input gradient whose consumer could not take it as a prologue.
BIGDL_EXPORT int bigdl_bn_bwd_apply_coef(const void* gm, const void* x, void* gx, long long M, int C,
                                         const float* coef, hipStream_t s) {
  if (C % 8 || M <= 0 || !gm || !x || !gx || !coef) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL((apply_unroll1() ? k_bn_bwd_apply<false, false, 1> : k_bn_bwd_apply<false, false, 4>),
                     dim3(apply_grid(M, C)), dim3(256), 0, s, (const bf16_t*)gm, (const bf16_t*)x,
                     (const bf16_t*)nullptr, (bf16_t*)gx, (bf16_t*)nullptr, M, C, coef);
  BIGDL_CHECK_LAUNCH();
}

// ------------------------------------------------------------------------------------------------ fused finalize
// Statistics accumulated with fp32 atomics (the producing conv's epilogue, ConvParams::stats_atomic,
// ADDS each tile's partial sums into sums[2][C]; sums[2C] is an arrival counter, zero between uses):
// the apply kernel derives the per-channel coefficients from those 2·C sums in its prologue, so a
// training BN is ONE launch after its conv (no fold / finalize kernels).  Every block reads the sums;
// after its last read each block takes an arrival ticket, and the block that arrives last (all the
// others have finished reading) writes the saved statistics, the coefficient vectors and the
// running-statistics update, then re-zeroes the sums and the counter for the next producer.  The
// running mean may be the statistics shift K itself (it is read by every block), which is why only
// the last arriver may update it.  Nothing is read that another block wrote, so the ticket needs no
// acquire; the writes reach later kernels through the kernel boundary.
struct BnFwdFin {
  float* sums;           // [2C] Σ(y−K), Σ(y−K)², then the counter word
  const float* kshift;   // K (nullable: 0)
  const float* gamma;
  const float* beta;
  const float* in_bias;
  float* run_mean;
  float* run_var;
  float* save_mean;
  float* save_invstd;
  float* coef;           // [2C] scale, shift
  double M;
  float momentum, eps;
  // SyncBN (bigdl_bn_fwd_train_sums_fin): the row count read on the device (the all-reduced count at
  // sums[2C]), the arrival ticket in a word of its own, and `keep` = leave the sums as they are
  const float* dM;
  unsigned* ticket;
  int keep;
  // early = nothing the kernel's blocks read is written by it (kshift is not the running mean and
  // the sums are kept): block 0 writes the saved statistics / coefficients / running statistics
  // right after its prologue, and there is no last-block election at all
  int early;
  // local BN, one launch (bigdl_bn_fwd_train_rep_fin): the statistics are the producing conv's R
  // replicated rows rep [2][R][C] (reduced per channel in every block's prologue, instead of a
  // separate finalize launch); block 0 clears zero_next (the OTHER replica set, which the next
  // producer adds into) — this kernel's own set is cleared by the next step's consumer
  const float* rep;
  int R;
  float* zero_next;
};

__device__ __forceinline__ void fin_fwd_sums(const BnFwdFin& f, int C, int c, double& s, double& q) {
  if (f.rep) {
    s = 0.0;
    q = 0.0;
    for (int r = 0; r < f.R; ++r) {
      s += (double)f.rep[(size_t)r * C + c];
      q += (double)f.rep[((size_t)f.R + r) * C + c];
    }
  } else {
    s = (double)f.sums[c];
    q = (double)f.sums[C + c];
  }
}

// zero n floats (n % 4 == 0, 16-B aligned) with this block's threads
__device__ __forceinline__ void block_zero(float* p, long long n) {
  for (long long i = (long long)threadIdx.x * 4; i < n; i += (long long)blockDim.x * 4)
    *reinterpret_cast<float4*>(p + i) = make_float4(0.f, 0.f, 0.f, 0.f);
}

__device__ __forceinline__ void fin_fwd_coef(const BnFwdFin& f, int C, int c, float& mean, float& var, float& invstd,
                                             float& sc, float& sh) {
  const double Mg = f.dM ? (double)*f.dM : f.M;
  double s1, s2;
  fin_fwd_sums(f, C, c, s1, s2);
  const double dm = s1 / Mg;
  var = (float)fmax(s2 / Mg - dm * dm, 0.0);
  mean = (f.kshift ? f.kshift[c] : 0.f) + (float)dm;
  invstd = rsqrtf(var + f.eps);
  sc = (f.gamma ? f.gamma[c] : 1.f) * invstd;
  sh = (f.beta ? f.beta[c] : 0.f) - mean * sc;
}

// the arrival ticket of a block that has finished reading `sums`; true in the last block
__device__ __forceinline__ bool last_arriver(unsigned* cnt) {
  __shared__ int last;
  __syncthreads();
  if (threadIdx.x == 0) last = atomicAdd(cnt, 1u) == gridDim.x - 1 ? 1 : 0;
  __syncthreads();
  return last != 0;
}

// Two-level election over a ticket block of kTicketLeaves + 1 words (root first): block b counts
// into leaf b % kTicketLeaves, each leaf's last arriver into the root.  ~1000 blocks arriving at
// once on ONE word serialise at its L2 channel for microseconds; 16 leaves cut that 16x.  Every
// word is back at zero when the elected block returns (the next launch reuses the block).
constexpr int kTicketLeaves = 16;
__device__ __forceinline__ bool last_arriver_tree(unsigned* cnt) {
  __shared__ int last;
  __syncthreads();
  if (threadIdx.x == 0) {
    const unsigned nb = gridDim.x, leaf = blockIdx.x % kTicketLeaves;
    const unsigned in_leaf = (nb - leaf + kTicketLeaves - 1) / kTicketLeaves;
    const unsigned leaves = nb < (unsigned)kTicketLeaves ? nb : (unsigned)kTicketLeaves;
    int l = 0;
    if (atomicAdd(&cnt[1 + leaf], 1u) == in_leaf - 1) {
      atomicExch(&cnt[1 + leaf], 0u);
      if (atomicAdd(&cnt[0], 1u) == leaves - 1) {
        atomicExch(&cnt[0], 0u);
        l = 1;
      }
    }
    last = l;
  }
  __syncthreads();
  return last != 0;
}

__device__ __forceinline__ void rezero_sums(float* sums, int C) {
  for (int i = threadIdx.x; i < 2 * C; i += blockDim.x) sums[i] = 0.f;
  if (threadIdx.x == 0) *reinterpret_cast<unsigned*>(sums + 2 * C) = 0u;
}

__device__ __forceinline__ void fin_fwd_side(const BnFwdFin& f, int C);

template <bool RES, bool RELU, bool BITS>
__global__ void __launch_bounds__(256) k_bn_apply_fin(const bf16_t* __restrict__ x, const bf16_t* __restrict__ res,
                                                      bf16_t* __restrict__ y, long long M, int C, BnFwdFin f,
                                                      uint8_t* __restrict__ bits) {
  // the block derives every channel's scale / shift once into LDS ([2][C], dynamic), then streams
  // exactly like k_bn_apply (per-thread derivation of its 8 channels cost 2x on the relu-only tails)
  extern __shared__ __attribute__((aligned(16))) float cf[];
  const int t = threadIdx.x;
  for (int c = t; c < C; c += blockDim.x) {
    float mean, var, invstd;
    fin_fwd_coef(f, C, c, mean, var, invstd, cf[c], cf[C + c]);
  }
  __syncthreads();
  if (f.early) {
    if (blockIdx.x == 0) {
      fin_fwd_side(f, C);
      if (f.zero_next) block_zero(f.zero_next, 2LL * f.R * C);
    }
    bn_apply_rows<RES, RELU, BITS, 4>(x, res, y, M, C, cf, cf + C, bits);
    return;
  }
  bn_apply_rows<RES, RELU, BITS, 4>(x, res, y, M, C, cf, cf + C, bits);
  if (!(f.ticket ? last_arriver_tree(f.ticket) : last_arriver(reinterpret_cast<unsigned*>(f.sums + 2 * C)))) return;
  fin_fwd_side(f, C);
  __syncthreads();  // every coefficient is computed before the sums are cleared
  if (!f.keep) rezero_sums(f.sums, C);
}

// The saved statistics, the coefficient vectors and the running-statistics update (one block).
__device__ __forceinline__ void fin_fwd_side(const BnFwdFin& f, int C) {
  const double Mg = f.dM ? (double)*f.dM : f.M;
  for (int c = threadIdx.x; c < C; c += blockDim.x) {
    float mean, var, invstd, sc, sh;
    fin_fwd_coef(f, C, c, mean, var, invstd, sc, sh);
    f.save_mean[c] = mean;
    f.save_invstd[c] = invstd;
    f.coef[c] = sc;
    f.coef[C + c] = sh;
    if (f.run_mean) {
      const float unb = Mg > 1.0 ? (float)(var * Mg / (Mg - 1.0)) : var;
      const float true_mean = mean + (f.in_bias ? f.in_bias[c] : 0.f);
      f.run_mean[c] = (1.f - f.momentum) * f.run_mean[c] + f.momentum * true_mean;
      f.run_var[c] = (1.f - f.momentum) * f.run_var[c] + f.momentum * unb;
    }
  }
}

// Training BN forward from atomically accumulated conv-epilogue statistics: ONE launch (see above).
// sums: [2C + 1] fp32 (counter word last, zero on entry); shift: the K the conv subtracted.
BIGDL_EXPORT int bigdl_bn_fwd_train_sums_apply(const void* x, const void* res, void* y, long long M, int C,
                                               const float* gamma, const float* beta, const float* in_bias,
                                               float* run_mean, float* run_var, float momentum, float eps,
                                               float* save_mean, float* save_invstd, float* sums, const float* shift,
                                               float* coef, int relu, void* bits, hipStream_t s) {
  if (C % 8 || C > 8192 || M <= 0 || !sums || !save_mean || !save_invstd || !coef || (bits && !relu))
    return (int)hipErrorInvalidValue;
  BnFwdFin f{sums, shift, gamma, beta, in_bias, run_mean, run_var, save_mean, save_invstd, coef, (double)M, momentum,
             eps};
  const int grid = apply_grid(M, C);
  const bf16_t* xr = (const bf16_t*)x;
  const bf16_t* rr = (const bf16_t*)res;
  bf16_t* yr = (bf16_t*)y;
  uint8_t* br = (uint8_t*)bits;
  if (relu && bits && res) hipLaunchKernelGGL((k_bn_apply_fin<true, true, true>), dim3(grid), dim3(256), 8 * C, s, xr, rr, yr, M, C, f, br);
  else if (relu && bits) hipLaunchKernelGGL((k_bn_apply_fin<false, true, true>), dim3(grid), dim3(256), 8 * C, s, xr, rr, yr, M, C, f, br);
  else if (res && relu) hipLaunchKernelGGL((k_bn_apply_fin<true, true, false>), dim3(grid), dim3(256), 8 * C, s, xr, rr, yr, M, C, f, br);
  else if (res) hipLaunchKernelGGL((k_bn_apply_fin<true, false, false>), dim3(grid), dim3(256), 8 * C, s, xr, rr, yr, M, C, f, br);
  else if (relu) hipLaunchKernelGGL((k_bn_apply_fin<false, true, false>), dim3(grid), dim3(256), 8 * C, s, xr, rr, yr, M, C, f, br);
  else hipLaunchKernelGGL((k_bn_apply_fin<false, false, false>), dim3(grid), dim3(256), 8 * C, s, xr, rr, yr, M, C, f, br);
  BIGDL_CHECK_LAUNCH();
}

// Local training BN forward in ONE launch from the producing conv's replicated statistics
// rep [2][R][C] (the conv epilogue's atomics, shifted by kshift): every block reduces the R rows
// of all C channels in its prologue, block 0 writes the saved statistics / coefficients / running
// statistics and clears zero_next [2][R][C] (the other replica set).  kshift must not be the
// running mean or save_mean (no block may read what block 0 writes: the caller's shift ring).
BIGDL_EXPORT int bigdl_bn_fwd_train_rep_fin(const void* x, const void* res, void* y, long long M, int C,
                                            const float* gamma, const float* beta, const float* in_bias,
                                            float* run_mean, float* run_var, float momentum, float eps,
                                            float* save_mean, float* save_invstd, const float* rep, int R,
                                            float* zero_next, const float* kshift, float* coef, int relu, void* bits,
                                            hipStream_t s) {
  if (C % 8 || C > 8192 || M <= 0 || !rep || R <= 0 || !save_mean || !save_invstd || !coef || (bits && !relu) ||
      (kshift && (kshift == run_mean || kshift == save_mean)) || ((uintptr_t)zero_next & 15))
    return (int)hipErrorInvalidValue;
  BnFwdFin f{nullptr, kshift, gamma, beta, in_bias, run_mean, run_var, save_mean, save_invstd, coef, (double)M,
             momentum, eps, nullptr, nullptr, 1, 1, rep, R, zero_next};
  const int grid = apply_grid(M, C);
  const bf16_t* xr = (const bf16_t*)x;
  const bf16_t* rr = (const bf16_t*)res;
  bf16_t* yr = (bf16_t*)y;
  uint8_t* br = (uint8_t*)bits;
  if (relu && bits && res) hipLaunchKernelGGL((k_bn_apply_fin<true, true, true>), dim3(grid), dim3(256), 8 * C, s, xr, rr, yr, M, C, f, br);
  else if (relu && bits) hipLaunchKernelGGL((k_bn_apply_fin<false, true, true>), dim3(grid), dim3(256), 8 * C, s, xr, rr, yr, M, C, f, br);
  else if (res && relu) hipLaunchKernelGGL((k_bn_apply_fin<true, true, false>), dim3(grid), dim3(256), 8 * C, s, xr, rr, yr, M, C, f, br);
  else if (res) hipLaunchKernelGGL((k_bn_apply_fin<true, false, false>), dim3(grid), dim3(256), 8 * C, s, xr, rr, yr, M, C, f, br);
  else if (relu) hipLaunchKernelGGL((k_bn_apply_fin<false, true, false>), dim3(grid), dim3(256), 8 * C, s, xr, rr, yr, M, C, f, br);
  else hipLaunchKernelGGL((k_bn_apply_fin<false, false, false>), dim3(grid), dim3(256), 8 * C, s, xr, rr, yr, M, C, f, br);
  BIGDL_CHECK_LAUNCH();
}

// Backward twin: the consumer conv's dgrad epilogue (bnx mode, stats_atomic) ADDED Σg', Σg'·(x − μ)
// into sums; gx = A·g' + B·x + Cc with the coefficients derived per block in the prologue; the last
// arriver accumulates dγ / dβ (and a folded producer bias's gradient), writes the coefficients (when
// `coef` is given: a deferred-gradient consumer), re-zeroes the sums.  gx == null: coefficients and
// parameter gradients only (one block).
struct BnBwdFin {
  float* sums;
  const float* gamma;
  const float* mean;
  const float* invstd;
  float* ggamma;
  float* gbeta;
  float gscale;
  float* cbias;
  float cbscale;
  float* coef;
  float M;
  // SyncBN (bigdl_bn_bwd_apply_sums): `sums` are the GLOBAL sums (the coefficients), `lsums` this
  // rank's (dγ, dβ and the folded bias over its Ml rows); dM / ticket / keep as in BnFwdFin
  const float* lsums;
  float Ml;
  const float* dM;
  unsigned* ticket;
  int keep;
  int early;  // as BnFwdFin: block 0 writes the side results after its prologue, no election
  const float* rep;  // as BnFwdFin: the consumer dgrad's replicated [2][R][C] sums
  int R;
  float* zero_next;
};

__device__ __forceinline__ void fin_bwd_coef(const BnBwdFin& f, int C, int c, float& a, float& dg, float& A, float& B,
                                             float& Cc) {
  if (f.rep) {
    double s = 0.0, q = 0.0;
    for (int r = 0; r < f.R; ++r) {
      s += (double)f.rep[(size_t)r * C + c];
      q += (double)f.rep[((size_t)f.R + r) * C + c];
    }
    a = (float)s;
    dg = (float)q;
  } else {
    a = f.sums[c];
    dg = f.sums[C + c];
  }
  const float is = f.invstd[c];
  dg *= is;
  const float gm = f.gamma ? f.gamma[c] : 1.f;
  A = gm * is;
  const float Mg = f.dM ? *f.dM : f.M;
  B = -gm * is * is * dg / Mg;
  Cc = -gm * is * a / Mg - B * f.mean[c];
}

__device__ __forceinline__ void fin_bwd_side(const BnBwdFin& f, int C);

__global__ void __launch_bounds__(256) k_bn_bwd_apply_fin(const bf16_t* __restrict__ gy, const bf16_t* __restrict__ x,
                                                          bf16_t* __restrict__ gx, long long M, int C, BnBwdFin f) {
  // coefficients once per block into LDS ([3][C], dynamic), then the k_bn_bwd_apply stream
  extern __shared__ __attribute__((aligned(16))) float cf[];
  const int t = threadIdx.x;
  if (gx) {
    for (int c = t; c < C; c += blockDim.x) {
      float a, dg;
      fin_bwd_coef(f, C, c, a, dg, cf[c], cf[C + c], cf[2 * C + c]);
    }
    __syncthreads();
  }
  if (f.early) {
    if (blockIdx.x == 0) {
      fin_bwd_side(f, C);
      if (f.zero_next) block_zero(f.zero_next, 2LL * f.R * C);
    }
    if (gx) bn_bwd_apply_rows<false, false, 4>(gy, x, nullptr, gx, nullptr, M, C, cf);
    return;
  }
  if (gx) bn_bwd_apply_rows<false, false, 4>(gy, x, nullptr, gx, nullptr, M, C, cf);
  if (!(f.ticket ? last_arriver_tree(f.ticket) : last_arriver(reinterpret_cast<unsigned*>(f.sums + 2 * C)))) return;
  fin_bwd_side(f, C);
  __syncthreads();
  if (!f.keep) rezero_sums(f.sums, C);
}

// dγ / dβ, the folded producer bias's gradient and the coefficient vectors (one block).
__device__ __forceinline__ void fin_bwd_side(const BnBwdFin& f, int C) {
  const float Ml = f.lsums ? f.Ml : (f.dM ? *f.dM : f.M);
  for (int c = threadIdx.x; c < C; c += blockDim.x) {
    float a, dg, A, B, Cc;
    fin_bwd_coef(f, C, c, a, dg, A, B, Cc);
    if (f.lsums) {  // this rank's share: dγ, dβ (and the bias) over its own rows
      a = f.lsums[c];
      dg = f.lsums[C + c] * f.invstd[c];
    }
    if (f.ggamma) f.ggamma[c] += f.gscale * dg;
    if (f.gbeta) f.gbeta[c] += f.gscale * a;
    if (f.cbias) f.cbias[c] += f.cbscale * (A * a + B * Ml * f.mean[c] + Ml * Cc);
    if (f.coef) {
      f.coef[c] = A;
      f.coef[C + c] = B;
      f.coef[2 * C + c] = Cc;
    }
  }
}

BIGDL_EXPORT int bigdl_bn_bwd_sums_apply(const void* gm, const void* x, void* gx, long long M, int C, const float* gamma,
                                         const float* mean, const float* invstd, float* ggamma, float* gbeta,
                                         float gscale, float* cbias, float cbscale, float* sums, float* coef,
                                         hipStream_t s) {
  if (C % 8 || C > 4096 || M <= 0 || !sums || !mean || !invstd || (gx && (!gm || !x))) return (int)hipErrorInvalidValue;
  BnBwdFin f{sums, gamma, mean, invstd, ggamma, gbeta, gscale, cbias, cbscale, coef, (float)M};
  const int grid = gx ? apply_grid(M, C) : 1;
  hipLaunchKernelGGL(k_bn_bwd_apply_fin, dim3(grid), dim3(256), gx ? 12 * C : 0, s, (const bf16_t*)gm, (const bf16_t*)x,
                     (bf16_t*)gx, M, C, f);
  BIGDL_CHECK_LAUNCH();
}

// Backward twin of bigdl_bn_fwd_train_rep_fin: the consumer dgrad epilogue's replicated
// [Σg', Σg'·(x − μ)] rows; gx = A·g' + B·x + Cc (gm already ReLU-masked), block 0 accumulates dγ / dβ
// (and a folded producer bias) and clears zero_next.  gx null: one block, parameter gradients only.
BIGDL_EXPORT int bigdl_bn_bwd_rep_fin(const void* gm, const void* x, void* gx, long long M, int C, const float* gamma,
                                      const float* mean, const float* invstd, float* ggamma, float* gbeta, float gscale,
                                      float* cbias, float cbscale, const float* rep, int R, float* zero_next,
                                      float* coef, hipStream_t s) {
  if (C % 8 || C > 4096 || M <= 0 || !rep || R <= 0 || !mean || !invstd || (gx && (!gm || !x)) ||
      ((uintptr_t)zero_next & 15))
    return (int)hipErrorInvalidValue;
  BnBwdFin f{nullptr, gamma, mean, invstd, ggamma, gbeta, gscale, cbias, cbscale, coef, (float)M, nullptr, 0.f,
             nullptr, nullptr, 1, 1, rep, R, zero_next};
  const int grid = gx ? apply_grid(M, C) : 1;
  hipLaunchKernelGGL(k_bn_bwd_apply_fin, dim3(grid), dim3(256), gx ? 12 * C : 0, s, (const bf16_t*)gm, (const bf16_t*)x,
                     (bf16_t*)gx, M, C, f);
  BIGDL_CHECK_LAUNCH();
}


// ------------------------------------------------------------------------------------------------ SyncBN
// Cross-rank BatchNormalization (P6 / X11, SpatialBatchNormalization.scala:1114-1151,1257-1329):
// each rank reduces its partials to one [2][C] fp32 vector (Σ(x−K), Σ(x−K)² forward; Σg, Σg·(x−μ)
// backward), the host all-reduces those 2·C floats over RCCL, and the finalize/apply kernels below
// take the GLOBAL sums (G = 1 row) with the global row count — the same finalize code as the local
// path, so SyncBN costs two tiny kernels and one 2·C collective per direction.
template <typename T>
__global__ void __launch_bounds__(32 * kFinRG) k_bn_sum_rows(const T* __restrict__ partial, int G, int C,
                                                      float* __restrict__ out, float* __restrict__ out2, float cnt,
                                                      float* rezero = nullptr) {
  __shared__ double lds[kFinRG][2][33];
  double a, b;
  reduce_partials(partial, G, C, blockIdx.x * 32, lds, a, b, rezero);
  const int c = blockIdx.x * 32 + (threadIdx.x & 31);
  if ((threadIdx.x >> 5) != 0 || c >= C) return;
  // this rank's row count behind the sums of the buffer the collective reduces ([2C + 1])
  if (cnt >= 0.f && c == 0) (out2 ? out2 : out)[2 * C] = cnt;
  out[c] = (float)a;
  out[C + c] = (float)b;
  if (out2) {  // a second copy (the buffer the collective sums in place, next to the local sums)
    out2[c] = (float)a;
    out2[C + c] = (float)b;
  }
}

static void sum_rows(const float* partial, int G, int C, float* scratch, float* out, hipStream_t s,
                     float* out2 = nullptr, float cnt = -1.f, bool rezero = false) {
  if (!rezero && maybe_fold(partial, G, C, scratch, s))
    hipLaunchKernelGGL(k_bn_sum_rows<double>, dim3((C + 31) / 32), dim3(32 * kFinRG), 0, s, (const double*)scratch, G, C, out,
                       out2, cnt);
  else
    hipLaunchKernelGGL(k_bn_sum_rows<float>, dim3((C + 31) / 32), dim3(32 * kFinRG), 0, s, partial, G, C, out, out2, cnt,
                       rezero ? const_cast<float*>(partial) : nullptr);
}

// Local shifted sums of x (kshift = the running mean, identical on every rank): out[2C], and the row
// count (cnt ≥ 0) at out[2C].
BIGDL_EXPORT int bigdl_bn_stats_sums(const void* x, long long M, int C, const float* kshift, float* ws,
                                     float* scratch, float* out, float cnt, hipStream_t s) {
  if (C % 8 || M <= 0 || !kshift) return (int)hipErrorInvalidValue;
  int G = bigdl_bn_num_partials(M, C);
  long long rpb = (M + G - 1) / G;
  size_t sm = stats_smem(C);
  if (sm > 64 * 1024) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(k_bn_stats, dim3(G), dim3(256), sm, s, (const bf16_t*)x, M, C, rpb, ws, G, kshift);
  sum_rows(ws, G, C, scratch, out, s, nullptr, cnt);
  BIGDL_CHECK_LAUNCH();
}

// Reduce G partial rows (a conv epilogue's, or any [2][G][C] fp32 block) to out[2C] (and the same
// values to out2[2C] when given: the copy an in-place all-reduce turns into the global sums).
// rezero: `partial` is a replicated atomic-statistics buffer (G ≤ 512 replicas) cleared after reading
BIGDL_EXPORT int bigdl_bn_partials_sums(const float* partial, int G, int C, float* scratch, float* out, float cnt,
                                        int rezero, hipStream_t s) {
  if (C <= 0 || G <= 0 || (rezero && G > 512)) return (int)hipErrorInvalidValue;
  sum_rows(partial, G, C, scratch, out, s, nullptr, cnt, rezero != 0);
  BIGDL_CHECK_LAUNCH();
}

BIGDL_EXPORT int bigdl_bn_partials_sums2(const float* partial, int G, int C, float* scratch, float* out, float* out2,
                                         float cnt, int rezero, hipStream_t s) {
  if (C <= 0 || G <= 0 || (rezero && G > 512)) return (int)hipErrorInvalidValue;
  sum_rows(partial, G, C, scratch, out, s, out2, cnt, rezero != 0);
  BIGDL_CHECK_LAUNCH();
}

// Forward from GLOBAL sums (2C, shifted by kshift): finalize over `count` rows (all ranks; 0 = the
// all-reduced count stored at sums[2C]), apply to this rank's M rows.  y == null: finalize only (a
// SyncBN shortcut BN whose apply is deferred into the block tail's); rcoef (with res): the residual is
// a deferred BN output res·rcoef[c] + rcoef[C + c], applied inside this pass (as
// bigdl_bn_fwd_train_partials2).
BIGDL_EXPORT int bigdl_bn_fwd_train_sums(const void* x, const void* res, const float* rcoef, void* y, long long M,
                                         long long count, int C, const float* gamma, const float* beta,
                                         const float* in_bias, float* run_mean, float* run_var, float momentum,
                                         float eps, float* save_mean, float* save_invstd, const float* sums,
                                         const float* kshift, float* coef, int relu, void* bits, unsigned* ticket,
                                         hipStream_t s) {
  if (C % 8 || M <= 0 || count < 0 || (bits && !relu) || (rcoef && !res) || (!y && (res || bits)))
    return (int)hipErrorInvalidValue;
  if (ticket && C <= 8192 && y && !rcoef) {
    // ONE launch: every block derives its channels' coefficients from the global sums, the last
    // arriver writes the saved statistics / coefficients / running statistics (k_bn_apply_fin)
    BnFwdFin f{const_cast<float*>(sums), kshift, gamma, beta, in_bias, run_mean, run_var, save_mean, save_invstd, coef,
               (double)count, momentum, eps, count == 0 ? sums + 2 * C : nullptr, ticket, 1,
               (kshift != run_mean && kshift != save_mean) ? 1 : 0};
    const int grid = apply_grid(M, C);
    const bf16_t* xr = (const bf16_t*)x;
    const bf16_t* rr = (const bf16_t*)res;
    bf16_t* yr = (bf16_t*)y;
    uint8_t* br = (uint8_t*)bits;
    if (relu && bits && res) hipLaunchKernelGGL((k_bn_apply_fin<true, true, true>), dim3(grid), dim3(256), 8 * C, s, xr, rr, yr, M, C, f, br);
    else if (relu && bits) hipLaunchKernelGGL((k_bn_apply_fin<false, true, true>), dim3(grid), dim3(256), 8 * C, s, xr, rr, yr, M, C, f, br);
    else if (res && relu) hipLaunchKernelGGL((k_bn_apply_fin<true, true, false>), dim3(grid), dim3(256), 8 * C, s, xr, rr, yr, M, C, f, br);
    else if (res) hipLaunchKernelGGL((k_bn_apply_fin<true, false, false>), dim3(grid), dim3(256), 8 * C, s, xr, rr, yr, M, C, f, br);
    else if (relu) hipLaunchKernelGGL((k_bn_apply_fin<false, true, false>), dim3(grid), dim3(256), 8 * C, s, xr, rr, yr, M, C, f, br);
    else hipLaunchKernelGGL((k_bn_apply_fin<false, false, false>), dim3(grid), dim3(256), 8 * C, s, xr, rr, yr, M, C, f, br);
    BIGDL_CHECK_LAUNCH();
  }
  hipLaunchKernelGGL(k_bn_finalize<float>, dim3((C + 31) / 32), dim3(32 * kFinRG), 0, s, (const bf16_t*)nullptr, kshift, sums,
                     1, count, C, gamma, beta, in_bias, run_mean, run_var, momentum, eps, save_mean, save_invstd, coef,
                     coef + C, count == 0 ? sums + 2 * C : nullptr);
  if (y) launch_apply(x, res, y, M, C, coef, relu, bits, s, rcoef);
  BIGDL_CHECK_LAUNCH();
}

// Backward local sums: Σg', Σg'·(x − mean) (g' = gy masked by y > 0 when relu) → out[2C] and the
// same values in out[2C..4C) (the copy the all-reduce turns into the global sums).
BIGDL_EXPORT int bigdl_bn_bwd_sums(const void* gy, const void* x, const void* y, long long M, int C, const float* mean,
                                   float* ws, float* scratch, float* out, int relu, float cnt, hipStream_t s) {
  if (C % 8 || M <= 0) return (int)hipErrorInvalidValue;
  int G = bigdl_bn_num_partials(M, C);
  long long rpb = (M + G - 1) / G;
  size_t sm = stats_smem(C);
  if (relu)
    hipLaunchKernelGGL(k_bn_bwd_reduce<true>, dim3(G), dim3(256), sm, s, (const bf16_t*)gy, (const bf16_t*)x,
                       (const bf16_t*)y, M, C, rpb, mean, ws, G);
  else
    hipLaunchKernelGGL(k_bn_bwd_reduce<false>, dim3(G), dim3(256), sm, s, (const bf16_t*)gy, (const bf16_t*)x,
                       (const bf16_t*)y, M, C, rpb, mean, ws, G);
  sum_rows(ws, G, C, scratch, out, s, out + 2 * C, cnt);
  BIGDL_CHECK_LAUNCH();
}

// Gradient of a producer bias folded into a SyncBN: this rank's Σ_rows gx = A·Σ_l g' + B·Σ_l x +
// M_l·Cc with the GLOBAL coefficients; Σ_l x is taken as M_l·μ (exact at one rank; across ranks the
// per-rank deviations B·(Σ_l x − M_l·μ) cancel in the gradient all-reduce, since Σ_ranks = N·μ).
__global__ void __launch_bounds__(256) k_bn_cbias_sync(const float* __restrict__ local_sums,
                                                       const float* __restrict__ coef, const float* __restrict__ mean,
                                                       long long M, int C, float* __restrict__ cbias, float cbscale) {
  const int c = blockIdx.x * 256 + threadIdx.x;
  if (c >= C) return;
  const float A = coef[c], B = coef[C + c], Cc = coef[2 * C + c];
  cbias[c] += cbscale * (A * local_sums[c] + (float)M * (B * mean[c] + Cc));
}

// Backward from sums: the LOCAL sums accumulate this rank's dγ, dβ (the data-parallel gradient
// all-reduce sums them across ranks); the GLOBAL sums over `count` rows give the input-gradient
// coefficients, applied to this rank's M rows.  ``cbias``: see k_bn_cbias_sync.
BIGDL_EXPORT int bigdl_bn_bwd_apply_sums(const void* gy, const void* x, const void* y, void* gx, long long M,
                                         long long count, int C, const float* gamma, const float* mean,
                                         const float* invstd, float* ggamma, float* gbeta, float gscale,
                                         const float* local_sums, const float* global_sums, float* coef,
                                         float* coef_scratch, int relu, float* cbias, float cbscale, unsigned* ticket,
                                         hipStream_t s) {
  if (C % 8 || M <= 0 || count < 0) return (int)hipErrorInvalidValue;
  const float* dM = count == 0 ? global_sums + 2 * C : nullptr;  // the all-reduced count
  if (ticket && !relu && C <= 4096) {
    // ONE launch (k_bn_bwd_apply_fin): coefficients from the global sums in every block, this rank's
    // dγ / dβ / folded-bias share from its local sums in the last arriver
    BnBwdFin f{const_cast<float*>(global_sums), gamma, mean, invstd, ggamma, gbeta, gscale, cbias, cbscale, nullptr,
               (float)count, local_sums, (float)M, dM, ticket, 1, 1};
    const int grid = gx ? apply_grid(M, C) : 1;
    hipLaunchKernelGGL(k_bn_bwd_apply_fin, dim3(grid), dim3(256), gx ? 12 * C : 0, s, (const bf16_t*)gy,
                       (const bf16_t*)x, (bf16_t*)gx, M, C, f);
    BIGDL_CHECK_LAUNCH();
  }
  if (ggamma || gbeta)
    hipLaunchKernelGGL(k_bn_bwd_finalize<float>, dim3((C + 31) / 32), dim3(32 * kFinRG), 0, s, local_sums, 1, count, C, gamma,
                       mean, invstd, ggamma, gbeta, gscale, (float*)nullptr, 0.f, coef_scratch, dM);
  hipLaunchKernelGGL(k_bn_bwd_finalize<float>, dim3((C + 31) / 32), dim3(32 * kFinRG), 0, s, global_sums, 1, count, C, gamma,
                     mean, invstd, (float*)nullptr, (float*)nullptr, 0.f, (float*)nullptr, 0.f, coef, dM);
  if (cbias)
    hipLaunchKernelGGL(k_bn_cbias_sync, dim3((C + 255) / 256), dim3(256), 0, s, local_sums, coef, mean, M, C, cbias,
                       cbscale);
  if (gx) {
    int grid = apply_grid(M, C);
    const bf16_t *g_ = (const bf16_t*)gy, *x_ = (const bf16_t*)x, *y_ = (const bf16_t*)y;
    bf16_t* gx_ = (bf16_t*)gx;
    if (relu)
      hipLaunchKernelGGL((apply_unroll1() ? k_bn_bwd_apply<true, false, 1> : k_bn_bwd_apply<true, false, 4>), dim3(grid), dim3(256), 0, s, g_, x_, y_, gx_, (bf16_t*)nullptr, M, C,
                         coef);
    else
      hipLaunchKernelGGL((apply_unroll1() ? k_bn_bwd_apply<false, false, 1> : k_bn_bwd_apply<false, false, 4>), dim3(grid), dim3(256), 0, s, g_, x_, y_, gx_, (bf16_t*)nullptr, M,
                         C, coef);
  }
  BIGDL_CHECK_LAUNCH();
}

// ------------------------------------------------------------------------------------------------ fp32
// fp32 NHWC BatchNormalization (bigdl.compute.dtype=fp32 on a GPU, next to the bf16x3 convolutions of
// precision.hip): the same pass structure and finalize kernels as the bf16 path, 8 fp32 channels
// (two 16-B loads) per thread and row.  Statistics are shifted by row 0 (kshift = x itself).
__device__ __forceinline__ void ld8f(const float* __restrict__ p, float (&v)[8]) {
  const float4 a = *reinterpret_cast<const float4*>(p), b = *reinterpret_cast<const float4*>(p + 4);
  v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w; v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
}
__device__ __forceinline__ void st8f(float* __restrict__ p, const float (&v)[8]) {
  *reinterpret_cast<float4*>(p) = make_float4(v[0], v[1], v[2], v[3]);
  *reinterpret_cast<float4*>(p + 4) = make_float4(v[4], v[5], v[6], v[7]);
}

// mode 0: partial = Σ(x − x[row 0]), Σ(x − x[row 0])²;  mode 1 (backward): Σg', Σg'·(x − mean)
template <int MODE, bool RELU>
__global__ void __launch_bounds__(256) k_bn32_reduce(const float* __restrict__ x, const float* __restrict__ gy,
                                                     const float* __restrict__ y, long long M, int C,
                                                     long long rows_per_block, const float* __restrict__ ref,
                                                     float* __restrict__ partial, int G,
                                                     const uint8_t* __restrict__ mbits = nullptr) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  BnGeom g = bn_geom(C);
  const int t = threadIdx.x;
  const int cg_local = t % g.tpr;
  const int r_off = t / g.tpr;
  const long long r0 = (long long)blockIdx.x * rows_per_block;
  long long r1 = r0 + rows_per_block;
  if (r1 > M) r1 = M;
  float* s_a = smem;
  float* s_b = smem + g.RPI * C;
  for (int cg = cg_local; cg < g.CG; cg += g.tpr) {
    float K[8], a[8], b[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) { K[k] = ref[cg * 8 + k]; a[k] = 0.f; b[k] = 0.f; }
    if (r_off < g.RPI) {
      for (long long r = r0 + r_off; r < r1; r += g.RPI) {
        const size_t off = (size_t)r * C + (size_t)cg * 8;
        float xv[8];
        ld8f(x + off, xv);
        if (MODE == 0) {
#pragma unroll
          for (int k = 0; k < 8; ++k) {
            const float d = xv[k] - K[k];
            a[k] += d;
            b[k] = fmaf(d, d, b[k]);
          }
        } else {
          float gv[8];
          ld8f(gy + off, gv);
          if (RELU) {
            if (mbits) {  // the forward's ReLU mask, one bit per element (8 channels per byte)
              const unsigned mb = mbits[(size_t)r * (C >> 3) + cg];
#pragma unroll
              for (int k = 0; k < 8; ++k) gv[k] = (mb >> k) & 1u ? gv[k] : 0.f;
            } else {
              float yv[8];
              ld8f(y + off, yv);
#pragma unroll
              for (int k = 0; k < 8; ++k) gv[k] = yv[k] > 0.f ? gv[k] : 0.f;
            }
          }
#pragma unroll
          for (int k = 0; k < 8; ++k) {
            a[k] += gv[k];
            b[k] = fmaf(gv[k], xv[k] - K[k], b[k]);
          }
        }
      }
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        s_a[r_off * C + cg * 8 + k] = a[k];
        s_b[r_off * C + cg * 8 + k] = b[k];
      }
    }
  }
  __syncthreads();
  for (int c = t; c < C; c += 256) {
    float a = 0.f, b = 0.f;
    for (int i = 0; i < g.RPI; ++i) {
      a += s_a[i * C + c];
      b += s_b[i * C + c];
    }
    partial[(size_t)blockIdx.x * C + c] = a;
    partial[(size_t)(G + blockIdx.x) * C + c] = b;
  }
}

// forward: y = relu?(x·scale + shift (+ res));  backward (BWD): gx = A·g' + B·x + Cc, g' = gy masked
// by y > 0 (RELU), g' also stored to gres when given.
// kU32 rows per trip with every load issued before the first use (as bn_apply_rows): one row per trip
// left each thread with a single 32-B request in flight and the pass latency-bound (11.4 ms of the
// fp32 ResNet-50 step at ≈3.6 TB/s, profiles/r5_fp32_profile.txt).  x / aux are read once per pass:
// non-temporal loads keep them from displacing reusable lines.
__device__ __forceinline__ void ld8f_nt(const float* __restrict__ p, float (&v)[8]) {
  typedef float f32x4 __attribute__((ext_vector_type(4)));
  const f32x4 a = __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(p));
  const f32x4 b = __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(p + 4));
  v[0] = a[0]; v[1] = a[1]; v[2] = a[2]; v[3] = a[3]; v[4] = b[0]; v[5] = b[1]; v[6] = b[2]; v[7] = b[3];
}

template <bool BWD, bool RELU, int kU32 = 4>
__global__ void __launch_bounds__(256) k_bn32_apply(const float* __restrict__ x, const float* __restrict__ aux,
                                                    const float* __restrict__ y_mask, float* __restrict__ out,
                                                    float* __restrict__ gres, long long M, int C,
                                                    const float* __restrict__ coef, bf16_t* __restrict__ sp = nullptr,
                                                    uint8_t* __restrict__ mbits = nullptr) {
  BnGeom g = bn_geom(C);
  const int t = threadIdx.x;
  const int cg_local = t % g.tpr;
  const int r_off = t / g.tpr;
  if (r_off >= g.RPI) return;
  const long long rstride = (long long)gridDim.x * g.RPI;
  for (int cg = cg_local; cg < g.CG; cg += g.tpr) {
    float A[8], B[8], Cc[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      A[k] = coef[cg * 8 + k];
      B[k] = coef[C + cg * 8 + k];
      Cc[k] = BWD ? coef[2 * C + cg * 8 + k] : 0.f;
    }
    for (long long r = (long long)blockIdx.x * g.RPI + r_off; r < M; r += kU32 * rstride) {
      float xv[kU32][8], av[kU32][8];
      unsigned mbv[kU32];
#pragma unroll
      for (int u = 0; u < kU32; ++u) {
        const long long ru = r + u * rstride;
        const size_t off = (size_t)(ru < M ? ru : r) * C + (size_t)cg * 8;
        ld8f_nt(x + off, xv[u]);
        if (BWD || aux) ld8f_nt(aux + off, av[u]);
        if (BWD && RELU) {
          if (mbits) {
            mbv[u] = mbits[(size_t)(ru < M ? ru : r) * (C >> 3) + cg];
          } else {
            float yv[8];
            ld8f(y_mask + off, yv);
            unsigned m = 0;
#pragma unroll
            for (int k = 0; k < 8; ++k) m |= (yv[k] > 0.f ? 1u : 0u) << k;
            mbv[u] = m;
          }
        }
      }
#pragma unroll
      for (int u = 0; u < kU32; ++u) {
        const long long ru = r + u * rstride;
        if (ru >= M) break;
        const size_t off = (size_t)ru * C + (size_t)cg * 8;
        float o[8];
        if (BWD) {
          float gv[8];
#pragma unroll
          for (int k = 0; k < 8; ++k) gv[k] = (!RELU || ((mbv[u] >> k) & 1u)) ? av[u][k] : 0.f;
          if (gres) st8f(gres + off, gv);
#pragma unroll
          for (int k = 0; k < 8; ++k) o[k] = fmaf(A[k], gv[k], fmaf(B[k], xv[u][k], Cc[k]));
        } else {
#pragma unroll
          for (int k = 0; k < 8; ++k) {
            const float v = fmaf(xv[u][k], A[k], B[k]) + (aux ? av[u][k] : 0.f);
            o[k] = RELU ? fmaxf(v, 0.f) : v;
          }
          if (RELU && mbits) {  // the ReLU mask as bits for the backward (instead of re-reading y)
            unsigned mb = 0;
#pragma unroll
            for (int k = 0; k < 8; ++k) mb |= (o[k] > 0.f ? 1u : 0u) << k;
            mbits[(size_t)ru * (C >> 3) + cg] = (uint8_t)mb;
          }
        }
        if (out) st8f(out + off, o);
        if (sp) {  // the bf16x3 [hi | lo] split of the output for the consuming conv (fp32x3.py split2)
          uint32_t hw[4], lw[4];
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const bf16_t h0 = f2bf(o[2 * e]), h1 = f2bf(o[2 * e + 1]);
            const bf16_t l0 = f2bf(o[2 * e] - bf2f(h0)), l1 = f2bf(o[2 * e + 1] - bf2f(h1));
            hw[e] = (uint32_t)h0 | ((uint32_t)h1 << 16);
            lw[e] = (uint32_t)l0 | ((uint32_t)l1 << 16);
          }
          bf16_t* d = sp + (size_t)ru * 2 * C + (size_t)cg * 8;
          *reinterpret_cast<uint4*>(d) = make_uint4(hw[0], hw[1], hw[2], hw[3]);
          *reinterpret_cast<uint4*>(d + C) = make_uint4(lw[0], lw[1], lw[2], lw[3]);
        }
      }
    }
  }
}

// A/B knobs of the fp32 apply pass: BIGDL_BN32_UNROLL (rows in flight per thread: 1, 2 = default, 4,
// 8) and BIGDL_BN32_BLOCKS (grid cap, default the bf16 pass's apply_cap).  Round 6, whole fp32 step, 3
// interleaved repeats on two boxes: 2 rows 45.06-45.23 / 44.41-44.83 ms vs 4 rows 45.50-45.65 /
// 44.64-44.99 (8 rows and a 4096-block cap slower; profiles/r6_fp32_bn_unroll_ab.txt)
static int bn32_unroll() {
  static int u = [] {
    const char* e = getenv("BIGDL_BN32_UNROLL");
    const int v = e ? atoi(e) : 2;
    return (v == 1 || v == 4 || v == 8) ? v : 2;
  }();
  return u;
}
static int bn32_grid(long long M, int C) {
  static int cap = [] {
    const char* e = getenv("BIGDL_BN32_BLOCKS");
    return e ? atoi(e) : 0;
  }();
  if (cap < 64) return apply_grid(M, C);
  int CG = C / 8, tpr = CG < 256 ? CG : 256, rpi = 256 / tpr;
  long long blocks = (M + rpi - 1) / rpi;
  if (blocks > cap) blocks = cap;
  return (int)(blocks < 1 ? 1 : blocks);
}
template <bool BWD, bool RELU>
static void launch_bn32_apply(long long M, int C, hipStream_t s, const float* x, const float* aux, const float* y_mask,
                              float* out, float* gres, const float* coef, bf16_t* sp = nullptr,
                              uint8_t* mbits = nullptr) {
  const dim3 g(bn32_grid(M, C)), b(256);
  switch (bn32_unroll()) {
    case 1: hipLaunchKernelGGL((k_bn32_apply<BWD, RELU, 1>), g, b, 0, s, x, aux, y_mask, out, gres, M, C, coef, sp, mbits); break;
    case 4: hipLaunchKernelGGL((k_bn32_apply<BWD, RELU, 4>), g, b, 0, s, x, aux, y_mask, out, gres, M, C, coef, sp, mbits); break;
    case 8: hipLaunchKernelGGL((k_bn32_apply<BWD, RELU, 8>), g, b, 0, s, x, aux, y_mask, out, gres, M, C, coef, sp, mbits); break;
    default: hipLaunchKernelGGL((k_bn32_apply<BWD, RELU, 2>), g, b, 0, s, x, aux, y_mask, out, gres, M, C, coef, sp, mbits); break;
  }
}

static bool bn32_ok(const void* p) { return ((uintptr_t)p & 15) == 0; }

BIGDL_EXPORT int bigdl_bn32_fwd_train(const float* x, const float* res, float* y, long long M, int C,
                                      const float* gamma, const float* beta, const float* in_bias, float* run_mean,
                                      float* run_var, float momentum, float eps, float* save_mean, float* save_invstd,
                                      float* ws, float* coef, int relu, void* split, void* bits, hipStream_t s) {
  if (C % 8 || M <= 0 || !bn32_ok(x) || !bn32_ok(y) || (res && !bn32_ok(res)) || (split && !bn32_ok(split)))
    return (int)hipErrorInvalidValue;
  bf16_t* sp = (bf16_t*)split;
  const int G = bigdl_bn_num_partials(M, C);
  const long long rpb = (M + G - 1) / G;
  const size_t sm = stats_smem(C);
  if (sm > 64 * 1024) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL((k_bn32_reduce<0, false>), dim3(G), dim3(256), sm, s, x, nullptr, nullptr, M, C, rpb, x, ws, G);
  hipLaunchKernelGGL(k_bn_finalize<float>, dim3((C + 31) / 32), dim3(32 * kFinRG), 0, s, (const bf16_t*)nullptr, x,
                     (const float*)ws, G, M, C, gamma, beta, in_bias, run_mean, run_var, momentum, eps, save_mean,
                     save_invstd, coef, coef + C);
  if (relu)
    launch_bn32_apply<false, true>(M, C, s, x, res, nullptr, y, nullptr, coef, sp, (uint8_t*)bits);
  else
    launch_bn32_apply<false, false>(M, C, s, x, res, nullptr, y, nullptr, coef, sp);
  BIGDL_CHECK_LAUNCH();
}

// fp32 training forward from the replicated statistics the producing fp32-output conv added
// (bigdl_conv_fwd_f32out2_stats: [2][G][C], shifted by kshift, cleared here after reading): finalize +
// apply (+ the consuming conv's split and the ReLU mask bits, as bigdl_bn32_fwd_train).
BIGDL_EXPORT int bigdl_bn32_fwd_train_partials(const float* x, const float* res, float* y, long long M, int C,
                                               const float* gamma, const float* beta, const float* in_bias,
                                               float* run_mean, float* run_var, float momentum, float eps,
                                               float* save_mean, float* save_invstd, float* partial, int G,
                                               const float* kshift, float* coef, int relu, void* split, void* bits,
                                               hipStream_t s) {
  // y == null: finalize only (the consumer conv applies the BN + ReLU in its operand prologue)
  if (C % 8 || M <= 0 || G <= 0 || G > 512 || !partial || !bn32_ok(x) || (y && !bn32_ok(y)) || (res && !bn32_ok(res)) ||
      (split && !bn32_ok(split)) || (!y && (res || split || bits || !coef)))
    return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(k_bn_finalize<float>, dim3((C + 31) / 32), dim3(32 * kFinRG), 0, s, (const bf16_t*)nullptr, kshift,
                     (const float*)partial, G, M, C, gamma, beta, in_bias, run_mean, run_var, momentum, eps, save_mean,
                     save_invstd, coef, coef + C, nullptr, partial);
  if (!y) BIGDL_CHECK_LAUNCH();
  bf16_t* sp = (bf16_t*)split;
  if (relu)
    launch_bn32_apply<false, true>(M, C, s, x, res, nullptr, y, nullptr, coef, sp, (uint8_t*)bits);
  else
    launch_bn32_apply<false, false>(M, C, s, x, res, nullptr, y, nullptr, coef, sp);
  BIGDL_CHECK_LAUNCH();
}

// fp32 training backward from the replicated Σg', Σg'·(x − μ) the consumer conv's fp32 dgrad epilogue
// added (bigdl_conv_fwd_f32out2_bnbwd; gm = the ReLU-masked gradient it stored): finalize (clears the
// replicas) + gx = A·gm + B·x + Cc, with the producing conv's [hi | lo] dY split (split, optional).
BIGDL_EXPORT int bigdl_bn32_bwd_partials(const float* gm, const float* x, float* gx, long long M, int C,
                                         const float* gamma, const float* mean, const float* invstd, float* ggamma,
                                         float* gbeta, float gscale, float* cbias, float cbscale, float* partial, int G,
                                         float* coef, void* split, hipStream_t s) {
  if (C % 8 || M <= 0 || G <= 0 || G > 512 || !partial || !bn32_ok(x) || !bn32_ok(gm) || (gx && !bn32_ok(gx)) ||
      (split && (!gx || !bn32_ok(split))))
    return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(k_bn_bwd_finalize<float>, dim3((C + 31) / 32), dim3(32 * kFinRG), 0, s, (const float*)partial, G, M,
                     C, gamma, mean, invstd, ggamma, gbeta, gscale, cbias, cbscale, coef, nullptr, partial);
  if (gx) {
    launch_bn32_apply<true, false>(M, C, s, x, gm, nullptr, gx, nullptr, coef, (bf16_t*)split);
  }
  BIGDL_CHECK_LAUNCH();
}

BIGDL_EXPORT int bigdl_bn32_fwd_infer(const float* x, float* y, long long M, int C, const float* gamma,
                                      const float* beta, const float* run_mean, const float* run_var,
                                      const float* in_bias, float eps, float* coef, int relu, hipStream_t s) {
  if (C % 8 || M <= 0 || !bn32_ok(x) || !bn32_ok(y)) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(k_bn_infer_coef, dim3((C + 255) / 256), dim3(256), 0, s, C, gamma, beta, run_mean, run_var,
                     in_bias, eps, coef, coef + C);
  if (relu)
    launch_bn32_apply<false, true>(M, C, s, x, nullptr, nullptr, y, nullptr, coef);
  else
    launch_bn32_apply<false, false>(M, C, s, x, nullptr, nullptr, y, nullptr, coef);
  BIGDL_CHECK_LAUNCH();
}

// Backward.  ws: 2·G·C floats; coef: 3·C floats.  gx / gres optional; y is the BN+ReLU output (relu).
BIGDL_EXPORT int bigdl_bn32_bwd(const float* gy, const float* x, const float* y, float* gx, float* gres, long long M,
                                int C, const float* gamma, const float* mean, const float* invstd, float* ggamma,
                                float* gbeta, float gscale, float* cbias, float cbscale, float* ws, float* coef,
                                int relu, void* split, const void* bits, hipStream_t s) {
  if (C % 8 || M <= 0 || !bn32_ok(x) || !bn32_ok(gy) || (relu && !bits && (!y || !bn32_ok(y))) || (gx && !bn32_ok(gx)) ||
      (gres && !bn32_ok(gres)) || (split && (!gx || !bn32_ok(split))))
    return (int)hipErrorInvalidValue;
  bf16_t* sp = (bf16_t*)split;
  const int G = bigdl_bn_num_partials(M, C);
  const long long rpb = (M + G - 1) / G;
  const size_t sm = stats_smem(C);
  if (sm > 64 * 1024) return (int)hipErrorInvalidValue;
  uint8_t* mb = (uint8_t*)bits;
  if (relu)
    hipLaunchKernelGGL((k_bn32_reduce<1, true>), dim3(G), dim3(256), sm, s, x, gy, y, M, C, rpb, mean, ws, G, mb);
  else
    hipLaunchKernelGGL((k_bn32_reduce<1, false>), dim3(G), dim3(256), sm, s, x, gy, y, M, C, rpb, mean, ws, G);
  hipLaunchKernelGGL(k_bn_bwd_finalize<float>, dim3((C + 31) / 32), dim3(32 * kFinRG), 0, s, (const float*)ws, G, M, C,
                     gamma, mean, invstd, ggamma, gbeta, gscale, cbias, cbscale, coef);
  if (gx || gres) {
    if (relu)
      launch_bn32_apply<true, true>(M, C, s, x, gy, y, gx, gres, coef, sp, mb);
    else
      launch_bn32_apply<true, false>(M, C, s, x, gy, y, gx, gres, coef, sp);
  }
  BIGDL_CHECK_LAUNCH();
}
