// fp32-mode weight operands of a whole training step in ONE launch.
//
// The bf16x3 conv kernels (conv_x3.hip) read every filter as 32-index chunks stored [hi | lo]
// (hi = bf16(v), lo = bf16(v − hi), one 128-B LDS row per k-tile), the Linear GEMMs as [hi | lo | hi]
// rows; the backward-data convs need the flipped, channel-transposed filter (one sub-filter per
// output parity class of a strided conv).  Per layer and per step that was a flip, a permute copy, an
// index gather and a split launch (≈ 120 small launches, 1.2 ms of split kernels, at::native copies
// on the backward critical path; profiles/r5_fp32_profile.txt).  The master weights change once per
// step (the optimizer update), so every derived operand of an arena is refreshed by one launch of
// k_wx3_multi the first time a conv asks for one after the update (ops/fp32x3.py _wprep).
//
// Job kinds (the fp32 master read through 4 element strides, so any physical layout works):
//   0 FWD   chunk-split of the KRSC flattening: row k = (r, s, c) (c fastest), R·S·C % 32 == 0
//   1 DGRAD per class q: row c = (i, j, k) of W[k][c][rmap[i]][smap[j]] (k fastest), K % 32 == 0;
//           classes back to back at out_off[q] (elements of the chunk-split output)
//   2 S2D   the space-to-depth stem filter: row k = (a, b, ch), ch = c·4 + bh·2 + bw of
//           W[k][c][2a + bh][2b + bw] (0 outside R×S / C), 32 channels per (a, b)
//   3 ROWS3 [rows][3·cp] = [hi | lo | hi] of M[row][col] (0 for col ≥ cols or row ≥ nrows); rows = R
//           (padded row count), cp = S, nrows = K, cols = C; element (row, col) at row·sK + col·sC
//   4 C4    the 4-channel stem filter (conv_x3.hip MODE 2): row k = ⌈R·S / 8⌉·32 indices, index
//           tap·4 + c of W[k][c][tap / S][tap % S] (0 for c ≥ C or tap ≥ R·S)
// Reference: the per-layer weight layouts of DL/nn/SpatialConvolution.scala:435-505 (col2im backward)
// and DL/nn/Linear.scala:108-158.
#include "common.h"

constexpr int WX_MAXC = 4;
constexpr int WX_MAXT = 8;

struct WxClass {
  int ro, so;
  int rmap[WX_MAXT], smap[WX_MAXT];
  long long out_off;
};

struct WxJob {
  const float* in;
  bf16_t* out;
  int kind, K, C, R, S;
  long long sK, sC, sR, sS;
  int ncls, tiles, taps;
  long long first_block, nblocks;
  WxClass cls[WX_MAXC];
};

__device__ __forceinline__ void split_store8(bf16_t* __restrict__ hi_dst, bf16_t* __restrict__ lo_dst, const float (&v)[8]) {
  uint32_t hw[4], lw[4];
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    const bf16_t h0 = f2bf(v[2 * e]), h1 = f2bf(v[2 * e + 1]);
    const bf16_t l0 = f2bf(v[2 * e] - bf2f(h0)), l1 = f2bf(v[2 * e + 1] - bf2f(h1));
    hw[e] = (uint32_t)h0 | ((uint32_t)h1 << 16);
    lw[e] = (uint32_t)l0 | ((uint32_t)l1 << 16);
  }
  *reinterpret_cast<uint4*>(hi_dst) = make_uint4(hw[0], hw[1], hw[2], hw[3]);
  if (lo_dst) *reinterpret_cast<uint4*>(lo_dst) = make_uint4(lw[0], lw[1], lw[2], lw[3]);
}

// the chunk-split address of logical element L (L % 8 == 0 → 8 consecutive elements share a chunk)
__device__ __forceinline__ bf16_t* chunk_hi(bf16_t* out, long long L) { return out + (L >> 5) * 64 + (L & 31); }

__device__ void wx_body(const WxJob& jb, long long local) {
  const int tid = threadIdx.x;
  if (jb.kind == 0 || jb.kind == 2 || jb.kind == 4) {
    // 8 consecutive output elements per thread
    const long long L = (local * 256 + tid) * 8;
    const int R2 = (jb.R + 1) >> 1, S2 = (jb.S + 1) >> 1;
    const int KW4 = (jb.R * jb.S + 7) / 8 * 32;  // C4 row length
    const long long n = jb.kind == 0   ? (long long)jb.K * jb.R * jb.S * jb.C
                        : jb.kind == 2 ? (long long)jb.K * R2 * S2 * 32
                                       : (long long)jb.K * KW4;
    if (L >= n) return;
    float v[8];
    if (jb.kind == 4) {
      const int k = (int)(L / KW4), i0 = (int)(L - (long long)k * KW4);
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const int idx = i0 + e, tap = idx >> 2, c = idx & 3, r = tap / jb.S, s = tap - (tap / jb.S) * jb.S;
        v[e] = (c < jb.C && tap < jb.R * jb.S) ? jb.in[k * jb.sK + r * jb.sR + s * jb.sS + c * jb.sC] : 0.f;
      }
    } else if (jb.kind == 0) {
      long long q = L;
      int c = (int)(q % jb.C);
      q /= jb.C;
      int s = (int)(q % jb.S);
      q /= jb.S;
      int r = (int)(q % jb.R);
      int k = (int)(q / jb.R);
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        v[e] = jb.in[k * jb.sK + r * jb.sR + s * jb.sS + c * jb.sC];
        if (++c == jb.C) {
          c = 0;
          if (++s == jb.S) {
            s = 0;
            if (++r == jb.R) { r = 0; ++k; }
          }
        }
      }
    } else {
      const int ch0 = (int)(L & 31);
      const long long kab = L >> 5;
      const int b = (int)(kab % S2), a = (int)((kab / S2) % R2), k = (int)(kab / ((long long)S2 * R2));
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const int ch = ch0 + e, c = ch >> 2, r = 2 * a + ((ch >> 1) & 1), s = 2 * b + (ch & 1);
        v[e] = (c < jb.C && r < jb.R && s < jb.S) ? jb.in[k * jb.sK + r * jb.sR + s * jb.sS + c * jb.sC] : 0.f;
      }
    }
    bf16_t* h = chunk_hi(jb.out, L);
    split_store8(h, h + 32, v);
    return;
  }
  if (jb.kind == 3) {
    // rows × (3·cp): thread = 8 consecutive columns of one part
    const int rows = jb.R, cp = jb.S;
    const long long L = (local * 256 + tid) * 8;
    if (L >= (long long)rows * 3 * cp) return;
    const int row = (int)(L / (3 * cp));
    const int j = (int)(L - (long long)row * 3 * cp), part = j / cp, col0 = j - part * cp;
    float v[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const int col = col0 + e;
      v[e] = (row < jb.K && col < jb.C) ? jb.in[row * jb.sK + col * jb.sC] : 0.f;
    }
    if (part == 1) {  // the lo part: write lo through the hi slot
      float lo[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) lo[e] = v[e] - bf2f(f2bf(v[e]));
      split_store8(jb.out + L, nullptr, lo);
    } else {
      split_store8(jb.out + L, nullptr, v);
    }
    return;
  }
  // kind 1: a 64(k) × 64(c) tile of one tap of one class through LDS
  __shared__ float t[64][65];
  const int q = (int)(local / ((long long)jb.tiles * jb.taps));
  local -= (long long)q * jb.tiles * jb.taps;
  const int tap = (int)(local / jb.tiles);
  const int tile = (int)(local - (long long)tap * jb.tiles);
  if (q >= jb.ncls) return;  // block-uniform
  const WxClass& cl = jb.cls[q];
  if (tap >= cl.ro * cl.so) return;
  const int i = tap / cl.so, j = tap - (tap / cl.so) * cl.so;
  const int r = cl.rmap[i], s = cl.smap[j];
  const int tiles_c = (jb.C + 63) / 64;
  const int c0 = (tile % tiles_c) * 64, k0 = (tile / tiles_c) * 64;
  // reads: 64 k-rows × 64 c (c fastest: coalesced for KRSC masters)
#pragma unroll
  for (int it = 0; it < 16; ++it) {
    const int idx = tid + 256 * it, kl = idx >> 6, cl_ = idx & 63;
    const int k = k0 + kl, c = c0 + cl_;
    t[kl][cl_] = (k < jb.K && c < jb.C) ? jb.in[k * jb.sK + c * jb.sC + r * jb.sR + s * jb.sS] : 0.f;
  }
  __syncthreads();
  // writes: 64 c-rows × 8 groups of 8 k (K % 32 == 0: a group never straddles a chunk)
#pragma unroll
  for (int it = 0; it < 2; ++it) {
    const int idx = tid + 256 * it, cr = idx >> 3, kg = idx & 7;
    const int c = c0 + cr, k = k0 + kg * 8;
    if (c >= jb.C || k >= jb.K) continue;
    float v[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] = t[kg * 8 + e][cr];
    const long long L = (((long long)c * cl.ro + i) * cl.so + j) * jb.K + k;
    bf16_t* h = chunk_hi(jb.out + cl.out_off, L);
    split_store8(h, h + 32, v);
  }
}

__global__ void __launch_bounds__(256) k_wx3_multi(const WxJob* __restrict__ jobs, int njobs) {
  const long long b = blockIdx.x;
  int lo = 0, hi = njobs - 1;  // last job with first_block <= b
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (jobs[mid].first_block <= b) lo = mid;
    else hi = mid - 1;
  }
  wx_body(jobs[lo], b - jobs[lo].first_block);
}

__global__ void __launch_bounds__(256) k_wx3_one(WxJob jb) { wx_body(jb, blockIdx.x); }

BIGDL_EXPORT int bigdl_wx3_job_size() { return (int)sizeof(WxJob); }

// Validate and fill one job record at ``rec``; *nblocks receives its block count.  Out-of-range
// geometry is refused here, on the host, so no launch can index outside the buffers the caller sized
// (FWD / DGRAD / S2D: the chunk-split element counts of ops/fp32x3.py; ROWS3: rows·3·cp).
BIGDL_EXPORT int bigdl_wx3_job(void* rec, const float* in, void* out, int kind, int K, int C, int R, int S,
                               long long sK, long long sC, long long sR, long long sS, int ncls, const int* ros,
                               const int* sos, const int* rmaps, const int* smaps, const long long* out_offs,
                               long long first_block, long long* nblocks) {
  if (!in || !out || K <= 0 || C <= 0 || R <= 0 || S <= 0 || ((uintptr_t)out & 15) || kind < 0 || kind > 4)
    return (int)hipErrorInvalidValue;
  WxJob jb{};
  jb.in = in;
  jb.out = (bf16_t*)out;
  jb.kind = kind;
  jb.K = K; jb.C = C; jb.R = R; jb.S = S;
  jb.sK = sK; jb.sC = sC; jb.sR = sR; jb.sS = sS;
  jb.first_block = first_block;
  long long nb = 0;
  if (kind == 0) {
    const long long n = (long long)K * R * S * C;
    if (((long long)R * S * C) % 32) return (int)hipErrorInvalidValue;
    nb = (n + 2047) / 2048;
  } else if (kind == 2) {
    if (4 * C > 32) return (int)hipErrorInvalidValue;
    const long long n = (long long)K * ((R + 1) / 2) * ((S + 1) / 2) * 32;
    nb = (n + 2047) / 2048;
  } else if (kind == 4) {
    if (C > 4 || R * S > 64) return (int)hipErrorInvalidValue;
    const long long n = (long long)K * ((R * S + 7) / 8) * 32;
    nb = (n + 2047) / 2048;
  } else if (kind == 3) {
    // R = padded rows (≥ K), S = part width cp (% 8, ≥ C)
    if (R < K || S % 8 || S < C) return (int)hipErrorInvalidValue;
    nb = ((long long)R * 3 * S + 2047) / 2048;
  } else {
    if (ncls < 1 || ncls > WX_MAXC || K % 32) return (int)hipErrorInvalidValue;
    jb.ncls = ncls;
    int taps = 0;
    for (int q = 0; q < ncls; ++q) {
      WxClass& c = jb.cls[q];
      c.ro = ros[q];
      c.so = sos[q];
      if (c.ro < 1 || c.so < 1 || c.ro > WX_MAXT || c.so > WX_MAXT) return (int)hipErrorInvalidValue;
      for (int i = 0; i < WX_MAXT; ++i) {
        c.rmap[i] = i < c.ro ? rmaps[q * WX_MAXT + i] : 0;
        c.smap[i] = i < c.so ? smaps[q * WX_MAXT + i] : 0;
        if (i < c.ro && (c.rmap[i] < 0 || c.rmap[i] >= R)) return (int)hipErrorInvalidValue;
        if (i < c.so && (c.smap[i] < 0 || c.smap[i] >= S)) return (int)hipErrorInvalidValue;
      }
      c.out_off = out_offs[q];
      if (c.out_off % 64) return (int)hipErrorInvalidValue;
      if (c.ro * c.so > taps) taps = c.ro * c.so;
    }
    jb.tiles = ((C + 63) / 64) * ((K + 63) / 64);
    jb.taps = taps;
    nb = (long long)jb.tiles * taps * ncls;
  }
  jb.nblocks = nb;
  *nblocks = nb;
  *reinterpret_cast<WxJob*>(rec) = jb;
  return 0;
}

BIGDL_EXPORT int bigdl_wx3_multi(const void* jobs_dev, int njobs, long long total_blocks, hipStream_t s) {
  if (njobs <= 0 || total_blocks <= 0 || total_blocks > 0x7fffffffLL || ((uintptr_t)jobs_dev & 15))
    return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(k_wx3_multi, dim3((unsigned)total_blocks), dim3(256), 0, s, (const WxJob*)jobs_dev, njobs);
  BIGDL_CHECK_LAUNCH();
}

// one job, passed by value (no device table): HIP-graph capture and weights outside an arena
BIGDL_EXPORT int bigdl_wx3_one(const void* rec, hipStream_t s) {
  const WxJob& jb = *reinterpret_cast<const WxJob*>(rec);
  if (jb.nblocks <= 0 || jb.nblocks > 0x7fffffffLL) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(k_wx3_one, dim3((unsigned)jb.nblocks), dim3(256), 0, s, jb);
  BIGDL_CHECK_LAUNCH();
}

// ------------------------------------------------------------------------------------------------
// The s2d stem's weight gradient folded back onto the R×S×C taps: gw[k][c][r][s] += scale ·
// g2[k][a][b][c·4 + bh·2 + bw] (r = 2a + bh, s = 2b + bw), and every g2 entry cleared after it is read
// (g2 is a persistent accumulation buffer of the split-K wgrad; one thread per g2 element).
// ------------------------------------------------------------------------------------------------
__global__ void __launch_bounds__(256) k_s2d_wgrad_fold(float* __restrict__ g2, float* __restrict__ gw, int K, int C,
                                                        int R, int S, long long sK, long long sC, long long sR,
                                                        long long sS, float scale) {
  const int R2 = (R + 1) >> 1, S2 = (S + 1) >> 1;
  const long long n = (long long)K * R2 * S2 * 32;
  for (long long e = blockIdx.x * 256LL + threadIdx.x; e < n; e += (long long)gridDim.x * 256) {
    const int ch = (int)(e & 31);
    const long long kab = e >> 5;
    const int b = (int)(kab % S2), a = (int)((kab / S2) % R2), k = (int)(kab / ((long long)S2 * R2));
    const int c = ch >> 2, r = 2 * a + ((ch >> 1) & 1), s = 2 * b + (ch & 1);
    const float v = g2[e];
    if (c < C && r < R && s < S) gw[k * sK + c * sC + r * sR + s * sS] += scale * v;
    g2[e] = 0.f;
  }
}

BIGDL_EXPORT int bigdl_s2d_wgrad_fold(float* g2, float* gw, int K, int C, int R, int S, long long sK, long long sC,
                                      long long sR, long long sS, float scale, hipStream_t s) {
  if (!g2 || !gw || K <= 0 || C <= 0 || 4 * C > 32 || R <= 0 || S <= 0) return (int)hipErrorInvalidValue;
  const long long n = (long long)K * ((R + 1) / 2) * ((S + 1) / 2) * 32;
  hipLaunchKernelGGL(k_s2d_wgrad_fold, dim3(bigdl_grid(n, 256)), dim3(256), 0, s, g2, gw, K, C, R, S, sK, sC, sR, sS,
                     scale);
  BIGDL_CHECK_LAUNCH();
}

// The C4 stem's weight gradient onto the KCRS-strided master gradient: gw[k][c][r][s] += scale ·
// g4[k][r][s][c] (c < C), every g4 entry cleared after it is read (a persistent split-K buffer).
__global__ void __launch_bounds__(256) k_c4_wgrad_fold(float* __restrict__ g4, float* __restrict__ gw, int K, int C,
                                                       int R, int S, long long sK, long long sC, long long sR,
                                                       long long sS, float scale) {
  const long long n = (long long)K * R * S * 4;
  for (long long e = blockIdx.x * 256LL + threadIdx.x; e < n; e += (long long)gridDim.x * 256) {
    const int c = (int)(e & 3);
    const long long kt = e >> 2;
    const int tap = (int)(kt % (R * S)), k = (int)(kt / (R * S));
    const int r = tap / S, s = tap - (tap / S) * S;
    const float v = g4[e];
    if (c < C) gw[k * sK + c * sC + r * sR + s * sS] += scale * v;
    g4[e] = 0.f;
  }
}

BIGDL_EXPORT int bigdl_c4_wgrad_fold(float* g4, float* gw, int K, int C, int R, int S, long long sK, long long sC,
                                     long long sR, long long sS, float scale, hipStream_t s) {
  if (!g4 || !gw || K <= 0 || C <= 0 || C > 4 || R <= 0 || S <= 0) return (int)hipErrorInvalidValue;
  const long long n = (long long)K * R * S * 4;
  hipLaunchKernelGGL(k_c4_wgrad_fold, dim3(bigdl_grid(n, 256)), dim3(256), 0, s, g4, gw, K, C, R, S, sK, sC, sR, sS,
                     scale);
  BIGDL_CHECK_LAUNCH();
}
