// Shared definitions of the implicit-GEMM convolution kernels (conv_igemm.hip: 4-wave 16x16x32
// family; conv_mfma32.hip: 8-wave 32x32x16 / LDS-DMA family).
#pragma once
#include "common.h"

typedef short v8s __attribute__((ext_vector_type(8)));
typedef float v4f __attribute__((ext_vector_type(4)));

struct ConvParams {
  const bf16_t* x;     // [Nb][H][W][C]
  const bf16_t* w;     // [K][R][S][C]
  const float* bias;   // [K] or null
  bf16_t* y;           // [Nb][P][Q][K]
  int Nb, H, W, C, K, R, S, P, Q;
  int sh, sw, ph, pw, dh, dw;
  int M;               // Nb*P*Q
  int Kg;              // R*S*C
  int relu;
  int tiles_n;
  const bf16_t* res;   // optional [M][K] tensor added before the ReLU (residual / gradient sum)
  float* stats;        // optional BN partials: stats[tm][K] = Σ y, stats[G + tm][K] = Σ y² (G = #row tiles)
  int tiles_m;
  // optional output scatter (sub-pixel strided dgrad): output pixel (n, p, q) is stored at pixel
  // (n, p·osh + ooh, q·osw + oow) of a [Nb][oH][oW][K] tensor
  int scatter, osh, osw, ooh, oow, oH, oW;
  // optional fused BatchNorm-backward prologue for the BN (+ReLU) that produced this dgrad's
  // input gradient target: g ← g · [bnx·sc + sh > 0] (the ReLU mask recomputed from the BN input
  // and its forward coefficients), and per-row-tile partials Σg, Σg·(bnx − mean) into `stats`
  const bf16_t* bnx;
  const float* bn_sc;
  const float* bn_sh;
  const float* bn_mean;
  // optional explicit mask source for that mode (ResNet block tail: the block output, whose ReLU
  // saw BN(bnx) + shortcut): g ← (g + res) · [bn_mask > 0] instead of the recomputed mask
  const bf16_t* bn_mask;
  // the same mask as bits (one byte per 8-channel chunk, written by the tail BN's apply kernel):
  // read instead of bn_mask when set
  const uint8_t* bn_bits;
  // output row stride in elements (== K unless the conv writes a channel slice of a wider tensor,
  // e.g. its branch of an Inception concat: y points at the slice, rows are ldy apart)
  int ldy;
  // weight row stride in elements (== Kg, or Kg rounded up to 8 for the C = 4 stem, whose rows are
  // zero-padded so every weight chunk stays 16-B aligned)
  int ldw;
  // optional per-channel shift K of the BN statistics partials: Σ(y − K), Σ(y − K)² instead of the
  // raw sums, so E[y²] − E[y]² never cancels catastrophically (the BN passes its running mean —
  // any value is exact, one near the batch mean keeps the variance well conditioned)
  const float* stat_shift;
  // optional strided residual (res_sh > 0): `res` is a [Nb][res_H][res_W][K] tensor holding only
  // the output pixels (h, w) with h % res_sh == 0 and w % res_sw == 0 (the input gradient of a 1×1
  // stride-s shortcut conv); every other pixel's residual is zero — the dense zero-filled copy is
  // never materialised
  int res_sh, res_sw, res_H, res_W;
  // 3-D convolution (VolumetricConvolution, D3 instantiations only): input depth T, filter depth
  // KT, depth stride / pad / dilation, output depth To; x is [Nb][T][H][W][C], w [K][KT][R][S][C],
  // y [Nb][To][P][Q][K] (M = Nb·To·P·Q).  2-D launches leave T = KT = To = 1.
  int T, KT, st, pt, dtd, To;
  // Pixel stride of x in elements (C unless x is a channel slice of a wider NHWC tensor) and, for
  // grouped convolution (SpatialConvolution.scala nGroup; one launch, group = blockIdx.y), the
  // per-group element offsets of x (channels), w (filters·ldw) and y / bias (channels).
  int ldx;
  // bf16x3 two-part input (0 = off): logical channels [cdup, 2·cdup) re-read physical [0, cdup) — the
  // activation split is stored [hi | lo] (ldx = C − cdup) and read as [hi | hi | lo]
  int cdup;
  long long gx, gw, gy;
  // BatchNorm-backward prologue (AT instantiations, pointwise mode): the A operand x is the
  // gradient g' at a BN's output and ``ax`` that BN's input (same layout); the kernel reads
  // A·g' + B·ax + Cc per channel (acoef = [3][C] fp32) — the BN's input gradient — instead of a
  // materialised tensor (one fewer write + read of it per consumer).
  const bf16_t* ax;
  const float* acoef;
  // optional fp32 output [M][ldy] (the bf16x3 fp32 path, precision.hip): the accumulators (+ bias,
  // ReLU) are stored straight from registers as float4 per lane — no bf16 rounding, no LDS staging;
  // `y` is unused.  Plain epilogue only (no residual / statistics / BN prologue / scatter / groups).
  float* y32;
  // optional fp32 residual [M][ldy] added to the fp32 output before the ReLU (y32 mode only: the
  // data gradient of a block's first conv summed with the shortcut's, bf16x3 path)
  const float* res32;
  // fp32 BN-backward statistics in the y32 epilogue: the BN input [M][K] (with bn_mean, and the ReLU mask
  // from bn_bits or recomputed as bn_sc·x + bn_sh > 0); sums added into replicas (stats_atomic)
  const float* bnx32;
  // statistics mode: 0 = per-row-tile partial rows stats[2][tiles_m][K] (reduced later by a
  // fold / finalize pass), 1 = every tile ADDS its partial sums into stats[2][K] with fp32 atomics
  // (the consumer's apply kernel finalises in its prologue and re-zeroes the buffer: no separate
  // reduction launches; not bit-reproducible — bigdl.deterministic keeps mode 0)
  int stats_atomic;
  // optional int8 output (the calibrated int8 chain's bf16 RGB stem, nn/quantized): the epilogue
  // writes q = clamp(rint(ReLU?(y) · yq_inv)) as int8 [M][ldy] instead of bf16 — signed [-127, 127],
  // or (yq_u8) unsigned [0, 255] stored offset by -128 with the 16-byte 0x80 tail after the tensor
  // (conv_i8.hip's unsigned activation contract).  Plain epilogue only (no residual / statistics).
  int8_t* yq;
  float yq_inv;
  int yq_u8;
};

// one tile's per-channel partial sum `v` of statistic `which` (0: Σ, 1: Σ²) for channel n, row group g
// stats_atomic = R ≥ 1: the partial is ADDED into replica g % R of a zeroed [2][R][K] buffer (R = 1:
// the [2][K] sums): R replicas cut the same-address atomic contention R-fold while keeping the BN's
// finalize input at R ≤ 512 rows (no fold pass)
__device__ __forceinline__ void put_stat(const ConvParams& p, int which, int g, int n, float v) {
  if (p.stats_atomic)
    atomicAdd(&p.stats[((size_t)which * p.stats_atomic + (g % p.stats_atomic)) * p.K + n], v);
  else
    p.stats[((size_t)which * p.tiles_m + g) * p.K + n] = v;
}

// Residual offset of output pixel m, channel n (dense: the output offset itself); false = the
// residual is zero at this pixel (strided residual, off-grid pixel).
__device__ __forceinline__ bool res_at(const ConvParams& p, int m, int n, size_t dense_off, size_t& roff) {
  if (p.res_sh == 0) {
    roff = dense_off;
    return true;
  }
  const int img = m / (p.P * p.Q);
  const int pq = m - img * p.P * p.Q;
  const int h = pq / p.Q, w = pq - h * p.Q;
  if (h % p.res_sh || w % p.res_sw) return false;
  roff = ((size_t)(img * p.res_H + h / p.res_sh) * p.res_W + w / p.res_sw) * p.K + n;
  return true;
}

constexpr int SBM = 128;  // row granularity of the BN-statistics partials (any BM writes BM / SBM rows)

__device__ __forceinline__ int xcd_remap(int bid, int nwg) {
  const int xcd = bid & 7, q = nwg >> 3, r = nwg & 7;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (bid >> 3);
}


// Second half of the conv epilogue, shared by both kernel families: the block's output tile is staged
// as bf16 in LDS (`et`, [BM][BN] with the chunk ^ (row & CMASK) swizzle) and the block walks it
// row-major, 8 channels per thread: optional residual add, ReLU, BN-backward mask, scatter, one
// 16-B global store per chunk, and per-channel Σ / Σ² partials for a following BatchNormalization.
// ``rstats``: the statistics were already reduced from the fp32 accumulators into `red8`.
// ``skp`` (optional): this thread's 8 statistics-shift values, fetched by the caller ahead of time
// (channels n0 + (tid % (BN / 8))·8 …+7) instead of a dependent load here.
template <int BM, int BN, int NT>
__device__ __forceinline__ void conv_store_pass(const ConvParams& p, bf16_t* et, int tid, int m0, int n0, int tm,
                                                bool rstats, const float* skp = nullptr) {
  constexpr int LDR = BN;
  constexpr int CMASK = (BN / 8 - 1) & 15;
  constexpr int SRED = 8;
  float* red8 = reinterpret_cast<float*>(&et[BM * LDR]);
  auto rd_chunk = [&](int r, int c) -> uint4 {
    return *reinterpret_cast<const uint4*>(&et[r * LDR + ((c ^ (r & CMASK)) << 3)]);
  };
  constexpr int CPR = BN / 8;      // 16-B chunks per tile row
  constexpr int RPP = NT / CPR;   // rows per pass
  const int cc = tid % CPR, rr = tid / CPR;
  const int n = n0 + cc * 8;
  if (p.yq) {  // int8 output (K % 8 == 0 checked by the launcher)
    const float qlo = p.yq_u8 ? 0.f : -127.f, qhi = p.yq_u8 ? 255.f : 127.f, qoff = p.yq_u8 ? 128.f : 0.f;
    const int rmax = p.M - m0;
    if (n < p.K) {
#pragma unroll 4
      for (int r = rr; r < BM; r += RPP) {
        if (r >= rmax) break;
        float v[8];
        unpack8(rd_chunk(r, cc), v);
        uint32_t w2[2] = {0u, 0u};
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const float t = p.relu ? fmaxf(v[e], 0.f) : v[e];
          const float q = fminf(fmaxf(rintf(t * p.yq_inv), qlo), qhi) - qoff;
          w2[e >> 2] |= ((uint32_t)(int)q & 0xFFu) << (8 * (e & 3));
        }
        *reinterpret_cast<uint2*>(p.yq + (size_t)(m0 + r) * p.ldy + n) = make_uint2(w2[0], w2[1]);
      }
    }
    if (p.yq_u8 && m0 == 0 && n0 == 0 && tid == 0)
      *reinterpret_cast<uint4*>(p.yq + (size_t)p.M * p.ldy) = make_uint4(0x80808080u, 0x80808080u, 0x80808080u,
                                                                         0x80808080u);
    return;
  }
  // plain store (no residual / ReLU / BN prologue / scatter, whole channel tile): one LDS read and
  // one 16-B global store per chunk on an incrementally advanced row pointer
  if (!p.res && !p.relu && !p.bnx && !p.scatter && (p.stats == nullptr || rstats) && n0 + BN <= p.K) {
    bf16_t* yp = p.y + (size_t)(m0 + rr) * p.ldy + n;
    const size_t step = (size_t)RPP * p.ldy;
    const int rmax = p.M - m0;
#pragma unroll 4
    for (int r = rr; r < BM; r += RPP, yp += step)
      if (r < rmax) *reinterpret_cast<uint4*>(yp) = rd_chunk(r, cc);
    if (rstats && tid < 2 * BN) {
      const int which = tid / BN, c = tid - which * BN;
      float a = 0.f;
#pragma unroll
      for (int g = 0; g < SRED; ++g) a += red8[(which * SRED + g) * BN + c];
      if (tm < p.tiles_m) put_stat(p, which, tm, n0 + c, a);
    }
    return;
  }
  // residual (+ ReLU) epilogue of a whole channel tile (the inference conv+sum+ReLU, FusedConvSum):
  // all of this thread's residual chunks are requested before the first is used — one chunk in
  // flight per row (the general loop below) left the 56² block tails at ~3.9 TB/s
  if (p.res && p.res_sh == 0 && !p.bnx && !p.scatter && !p.stats && n0 + BN <= p.K) {
    constexpr int NR = BM / RPP;
    const int rmax = p.M - m0;
    uint4 rv[NR];
#pragma unroll
    for (int i = 0; i < NR; ++i) {
      const int r = rr + i * RPP;
      rv[i] = r < rmax ? *reinterpret_cast<const uint4*>(p.res + (size_t)(m0 + r) * p.K + n) : make_uint4(0, 0, 0, 0);
    }
#pragma unroll
    for (int i = 0; i < NR; ++i) {
      const int r = rr + i * RPP;
      if (r >= rmax) break;
      float v[8], a[8];
      unpack8(rd_chunk(r, cc), v);
      unpack8(rv[i], a);
      uint32_t w4[4];
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        v[e] += a[e];
        if (p.relu) v[e] = fmaxf(v[e], 0.f);
      }
#pragma unroll
      for (int e = 0; e < 4; ++e) w4[e] = (uint32_t)f2bf(v[2 * e]) | ((uint32_t)f2bf(v[2 * e + 1]) << 16);
      *reinterpret_cast<uint4*>(p.y + (size_t)(m0 + r) * p.ldy + n) = make_uint4(w4[0], w4[1], w4[2], w4[3]);
    }
    return;
  }
  float s8[8], q8[8];
  const bool full = n + 8 <= p.K;
  float sk[8];  // statistics shift of this thread's 8 channels
#pragma unroll
  for (int e = 0; e < 8; ++e)
    sk[e] = skp ? skp[e] : (p.stat_shift && p.stats && !p.bnx && n + e < p.K) ? p.stat_shift[n + e] : 0.f;
  float bsc[8], bsh[8], bmu[8];
  if (p.bnx && full) {
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      bsc[e] = p.bn_mask ? 0.f : p.bn_sc[n + e];
      bsh[e] = p.bn_mask ? 0.f : p.bn_sh[n + e];
      bmu[e] = p.bn_mean[n + e];
    }
  }
  // BN-backward dgrad epilogue (bnx, dense output): every global operand of this thread's rows —
  // the BN input chunk, the ReLU mask (bits or bf16) and the residual chunk — is requested before
  // the first is used (the row-at-a-time loop below kept one or two rows in flight: the 56² stage-1
  // dgrads, ~1.3 GB each, ran at ~3 TB/s)
  constexpr int NRH = SBM / RPP;
  const bool bnfast = p.bnx && full && !p.scatter && (!p.bn_mask || p.bn_bits);
  // the statistics partials are per SBM-row group: a BM = 256 tile reduces its two halves separately
  for (int h = 0; h < BM / SBM; ++h) {
#pragma unroll
  for (int e = 0; e < 8; ++e) { s8[e] = 0.f; q8[e] = 0.f; }
  if (bnfast) {
    uint4 xq[NRH], rq[NRH];
    uint32_t bq[NRH];
#pragma unroll
    for (int i = 0; i < NRH; ++i) {
      const int r = h * SBM + rr + i * RPP, m = m0 + r;
      const bool live = m < p.M;
      const size_t off = (size_t)(live ? m : m0) * p.K + n;
      xq[i] = live ? *reinterpret_cast<const uint4*>(p.bnx + off) : make_uint4(0, 0, 0, 0);
      bq[i] = (live && p.bn_mask) ? (uint32_t)p.bn_bits[off >> 3] : 0xFFu;
      size_t ro;
      rq[i] = (live && p.bn_mask && p.res && res_at(p, m, n, off, ro)) ? *reinterpret_cast<const uint4*>(p.res + ro)
                                                         : make_uint4(0, 0, 0, 0);
    }
#pragma unroll
    for (int i = 0; i < NRH; ++i) {
      const int r = h * SBM + rr + i * RPP, m = m0 + r;
      if (m >= p.M) break;
      float g[8], xv[8], rv[8];
      unpack8(rd_chunk(r, cc), g);
      unpack8(xq[i], xv);
      unpack8(rq[i], rv);
      uint32_t w4[4];
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const bool live = p.bn_mask ? ((bq[i] >> e) & 1u) != 0 : fmaf(xv[e], bsc[e], bsh[e]) > 0.f;
        g[e] = live ? g[e] + (p.bn_mask ? rv[e] : 0.f) : 0.f;
      }
#pragma unroll
      for (int e = 0; e < 4; ++e) w4[e] = (uint32_t)f2bf(g[2 * e]) | ((uint32_t)f2bf(g[2 * e + 1]) << 16);
      *reinterpret_cast<uint4*>(p.y + (size_t)m * p.ldy + n) = make_uint4(w4[0], w4[1], w4[2], w4[3]);
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float a = __uint_as_float(w4[e] << 16), b = __uint_as_float(w4[e] & 0xFFFF0000u);
        s8[2 * e] += a;
        q8[2 * e] = fmaf(a, xv[2 * e] - bmu[2 * e], q8[2 * e]);
        s8[2 * e + 1] += b;
        q8[2 * e + 1] = fmaf(b, xv[2 * e + 1] - bmu[2 * e + 1], q8[2 * e + 1]);
      }
    }
  } else
#pragma unroll 2
  for (int r = h * SBM + rr; r < (h + 1) * SBM; r += RPP) {
    const int m = m0 + r;
    if (m >= p.M || n >= p.K) continue;
    size_t off = (size_t)m * p.K + n;
    size_t yoff = (size_t)m * p.ldy + n;
    if (p.scatter) {
      const int nimg = m / (p.P * p.Q);
      const int pq = m - nimg * p.P * p.Q;
      const int pp = pq / p.Q, qq = pq - pp * p.Q;
      off = ((size_t)(nimg * p.oH + pp * p.osh + p.ooh) * p.oW + qq * p.osw + p.oow) * p.K + n;
      yoff = off;
    }
    if (full && p.bnx) {
      float g[8], xv[8];
      unpack8(rd_chunk(r, cc), g);
      load8(p.bnx + off, xv);
      uint32_t w4[4];
      if (p.bn_mask) {
        float rv[8], mv[8];
        if (p.bn_bits) {
          const uint32_t b = p.bn_bits[off >> 3];
#pragma unroll
          for (int e = 0; e < 8; ++e) mv[e] = (b >> e) & 1u ? 1.f : 0.f;
        } else {
          load8(p.bn_mask + off, mv);
        }
        size_t ro;
        if (p.res && res_at(p, m, n, off, ro)) {
          load8(p.res + ro, rv);
#pragma unroll
          for (int e = 0; e < 8; ++e) g[e] += rv[e];
        }
#pragma unroll
        for (int e = 0; e < 8; ++e) g[e] = mv[e] > 0.f ? g[e] : 0.f;
      } else {
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const bool live = fmaf(xv[e], bsc[e], bsh[e]) > 0.f;
          g[e] = live ? g[e] : 0.f;
        }
      }
#pragma unroll
      for (int e = 0; e < 4; ++e) w4[e] = (uint32_t)f2bf(g[2 * e]) | ((uint32_t)f2bf(g[2 * e + 1]) << 16);
      *reinterpret_cast<uint4*>(p.y + yoff) = make_uint4(w4[0], w4[1], w4[2], w4[3]);
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float a = __uint_as_float(w4[e] << 16), b = __uint_as_float(w4[e] & 0xFFFF0000u);
        s8[2 * e] += a;
        q8[2 * e] = fmaf(a, xv[2 * e] - bmu[2 * e], q8[2 * e]);
        s8[2 * e + 1] += b;
        q8[2 * e + 1] = fmaf(b, xv[2 * e + 1] - bmu[2 * e + 1], q8[2 * e + 1]);
      }
    } else if (full) {
      uint4 u = rd_chunk(r, cc);
      if (p.res || p.relu) {
        float v[8];
        unpack8(u, v);
        size_t ro;
        if (p.res && res_at(p, m, n, off, ro)) {
          float rv[8];
          load8(p.res + ro, rv);
#pragma unroll
          for (int e = 0; e < 8; ++e) v[e] += rv[e];
        }
        if (p.relu) {
#pragma unroll
          for (int e = 0; e < 8; ++e) v[e] = fmaxf(v[e], 0.f);
        }
        uint32_t w4[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) w4[e] = (uint32_t)f2bf(v[2 * e]) | ((uint32_t)f2bf(v[2 * e + 1]) << 16);
        u = make_uint4(w4[0], w4[1], w4[2], w4[3]);
      }
      *reinterpret_cast<uint4*>(p.y + yoff) = u;
      if (p.stats && !rstats) {
        // statistics of the values as stored (bf16-rounded), which is what the BN reads
        const uint32_t uw[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const float a = __uint_as_float(uw[e] << 16) - sk[2 * e];
          const float b = __uint_as_float(uw[e] & 0xFFFF0000u) - sk[2 * e + 1];
          s8[2 * e] += a;
          q8[2 * e] = fmaf(a, a, q8[2 * e]);
          s8[2 * e + 1] += b;
          q8[2 * e + 1] = fmaf(b, b, q8[2 * e + 1]);
        }
      }
    } else {
      float v[8];
      unpack8(rd_chunk(r, cc), v);
      size_t ro = 0;
      const bool rlive = p.res && res_at(p, m, n, off, ro);
      for (int e = 0; e < 8 && n + e < p.K; ++e) {
        float t = v[e] + (rlive ? bf2f(p.res[ro + e]) : 0.f);
        if (p.relu) t = fmaxf(t, 0.f);
        const bf16_t o = f2bf(t);
        p.y[yoff + e] = o;
        const float w = bf2f(o) - sk[e];
        s8[e] += w;
        q8[e] = fmaf(w, w, q8[e]);
      }
    }
  }
  if (rstats) {
    // the staging barrier above also ordered the partial writes: fold the SRED partials
    if (tid < 2 * BN) {
      const int which = tid / BN, c = tid - which * BN;
      float a = 0.f;
#pragma unroll
      for (int g = 0; g < SRED; ++g) a += red8[(which * SRED + g) * BN + c];
      if (n0 + c < p.K && tm < p.tiles_m) put_stat(p, which, tm, n0 + c, a);
    }
  } else if (p.stats) {
    // reduce the RPP row groups of each channel chunk through LDS (after the tile reads retire)
    float* red = reinterpret_cast<float*>(&et[BM * LDR]);  // [RPP][BN] Σ, then [RPP][BN] Σ²
    // 16-B stores: lanes (consecutive cc) land 32 B apart — conflict-free, where 8 scalar stores
    // per array at that stride were 8-way bank conflicts (profiles/r1_conv_pmc_v1.txt)
    float4* rs = reinterpret_cast<float4*>(&red[rr * BN + cc * 8]);
    float4* rq = reinterpret_cast<float4*>(&red[RPP * BN + rr * BN + cc * 8]);
    rs[0] = make_float4(s8[0], s8[1], s8[2], s8[3]);
    rs[1] = make_float4(s8[4], s8[5], s8[6], s8[7]);
    rq[0] = make_float4(q8[0], q8[1], q8[2], q8[3]);
    rq[1] = make_float4(q8[4], q8[5], q8[6], q8[7]);
    __syncthreads();
    constexpr int QP = NT >= BN ? NT / BN : 1;  // threads per channel in the fold (RPP / QP = 8 rows each)
    if constexpr (QP == 1) {
      for (int c = tid; c < BN; c += NT) {
        float a = 0.f, b = 0.f;
#pragma unroll 4
        for (int g = 0; g < RPP; ++g) {
          a += red[g * BN + c];
          b += red[RPP * BN + g * BN + c];
        }
        const int g = tm * (BM / SBM) + h;
        if (n0 + c < p.K && g < p.tiles_m) {
          put_stat(p, 0, g, n0 + c, a);
          put_stat(p, 1, g, n0 + c, b);
        }
      }
    } else {
      // every thread folds 8 of a channel's RPP partial rows (16 independent LDS reads in flight
      // instead of BN threads walking all RPP rows one dependent read at a time — ~5k cycles per
      // tile at one workgroup per CU), then BN threads add the QP results
      constexpr int RQ = RPP / QP;
      const int c = tid % BN, qp = tid / BN;
      float a = 0.f, b = 0.f;
#pragma unroll
      for (int g = 0; g < RQ; ++g) {
        a += red[(qp * RQ + g) * BN + c];
        b += red[RPP * BN + (qp * RQ + g) * BN + c];
      }
      float* red2 = reinterpret_cast<float*>(&et[h * SBM * LDR]);  // this half's staged rows are consumed
      red2[qp * BN + c] = a;
      red2[(QP + qp) * BN + c] = b;
      __syncthreads();
      if (tid < BN) {
        float sa = 0.f, sb = 0.f;
#pragma unroll
        for (int q = 0; q < QP; ++q) {
          sa += red2[q * BN + tid];
          sb += red2[(QP + q) * BN + tid];
        }
        const int g = tm * (BM / SBM) + h;
        if (n0 + tid < p.K && g < p.tiles_m) {
          put_stat(p, 0, g, n0 + tid, sa);
          put_stat(p, 1, g, n0 + tid, sb);
        }
      }
    }
    if (h + 1 < BM / SBM) __syncthreads();  // the next half rewrites `red`
  }
  }
}

// 8-wave 32x32x16 / direct-to-LDS implicit-GEMM kernel (conv_mfma32.hip).  ``bm`` / ``bn`` the block
// tile; mode 1 = tap-uniform FAST gather, 3 = pointwise.  Returns hipError_t; hipErrorNotSupported
// when the variant / mode pair is not instantiated.
int conv_x8_launch(const ConvParams& p, int mode, int bm, int bn, dim3 grid, hipStream_t s);
// conv_patch.hip: persistent halo-patch 3×3 s1 p1 64 → 64 conv (hipErrorNotSupported: not that shape)
int conv_patch_launch(ConvParams p, hipStream_t s);
bool conv_patch_ok(const ConvParams& p);
bool conv_x8_ok(int mode, int bm, int bn, const ConvParams& p);
