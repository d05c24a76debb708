// Int8 implicit-GEMM convolution for quantized inference: the MI355X form of BigQuant's
// ConvDataInit (im2col + quantise) + MixPrecisionGEMM (DL/nn/quantized/SpatialConvolution.scala:
// 163-208).  No im2col is materialised: the k-tiles of the implicit GEMM
//   acc[n][m] = Σ_k Wq[n][k] · Xq[m][k],   k = (r, s, c),  m = output pixel, n = output channel
// are gathered from the int8 NHWC activation straight into LDS by LDS-DMA (buffer_load_dwordx4 …
// lds; out-of-range offsets — conv padding, the M tail, taps past R·S — read as zeros), and
// multiplied with v_mfma_i32_32x32x32_i8 (2× the bf16 rate per clock).  The tile machinery is the
// 32x32x16 bf16 family's (conv_mfma32.hip): 128-byte LDS rows — 128 int8 k-elements here —, the
// chunk ^ ((row >> 1) & 7) swizzle applied on the per-lane source address and on the fragment read,
// a 3-deep LDS ring with counted vmcnt and raw s_barrier.  An i8 32x32x32 fragment is 16 bytes per
// lane at the same (row, chunk) positions as a bf16 32x32x16 fragment, so the read addressing is
// shared.
//
// Scales: activations per image (sx[n] = amax_n / 127, dynamic — k_absmax_img + k_quant_img below),
// weights per output channel (sw[k], symmetric); the epilogue dequantises acc·sx[img]·sw[k] + bias,
// applies ReLU and stores bf16 through the shared row-major store pass.
//
// Channel counts: C % 16 == 0 (a k-tile lies inside one tap: the tap is wave-uniform; C % 128 != 0 leaves
// the tap's last k-tile partial, its chunks past C read the pad code against zero weights) or C == 64
// (a k-tile holds two taps: chunks 0–3 tap 2t, chunks 4–7 tap 2t + 1, per-lane source offsets; an
// odd R·S leaves a zero half tile).  Weight rows are [K][ldw] int8, (r, s, c) order, zero-padded to
// ldw = KT·128.
#include "conv_params.h"

typedef int v4i __attribute__((ext_vector_type(4)));
typedef int v16i __attribute__((ext_vector_type(16)));
typedef __attribute__((address_space(3))) void i8_lds_void_t;

#define I8_WAIT(n) asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)" ::"n"(n) : "memory")
#define I8_BARRIER()                   \
  do {                                 \
    asm volatile("" ::: "memory");     \
    __builtin_amdgcn_s_barrier();      \
    asm volatile("" ::: "memory");     \
  } while (0)

__device__ __forceinline__ void i8_glds16(__amdgpu_buffer_rsrc_t r, void* lds, uint32_t voff) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (i8_lds_void_t*)lds, 16, voff, 0, 0, 0);
}

struct ConvI8Params {
  const int8_t* x;    // [Nb][H][W][C]
  const int8_t* w;    // [K][ldw]
  const float* sx;    // [Nb] per-image activation scales, or null: the static scale sxs
  const float* swt;   // [K]
  const float* bias;  // [K] or null
  bf16_t* y;          // [M][ldy] (bf16 output), or null when yq is set
  int Nb, H, W, C, K, R, S, P, Q, sh, sw, ph, pw, dh, dw;
  int M, KT, ldw, ldy, relu, tiles_n;
  float sxs;          // static (calibrated) activation scale
  int8_t* yq;         // int8 output [M][ldy] requantised with 1 / out_scale (the next layer's input)
  float out_inv;
  // unsigned 8-bit activations of a non-negative (post-ReLU) tensor, stored offset by −128 in int8:
  // x = (q + 128)·s with q ∈ [−128, 127] — twice the resolution of the symmetric int8 scale.  The
  // offset's share of the dot product, 128·Σ_(taps, c) w, is a per-channel constant the host folds
  // into the bias, provided a padded tap reads the code of x = 0, −128: such an input carries a
  // 16-byte tail of 0x80 right after its last byte and the loader points padded taps at it.
  // y_u8: write the (ReLU'd) output that way, tail included.
  int x_u8, y_u8;
  // residual summed before the ReLU (conv + sum, DL/nn/mkldnn/Fusion.scala:120-165): [M][ldr] int8 (the
  // block input's code: (q + res_zero) · res_scale) or bf16; res_kind 0 = none, 1 = int8, 2 = bf16
  const void* res;
  int res_kind, ldr;
  float res_scale, res_zero;
};

// the residual of output pixel m, channels n .. n + 3 (m < M, n + 3 < K)
__device__ __forceinline__ void i8_res4(const ConvI8Params& p, int m, int n, float (&r)[4]) {
  if (p.res_kind == 1) {
    const uint32_t u = *reinterpret_cast<const uint32_t*>((const int8_t*)p.res + (size_t)m * p.ldr + n);
#pragma unroll
    for (int e = 0; e < 4; ++e) r[e] = ((float)(int8_t)((u >> (8 * e)) & 0xFFu) + p.res_zero) * p.res_scale;
  } else {
    const uint2 u = *reinterpret_cast<const uint2*>((const bf16_t*)p.res + (size_t)m * p.ldr + n);
    r[0] = __uint_as_float(u.x << 16);
    r[1] = __uint_as_float(u.x & 0xFFFF0000u);
    r[2] = __uint_as_float(u.y << 16);
    r[3] = __uint_as_float(u.y & 0xFFFF0000u);
  }
}

// NS: LDS ring depth — 3 (the k-loop pipeline), or 2 for the short reductions (KT ≤ 2: the 1×1 convs
// over ≤ 256 channels) on 128-row tiles, where the launch is load → one or two MFMA tiles → store and
// two blocks per CU overlap one block's epilogue with the other's loads (one 147 KB block per CU did not)
// NS == 1 (KT == 1 launches only: the 1×1 convs over ≤ 128 channels, or C = 64): no ring at all.
// MINB: blocks per CU the register budget is sized for.
template <int BM, int BN, int WM, int WN, int TPT, int NS = 3, int MINB = (NS == 2 ? 2 : 1)>
__global__ void __launch_bounds__(64 * WM * WN, MINB) k_conv_i8(ConvI8Params p) {
  static_assert(NS >= 1 && NS <= 3, "LDS ring depth");
  constexpr int NT = 64 * WM * WN, NW = WM * WN;
  constexpr int STAGE = (BM + BN) * 128;
  constexpr int GA = BN / 8 / NW, GB = BM / 8 / NW;
  static_assert(GA * NW * 8 == BN && GB * NW * 8 == BM, "tile rows must split evenly over the waves");
  constexpr int L = GA + GB;
  constexpr int TMI = BM / WM / 32, TNI = BN / WN / 32;
  constexpr int EPI = BM * BN * 4;  // (the fp32 conv + sum tile; the bf16 tile needs half)
  constexpr int LDS_BYTES = NS * STAGE > EPI ? NS * STAGE : EPI;
  __shared__ __attribute__((aligned(16))) unsigned char lds[LDS_BYTES];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wave_m = wid % WM, wave_n = wid / WM;
  const int tile = xcd_remap(blockIdx.x, gridDim.x);
  const int tm = tile / p.tiles_n, tn = tile - tm * p.tiles_n;
  const int m0 = tm * BM, n0 = tn * BN;

  const uint32_t x_bytes = (uint32_t)((size_t)p.Nb * p.H * p.W * p.C);
  const uint32_t w_bytes = (uint32_t)((size_t)p.K * p.ldw);
  const __amdgpu_buffer_rsrc_t xr =
      __builtin_amdgcn_make_buffer_rsrc((void*)p.x, 0, (int)(x_bytes + (p.x_u8 ? 16u : 0u)), 0x00020000);
  const __amdgpu_buffer_rsrc_t wr = __builtin_amdgcn_make_buffer_rsrc((void*)p.w, 0, (int)w_bytes, 0x00020000);
  constexpr uint32_t OOB = 0x80000000u;
  const uint32_t XPAD = p.x_u8 ? x_bytes : OOB;  // a padded tap: the 0x80 tail, or zero-fill
  const int RS = p.R * p.S;

  const int lrow = lane >> 3, slot = lane & 7;
  uint32_t woff[GA];
#pragma unroll
  for (int i = 0; i < GA; ++i) {
    const int row = 8 * (wid + NW * i) + lrow;
    const int chunk = slot ^ ((row >> 1) & 7);
    const int n = n0 + row;
    woff[i] = n < p.K ? (uint32_t)n * (uint32_t)p.ldw + (uint32_t)chunk * 16u : OOB;
  }
  // per-lane activation source: pixel base + this lane's chunk inside the tap (TPT == 2: the low
  // four chunks belong to the tile's first tap, the high four to its second)
  int rbase[GB];
  uint64_t vmask[GB];
  int cinj[GB];  // TPT == 1: this lane's channel offset inside the k-tile (C % 128 != 0: the last k-tile
                 // of a tap is partial, its chunks past C read the pad code)
  int hi_half = 0;
  const bool pointwise = p.R == 1 && p.S == 1 && p.sh == 1 && p.sw == 1 && p.ph == 0 && p.pw == 0 &&
                         p.P == p.H && p.Q == p.W;
#pragma unroll
  for (int j = 0; j < GB; ++j) {
    const int row = 8 * (wid + NW * j) + lrow;
    const int chunk = slot ^ ((row >> 1) & 7);
    hi_half = chunk >> 2;  // the same for every j (rows 8 apart share (row >> 1) & 7 … per group)
    const int m = m0 + row;
    const int cin = TPT == 2 ? (chunk & 3) * 16 : chunk * 16;
    cinj[j] = cin;
    if (pointwise) {  // output pixel m reads input pixel m: no index divisions, one tap
      rbase[j] = m * p.C + cin;
      vmask[j] = m < p.M ? 1ull : 0ull;
      continue;
    }
    int img = -1, h = 0, w = 0;
    if (m < p.M) {
      const int n = m / (p.P * p.Q);
      const int pq = m - n * p.P * p.Q;
      const int pp = pq / p.Q, qq = pq - pp * p.Q;
      img = n;
      h = pp * p.sh - p.ph;
      w = qq * p.sw - p.pw;
    }
    rbase[j] = ((img * p.H + h) * p.W + w) * p.C + cin;
    uint64_t msk = 0;
    if (img >= 0) {
      for (int r = 0; r < p.R; ++r) {
        const int hh = h + r * p.dh;
        if ((unsigned)hh >= (unsigned)p.H) continue;
        for (int sx = 0; sx < p.S; ++sx) {
          const int ww = w + sx * p.dw;
          if ((unsigned)ww < (unsigned)p.W) msk |= 1ull << (r * p.S + sx);
        }
      }
    }
    vmask[j] = msk;
  }
  (void)hi_half;

  // wave-uniform tap iterator: (tap, offset of tap in the activation, channel base inside the tap)
  int it_tap = 0, it_s = 0, it_off = 0, it_c0 = 0;
  auto next_tap = [&]() {
    ++it_tap;
    if (++it_s == p.S) {
      it_s = 0;
      it_off += (p.dh * p.W - (p.S - 1) * p.dw) * p.C;
    } else {
      it_off += p.dw * p.C;
    }
  };
  auto stage = [&](int kt, int slotbuf) {
    unsigned char* base = lds + slotbuf * STAGE;
    const uint32_t kb = (uint32_t)kt * 128u;
#pragma unroll
    for (int i = 0; i < GA; ++i) i8_glds16(wr, base + 8 * (wid + NW * i) * 128, woff[i] + kb);
    int tap_a, off_a, tap_b = 0, off_b = 0, c0 = 0;
    if (TPT == 2) {
      tap_a = it_tap;
      off_a = it_off;
      next_tap();
      tap_b = it_tap;
      off_b = it_off;
      next_tap();
    } else {
      tap_a = it_tap;
      off_a = it_off;
      c0 = it_c0;
      it_c0 += 128;
      if (it_c0 >= p.C) {  // (C % 128 != 0: ⌈C / 128⌉ k-tiles per tap)
        it_c0 = 0;
        next_tap();
      }
    }
#pragma unroll
    for (int j = 0; j < GB; ++j) {
      const int row = 8 * (wid + NW * j) + lrow;
      const int chunk = slot ^ ((row >> 1) & 7);
      unsigned char* dst = base + (BN + 8 * (wid + NW * j)) * 128;
      uint32_t off;
      if (TPT == 2) {
        const bool hi = chunk >= 4;
        const int tap = hi ? tap_b : tap_a;
        const bool ok = tap < RS && ((vmask[j] >> tap) & 1ull);
        off = ok ? (uint32_t)(rbase[j] + (hi ? off_b : off_a)) : XPAD;
      } else {
        const bool ok = ((vmask[j] >> tap_a) & 1ull) && c0 + cinj[j] < p.C;
        off = ok ? (uint32_t)(rbase[j] + off_a + c0) : XPAD;
      }
      i8_glds16(xr, dst, off);
    }
  };

  v16i acc[TNI][TMI];
#pragma unroll
  for (int i = 0; i < TNI; ++i)
#pragma unroll
    for (int j = 0; j < TMI; ++j)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[i][j][e] = 0;

  const int frow = lane & 31, fh = lane >> 5;
  int foff[4];
#pragma unroll
  for (int kk = 0; kk < 4; ++kk) foff[kk] = frow * 128 + (((kk * 2 + fh) ^ ((frow >> 1) & 7)) << 4);
  const int a_row0 = wave_n * (BN / WN), b_row0 = BN + wave_m * (BM / WM);

  auto compute = [&](int slotbuf) {
    const unsigned char* base = lds + slotbuf * STAGE;
#pragma unroll
    for (int kk = 0; kk < 4; ++kk) {
      v4i af[TNI], bfr[TMI];
#pragma unroll
      for (int i = 0; i < TNI; ++i) af[i] = *reinterpret_cast<const v4i*>(base + (a_row0 + 32 * i) * 128 + foff[kk]);
#pragma unroll
      for (int j = 0; j < TMI; ++j) bfr[j] = *reinterpret_cast<const v4i*>(base + (b_row0 + 32 * j) * 128 + foff[kk]);
#pragma unroll
      for (int i = 0; i < TNI; ++i)
#pragma unroll
        for (int j = 0; j < TMI; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_i32_32x32x32_i8(af[i], bfr[j], acc[i][j], 0, 0, 0);
    }
  };

  // conv + sum with an int8 residual and int8 output: the row pass's residual codes (16 per item,
  // BM·BN/16/NT items per thread) are requested now, so their latency hides under the operand loads
  // and the MFMAs instead of following them (the short-reduction convs are one load → one k-tile →
  // epilogue per block: the residual round trip was a second exposed HBM latency)
  constexpr int RPI = (BM * (BN / 16) + NT - 1) / NT;
  uint4 rpre[RPI];
  const bool res_pre = p.yq && p.res_kind == 1;
  if (res_pre) {
#pragma unroll
    for (int it = 0; it < RPI; ++it) {
      const int idx = tid + NT * it;
      const int row = idx / (BN / 16), g16 = idx - row * (BN / 16);
      const int m = m0 + row, n = n0 + g16 * 16;
      rpre[it] = (idx < BM * (BN / 16) && m < p.M && n < p.K)
                     ? *reinterpret_cast<const uint4*>((const int8_t*)p.res + (size_t)m * p.ldr + n)
                     : make_uint4(0, 0, 0, 0);
    }
  }
  const int KT = p.KT;  // (NS == 2: the host launches KT ≤ 2 only)
  stage(0, 0);
  if (KT > 1) {
    stage(1, 1);
    I8_WAIT(L);
  } else {
    I8_WAIT(0);
  }
  I8_BARRIER();
  int cur = 0, nxt = 2;
  for (int t = 0; t + 2 < KT; ++t) {
    stage(t + 2, nxt);
    compute(cur);
    I8_WAIT(L);
    I8_BARRIER();
    cur = cur == NS - 1 ? 0 : cur + 1;
    nxt = nxt == NS - 1 ? 0 : nxt + 1;
  }
  if (KT >= 2) {
    compute(cur);
    I8_WAIT(0);
    I8_BARRIER();
    cur = cur == NS - 1 ? 0 : cur + 1;
  }
  compute(cur);
  I8_BARRIER();  // the epilogue reuses the ring's LDS

  // dequantise (acc · sx[img] · sw[n] + bias, ReLU) and park as bf16 [BM][BN]
  constexpr int CMASK = (BN / 8 - 1) & 15;
  bf16_t* et = reinterpret_cast<bf16_t*>(lds);
  const int pm = lane & 31;
  float sxm[TMI];
#pragma unroll
  for (int j = 0; j < TMI; ++j) {
    const int m = m0 + (b_row0 - BN) + 32 * j + pm;
    sxm[j] = m < p.M ? (p.sx ? p.sx[m / (p.P * p.Q)] : p.sxs) : 0.f;
  }
  if (p.yq && p.res_kind) {
    // conv + sum with an int8 output: park the dequantised tile as fp32 [BM][BN] (16-B chunk c of row r
    // at c ^ (r & (BN/4 − 1))), then a row-major pass adds the residual with whole-row reads (16
    // consecutive channels per thread), applies the ReLU, requantises and stores 16 B — the residual
    // is never read in the accumulator layout (32 rows × 4 B per wave-instruction)
    // The tile holds the pre-rounding code t = v/out_scale + cadd (+ the residual's constant term
    // for an int8 residual), so the row pass is one fma per element before the rounding.
    constexpr int CPRF = BN / 4;
    float* ef = reinterpret_cast<float*>(lds);
    const float cadd = (p.y_u8 ? 0.f : 128.f) +
                       (p.res_kind == 1 ? (p.res_zero - 128.f) * p.res_scale * p.out_inv : 0.f);
    const bool stat = p.sx == nullptr;
#pragma unroll
    for (int i = 0; i < TNI; ++i)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int nl = a_row0 + 32 * i + 8 * g + 4 * fh;
        float a4[4], c4[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int n = n0 + nl + e;
          const float sw = n < p.K ? p.swt[n] : 0.f;
          const float b = (p.bias && n < p.K) ? p.bias[n] : 0.f;
          a4[e] = sw * p.out_inv * (stat ? p.sxs : 1.f);
          c4[e] = fmaf(b, p.out_inv, cadd);
        }
#pragma unroll
        for (int j = 0; j < TMI; ++j) {
          const int ml = (b_row0 - BN) + 32 * j + pm;
          const float sj = stat ? 1.f : sxm[j];
          float4 v;
          v.x = fmaf((float)acc[i][j][4 * g + 0] * sj, a4[0], c4[0]);
          v.y = fmaf((float)acc[i][j][4 * g + 1] * sj, a4[1], c4[1]);
          v.z = fmaf((float)acc[i][j][4 * g + 2] * sj, a4[2], c4[2]);
          v.w = fmaf((float)acc[i][j][4 * g + 3] * sj, a4[3], c4[3]);
          *reinterpret_cast<float4*>(ef + ml * BN + (((nl >> 2) ^ (ml & (CPRF - 1))) << 2)) = v;
        }
      }
    __syncthreads();
    constexpr int G16 = BN / 16;  // 16-channel groups per tile row
#pragma unroll
    for (int it = 0; it < RPI; ++it) {
      const int idx = tid + NT * it;
      if (idx >= BM * G16) break;
      const int row = idx / G16, g16 = idx - row * G16;
      const int m = m0 + row, n = n0 + g16 * 16;
      if (m >= p.M || n >= p.K) continue;
      float v[16];
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        const float4 f = *reinterpret_cast<const float4*>(ef + row * BN + (((g16 * 4 + c) ^ (row & (CPRF - 1))) << 2));
        v[4 * c] = f.x; v[4 * c + 1] = f.y; v[4 * c + 2] = f.z; v[4 * c + 3] = f.w;
      }
      if (p.res_kind == 1) {
        // the int8 residual's 16 codes in one load; code q → q + 128 = byte ^ 0x80 as an unsigned
        // byte (v_cvt_f32_ubyteN): value (q + res_zero)·s = ub·s + (res_zero − 128)·s, the constant
        // already in the tile
        const uint4 rq = rpre[it];
        const uint32_t rw[4] = {rq.x ^ 0x80808080u, rq.y ^ 0x80808080u, rq.z ^ 0x80808080u, rq.w ^ 0x80808080u};
        const float rs = p.res_scale * p.out_inv;
#pragma unroll
        for (int c = 0; c < 4; ++c)
#pragma unroll
          for (int e = 0; e < 4; ++e)
            v[4 * c + e] = fmaf((float)((rw[c] >> (8 * e)) & 0xFFu), rs, v[4 * c + e]);
      } else {
#pragma unroll
        for (int c = 0; c < 4; ++c) {
          float r4[4];
          i8_res4(p, m, n + 4 * c, r4);
#pragma unroll
          for (int e = 0; e < 4; ++e) v[4 * c + e] = fmaf(r4[e], p.out_inv, v[4 * c + e]);
        }
      }
      const float ulo = p.y_u8 ? 0.f : (p.relu ? 128.f : 1.f);
      uint32_t w4[4];
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        uint32_t packed = 0;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          // an exact integer in [0, 255]: the byte convert-and-insert needs no rounding of its own
          const float u = __builtin_amdgcn_fmed3f(rintf(v[4 * c + e]), ulo, 255.f);
          packed = __builtin_amdgcn_cvt_pk_u8_f32(u, e, packed);
        }
        w4[c] = packed ^ 0x80808080u;
      }
      *reinterpret_cast<uint4*>(p.yq + (size_t)m * p.ldy + n) = make_uint4(w4[0], w4[1], w4[2], w4[3]);
    }
    if (p.y_u8 && p.ldy == p.K && blockIdx.x == 0 && tid == 0)
      *reinterpret_cast<uint4*>(p.yq + (size_t)p.M * p.ldy) = make_uint4(0x80808080u, 0x80808080u, 0x80808080u,
                                                                         0x80808080u);
    return;
  }
  if (p.yq) {
    // int8 output: requantise with the consumer's static scale and park the tile as bytes
    // ([BM][BN], 16-B chunk c of row r at chunk c ^ (r & 7)), then one 16-B store per chunk.
    // The code is formed unsigned — u = med3(rint(acc·a + c), lo, 255), a = sx·sw·(1/out_scale),
    // c = bias/out_scale (+128 for the signed code) — and stored as u ^ 0x80 (the offset u8 code, or
    // the signed code's two's complement): one fma, one rounding, one clamp per element (the separate
    // dequantise / ReLU / requantise / clamp / offset / mask sequence made this epilogue VALU-bound on
    // the short-reduction 1x1 convs: ~1700 VALU per wave for 16 MFMAs)
    int8_t* eq = reinterpret_cast<int8_t*>(lds);
    const float cadd = p.y_u8 ? 0.f : 128.f;
    const float ulo = p.y_u8 ? 0.f : (p.relu ? 128.f : 1.f);
    const bool stat = p.sx == nullptr && !p.res_kind;
#pragma unroll
    for (int i = 0; i < TNI; ++i)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int nl = a_row0 + 32 * i + 8 * g + 4 * fh;
        float a4[4], c4[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int n = n0 + nl + e;
          const float sw = n < p.K ? p.swt[n] : 0.f;
          const float b = (p.bias && n < p.K) ? p.bias[n] : 0.f;
          a4[e] = sw * p.out_inv * (stat ? p.sxs : 1.f);
          c4[e] = fmaf(b, p.out_inv, cadd);
        }
#pragma unroll
        for (int j = 0; j < TMI; ++j) {
          const int ml = (b_row0 - BN) + 32 * j + pm;
          uint32_t packed = 0;
          if (stat) {
#pragma unroll
            for (int e = 0; e < 4; ++e) {
              const float u = __builtin_amdgcn_fmed3f(rintf(fmaf((float)acc[i][j][4 * g + e], a4[e], c4[e])), ulo, 255.f);
              packed = __builtin_amdgcn_cvt_pk_u8_f32(u, e, packed);
            }
          } else {
            float r4[4] = {0.f, 0.f, 0.f, 0.f};
            if (p.res_kind && m0 + ml < p.M && n0 + nl < p.K) i8_res4(p, m0 + ml, n0 + nl, r4);
#pragma unroll
            for (int e = 0; e < 4; ++e) {
              const float v = fmaf((float)acc[i][j][4 * g + e] * sxm[j], a4[e], fmaf(r4[e], p.out_inv, c4[e]));
              const float u = __builtin_amdgcn_fmed3f(rintf(v), ulo, 255.f);
              packed = __builtin_amdgcn_cvt_pk_u8_f32(u, e, packed);
            }
          }
          const int off = ml * BN + ((((nl >> 4) ^ (ml & 7)) & (BN / 16 - 1)) << 4) + (nl & 15);
          *reinterpret_cast<uint32_t*>(eq + off) = packed ^ 0x80808080u;
        }
      }
    __syncthreads();
    constexpr int CPR = BN / 16;  // 16-B chunks per tile row
#pragma unroll
    for (int it = 0; it < BM * CPR / NT; ++it) {
      const int idx = tid + NT * it;
      const int row = idx / CPR, ch = idx - row * CPR;
      const int m = m0 + row, n = n0 + ch * 16;
      if (m < p.M && n < p.K) {
        const uint4 v = *reinterpret_cast<const uint4*>(eq + row * BN + (((ch ^ (row & 7)) & (CPR - 1)) << 4));
        *reinterpret_cast<uint4*>(p.yq + (size_t)m * p.ldy + n) = v;
      }
    }
    // the unsigned code's padding tail (the code of 0) for the consumer's padded taps
    if (p.y_u8 && p.ldy == p.K && blockIdx.x == 0 && tid == 0)
      *reinterpret_cast<uint4*>(p.yq + (size_t)p.M * p.ldy) = make_uint4(0x80808080u, 0x80808080u, 0x80808080u,
                                                                         0x80808080u);
    return;
  }
#pragma unroll
  for (int i = 0; i < TNI; ++i)
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const int nl = a_row0 + 32 * i + 8 * g + 4 * fh;
      float s4[4], b4[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int n = n0 + nl + e;
        s4[e] = n < p.K ? p.swt[n] : 0.f;
        b4[e] = (p.bias && n < p.K) ? p.bias[n] : 0.f;
      }
#pragma unroll
      for (int j = 0; j < TMI; ++j) {
        const int ml = (b_row0 - BN) + 32 * j + pm;
        float v[4], r4[4] = {0.f, 0.f, 0.f, 0.f};
        if (p.res_kind && m0 + ml < p.M && n0 + nl < p.K) i8_res4(p, m0 + ml, n0 + nl, r4);
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          v[e] = fmaf((float)acc[i][j][4 * g + e] * sxm[j], s4[e], b4[e]) + r4[e];
          if (p.relu) v[e] = fmaxf(v[e], 0.f);
        }
        const uint32_t lo = (uint32_t)f2bf(v[0]) | ((uint32_t)f2bf(v[1]) << 16);
        const uint32_t hi = (uint32_t)f2bf(v[2]) | ((uint32_t)f2bf(v[3]) << 16);
        *reinterpret_cast<uint2*>(&et[ml * BN + (((nl >> 3) ^ (ml & CMASK)) << 3) + (nl & 4)]) = make_uint2(lo, hi);
      }
    }
  __syncthreads();
  ConvParams q{};
  q.y = p.y;
  q.ldy = p.ldy;
  q.M = p.M;
  q.K = p.K;
  conv_store_pass<BM, BN, NT>(q, et, tid, m0, n0, tm, false);
}

// ---- activation quantisation: per-image absmax, then int8 with scale amax / 127 ----------------
__global__ void __launch_bounds__(256) k_absmax_img(const bf16_t* __restrict__ x, long long per_img,
                                                    float* __restrict__ amax) {
  const int n = blockIdx.y;
  const bf16_t* xp = x + (long long)n * per_img;
  float m = 0.f;
  for (long long i = ((long long)blockIdx.x * 256 + threadIdx.x) * 8; i < per_img; i += (long long)gridDim.x * 256 * 8) {
    float v[8];
    load8(xp + i, v);
#pragma unroll
    for (int e = 0; e < 8; ++e) m = fmaxf(m, fabsf(v[e]));
  }
  m = wave_max(m);
  __shared__ float red[4];
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = m;
  __syncthreads();
  if (threadIdx.x == 0) {
    const float b = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
    // non-negative floats order like their bit patterns: an integer max is a float max
    atomicMax(reinterpret_cast<unsigned int*>(amax + n), __float_as_uint(b));
  }
}

__global__ void __launch_bounds__(256) k_quant_img(const bf16_t* __restrict__ x, long long per_img,
                                                   const float* __restrict__ amax, int8_t* __restrict__ xq,
                                                   float* __restrict__ sx) {
  const int n = blockIdx.y;
  const float a = amax[n];
  const float scale = a > 0.f ? a / 127.f : 1.f;
  const float inv = 1.f / scale;
  if (blockIdx.x == 0 && threadIdx.x == 0) sx[n] = scale;
  const bf16_t* xp = x + (long long)n * per_img;
  int8_t* qp = xq + (long long)n * per_img;
  for (long long i = ((long long)blockIdx.x * 256 + threadIdx.x) * 16; i < per_img;
       i += (long long)gridDim.x * 256 * 16) {
    float v[16];
    load8(xp + i, v);
    load8(xp + i + 8, v + 8);
    uint32_t w[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      uint32_t acc = 0;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float r = fminf(fmaxf(rintf(v[4 * k + e] * inv), -127.f), 127.f);
        acc |= ((uint32_t)(int)r & 0xFFu) << (8 * e);
      }
      w[k] = acc;
    }
    *reinterpret_cast<uint4*>(qp + i) = make_uint4(w[0], w[1], w[2], w[3]);
  }
}

// Static (calibrated) quantisation: xq = clamp(rint(x / scale), ±127), 16 elements per thread.
template <typename T>
__global__ void __launch_bounds__(256) k_quant_static(const T* __restrict__ x, long long n, float inv,
                                                      int8_t* __restrict__ xq, int u8) {
  const float lo = u8 ? 0.f : -127.f, hi = u8 ? 255.f : 127.f, off = u8 ? 128.f : 0.f;
  if (u8 && blockIdx.x == 0 && threadIdx.x == 0)
    *reinterpret_cast<uint4*>(xq + n) = make_uint4(0x80808080u, 0x80808080u, 0x80808080u, 0x80808080u);
  for (long long i = ((long long)blockIdx.x * 256 + threadIdx.x) * 16; i < n; i += (long long)gridDim.x * 256 * 16) {
    float v[16];
    if constexpr (sizeof(T) == 2) {
      load8(x + i, v);
      load8(x + i + 8, v + 8);
    } else {
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const float4 f = *reinterpret_cast<const float4*>(x + i + 4 * q);
        v[4 * q] = f.x; v[4 * q + 1] = f.y; v[4 * q + 2] = f.z; v[4 * q + 3] = f.w;
      }
    }
    uint32_t w[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      uint32_t acc = 0;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float r = fminf(fmaxf(rintf(v[4 * k + e] * inv), lo), hi) - off;
        acc |= ((uint32_t)(int)r & 0xFFu) << (8 * e);
      }
      w[k] = acc;
    }
    *reinterpret_cast<uint4*>(xq + i) = make_uint4(w[0], w[1], w[2], w[3]);
  }
}

// dtype 0 = fp32, 1 = bf16; n % 16 == 0, 16-B aligned; u8: non-negative input stored offset by −128
BIGDL_EXPORT int bigdl_quant_static2(const void* x, int dtype, long long n, float scale, void* xq, int u8,
                                     hipStream_t s);
BIGDL_EXPORT int bigdl_quant_static(const void* x, int dtype, long long n, float scale, void* xq, hipStream_t s) {
  return bigdl_quant_static2(x, dtype, n, scale, xq, 0, s);
}

BIGDL_EXPORT int bigdl_quant_static2(const void* x, int dtype, long long n, float scale, void* xq, int u8,
                                     hipStream_t s) {
  // u8: xq has 16 more bytes, the padding tail (0x80) of the unsigned code
  if (!x || !xq || n <= 0 || n % 16 || !(scale > 0.f) || ((uintptr_t)x & 15) || ((uintptr_t)xq & 15))
    return (int)hipErrorInvalidValue;
  const dim3 g((unsigned)bigdl_grid((n + 15) / 16, 256, 16384));
  if (dtype == 0)
    hipLaunchKernelGGL(k_quant_static<float>, g, dim3(256), 0, s, (const float*)x, n, 1.f / scale, (int8_t*)xq, u8);
  else
    hipLaunchKernelGGL(k_quant_static<bf16_t>, g, dim3(256), 0, s, (const bf16_t*)x, n, 1.f / scale, (int8_t*)xq, u8);
  BIGDL_CHECK_LAUNCH();
}

// int8 NHWC max pooling (the int8 activation between quantised convs: max commutes with the
// monotone quantisation, so the scale carries over).  16 channels per thread (C % 16); window
// positions outside the input are skipped; P, Q given (ceil / floor mode decided by the caller).
__global__ void __launch_bounds__(256) k_maxpool_i8(const int8_t* __restrict__ x, int8_t* __restrict__ y, int Nb,
                                                    int H, int W, int C, int P, int Q, int kh, int kw, int sh, int sw,
                                                    int ph, int pw, int tail) {
  const int CG = C >> 4;
  const long long total = (long long)Nb * P * Q * CG;
  if (tail && blockIdx.x == 0 && threadIdx.x == 0)  // the unsigned code's padding tail
    *reinterpret_cast<uint4*>(y + total * 16) = make_uint4(0x80808080u, 0x80808080u, 0x80808080u, 0x80808080u);
  for (long long t = (long long)blockIdx.x * 256 + threadIdx.x; t < total; t += (long long)gridDim.x * 256) {
    const int cg = (int)(t % CG);
    const long long pix = t / CG;
    const int q = (int)(pix % Q);
    const long long r = pix / Q;
    const int pp = (int)(r % P);
    const int n = (int)(r / P);
    int m[16];
#pragma unroll
    for (int e = 0; e < 16; ++e) m[e] = -128;
    const int h0 = pp * sh - ph, w0 = q * sw - pw;
    for (int i = 0; i < kh; ++i) {
      const int h = h0 + i;
      if ((unsigned)h >= (unsigned)H) continue;
      for (int j = 0; j < kw; ++j) {
        const int w = w0 + j;
        if ((unsigned)w >= (unsigned)W) continue;
        const uint4 v = *reinterpret_cast<const uint4*>(x + (((long long)n * H + h) * W + w) * C + cg * 16);
        const uint32_t u[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
        for (int e = 0; e < 16; ++e) {
          const int b = (int)(int8_t)((u[e >> 2] >> (8 * (e & 3))) & 0xFFu);
          m[e] = m[e] > b ? m[e] : b;
        }
      }
    }
    uint32_t o[4] = {0, 0, 0, 0};
#pragma unroll
    for (int e = 0; e < 16; ++e) o[e >> 2] |= ((uint32_t)m[e] & 0xFFu) << (8 * (e & 3));
    *reinterpret_cast<uint4*>(y + pix * C + cg * 16) = make_uint4(o[0], o[1], o[2], o[3]);
  }
}

// Fixed-window form (3x3 and 2x2, the Inception / VGG / ResNet pools): all KH·KW 16-B window loads of
// a thread issued before the first compare (an out-of-image tap reads the clamped window centre, which
// is inside the window for pad ≤ 1), 32-bit index math, and the byte max done two bytes per lane of
// v_pk_max_u16 on the codes flipped to unsigned order (q ^ 0x80 orders the signed and the offset code
// alike): ~5 VALU per 4 bytes per tap where byte-wise extract / compare / insert took ~11.
typedef unsigned short u16x2_t __attribute__((ext_vector_type(2)));
__device__ __forceinline__ uint32_t pk_max_u16(uint32_t a, uint32_t b) {
  u16x2_t x = __builtin_bit_cast(u16x2_t, a), y = __builtin_bit_cast(u16x2_t, b);
  return __builtin_bit_cast(uint32_t, __builtin_elementwise_max(x, y));
}

template <int KH, int KW>
__global__ void __launch_bounds__(256) k_maxpool_i8_k(const int8_t* __restrict__ x, int8_t* __restrict__ y, int Nb,
                                                      int H, int W, int C, int P, int Q, int sh, int sw, int ph,
                                                      int pw, int tail) {
  const uint32_t CG = (uint32_t)C >> 4;
  const uint32_t total = (uint32_t)Nb * P * Q * CG;
  if (tail && blockIdx.x == 0 && threadIdx.x == 0)
    *reinterpret_cast<uint4*>(y + (size_t)total * 16) = make_uint4(0x80808080u, 0x80808080u, 0x80808080u, 0x80808080u);
  for (uint32_t t = blockIdx.x * 256u + threadIdx.x; t < total; t += gridDim.x * 256u) {
    const uint32_t cg = t % CG, pix = t / CG;
    const uint32_t q = pix % (uint32_t)Q, r = pix / (uint32_t)Q;
    const uint32_t pp = r % (uint32_t)P, n = r / (uint32_t)P;
    const int h0 = (int)pp * sh - ph, w0 = (int)q * sw - pw;
    const int hc = min(max(h0 + KH / 2, 0), H - 1), wc = min(max(w0 + KW / 2, 0), W - 1);
    // one 64-bit base (the clamped centre), 32-bit tap offsets from it
    const int8_t* base = x + ((size_t)(n * (uint32_t)H + (uint32_t)hc) * (uint32_t)W + (uint32_t)wc) * C + cg * 16;
    uint4 v[KH * KW];
#pragma unroll
    for (int i = 0; i < KH; ++i)
#pragma unroll
      for (int j = 0; j < KW; ++j) {
        const int h = h0 + i, w = w0 + j;
        const bool in = (unsigned)h < (unsigned)H && (unsigned)w < (unsigned)W;
        const int off = in ? ((h - hc) * W + (w - wc)) * C : 0;
        v[i * KW + j] = *reinterpret_cast<const uint4*>(base + off);
      }
    uint32_t ev[4] = {0, 0, 0, 0}, od[4] = {0, 0, 0, 0};
#pragma unroll
    for (int k = 0; k < KH * KW; ++k) {
      const uint32_t a[4] = {v[k].x ^ 0x80808080u, v[k].y ^ 0x80808080u, v[k].z ^ 0x80808080u, v[k].w ^ 0x80808080u};
#pragma unroll
      for (int d = 0; d < 4; ++d) {
        ev[d] = pk_max_u16(ev[d], a[d] & 0x00FF00FFu);
        od[d] = pk_max_u16(od[d], (a[d] >> 8) & 0x00FF00FFu);
      }
    }
    uint4 o;
    o.x = (ev[0] | (od[0] << 8)) ^ 0x80808080u;
    o.y = (ev[1] | (od[1] << 8)) ^ 0x80808080u;
    o.z = (ev[2] | (od[2] << 8)) ^ 0x80808080u;
    o.w = (ev[3] | (od[3] << 8)) ^ 0x80808080u;
    *reinterpret_cast<uint4*>(y + (size_t)pix * C + cg * 16) = o;
  }
}

BIGDL_EXPORT int bigdl_maxpool_i8_t(const void* x, void* y, int Nb, int H, int W, int C, int P, int Q, int kh, int kw,
                                    int sh, int sw, int ph, int pw, int tail, hipStream_t s);
BIGDL_EXPORT int bigdl_maxpool_i8(const void* x, void* y, int Nb, int H, int W, int C, int P, int Q, int kh, int kw,
                                  int sh, int sw, int ph, int pw, hipStream_t s) {
  return bigdl_maxpool_i8_t(x, y, Nb, H, W, C, P, Q, kh, kw, sh, sw, ph, pw, 0, s);
}

// tail: y has 16 more bytes after its last one, set to 0x80 (an unsigned-code input's padding)
BIGDL_EXPORT int bigdl_maxpool_i8_t(const void* x, void* y, int Nb, int H, int W, int C, int P, int Q, int kh, int kw,
                                    int sh, int sw, int ph, int pw, int tail, hipStream_t s) {
  if (!x || !y || Nb <= 0 || C % 16 || P <= 0 || Q <= 0 || kh <= 0 || kw <= 0 || sh <= 0 || sw <= 0 ||
      ((uintptr_t)x & 15) || ((uintptr_t)y & 15))
    return (int)hipErrorInvalidValue;
  const long long total = (long long)Nb * P * Q * (C / 16);
  const bool small = total < 0x7fffffffLL - 65536LL * 256 && (long long)Nb * H * W < 0x7fffffffLL;
  if (small && ph <= 1 && pw <= 1 && ((kh == 3 && kw == 3) || (kh == 2 && kw == 2))) {
    const dim3 g((unsigned)bigdl_grid(total, 256, 65536));
    if (kh == 3)
      hipLaunchKernelGGL((k_maxpool_i8_k<3, 3>), g, dim3(256), 0, s, (const int8_t*)x, (int8_t*)y, Nb, H, W, C, P, Q, sh,
                         sw, ph, pw, tail);
    else
      hipLaunchKernelGGL((k_maxpool_i8_k<2, 2>), g, dim3(256), 0, s, (const int8_t*)x, (int8_t*)y, Nb, H, W, C, P, Q, sh,
                         sw, ph, pw, tail);
    BIGDL_CHECK_LAUNCH();
  }
  hipLaunchKernelGGL(k_maxpool_i8, dim3((unsigned)bigdl_grid(total, 256, 65536)), dim3(256), 0, s, (const int8_t*)x,
                     (int8_t*)y, Nb, H, W, C, P, Q, kh, kw, sh, sw, ph, pw, tail);
  BIGDL_CHECK_LAUNCH();
}

// x: [Nb][per_img] bf16 (per_img % 16 == 0, 16-B aligned) → xq int8 (same layout) and sx[Nb] (the
// dequantisation scale of each image); amax: [Nb] fp32 workspace.
BIGDL_EXPORT int bigdl_quant_img(const void* x, int Nb, long long per_img, float* amax, void* xq, float* sx,
                                 hipStream_t s) {
  if (!x || !amax || !xq || !sx || Nb <= 0 || Nb > 65535 || per_img <= 0 || per_img % 16 ||
      ((uintptr_t)x & 15) || ((uintptr_t)xq & 15))
    return (int)hipErrorInvalidValue;
  hipError_t e = hipMemsetAsync(amax, 0, sizeof(float) * Nb, s);
  if (e != hipSuccess) return (int)e;
  long long chunks = (per_img + 256 * 8 * 8 - 1) / (256 * 8 * 8);  // ≥ 8 vectors per thread
  if (chunks > 1024) chunks = 1024;
  hipLaunchKernelGGL(k_absmax_img, dim3((unsigned)chunks, (unsigned)Nb), dim3(256), 0, s, (const bf16_t*)x, per_img,
                     amax);
  hipLaunchKernelGGL(k_quant_img, dim3((unsigned)chunks, (unsigned)Nb), dim3(256), 0, s, (const bf16_t*)x, per_img,
                     (const float*)amax, (int8_t*)xq, sx);
  BIGDL_CHECK_LAUNCH();
}

// y[m][n] (bf16, row stride ldy) = [ReLU](Σ_k w[n][k]·x̂[m][k] · sx[img(m)] · sw[n] + bias[n]).
// x: int8 NHWC [Nb][H][W][C] (C % 16 == 0 or C == 64); w: int8 [K][ldw], (r, s, c) order, each tap's
// C channels zero-padded to ⌈C / 128⌉·128, ldw = KT·128 (KT = R·S·⌈C / 128⌉, or ⌈R·S / 2⌉ for C == 64);
// R·S ≤ 64; K % 8 == 0.
// sx null: one static activation scale sxs for every image (calibrated, nn/quantized); yq non-null:
// int8 output requantised by 1 / out_scale (K % 16, ldy % 16, 16-B aligned) instead of bf16 y.
BIGDL_EXPORT int bigdl_conv_i8_fwd2(const void* x, const void* w, int ldw, const float* sx, float sxs, const float* swt,
                                    const float* bias, void* y, void* yq, float out_scale, int ldy, int Nb, int H,
                                    int W, int C, int K, int R, int S, int P, int Q, int sh, int sw, int ph, int pw,
                                    int dh, int dw, int relu, hipStream_t s);

BIGDL_EXPORT int bigdl_conv_i8_fwd(const void* x, const void* w, int ldw, const float* sx, const float* swt,
                                   const float* bias, void* y, int ldy, int Nb, int H, int W, int C, int K, int R,
                                   int S, int P, int Q, int sh, int sw, int ph, int pw, int dh, int dw, int relu,
                                   hipStream_t s) {
  if (!sx) return (int)hipErrorInvalidValue;
  return bigdl_conv_i8_fwd2(x, w, ldw, sx, 0.f, swt, bias, y, nullptr, 1.f, ldy, Nb, H, W, C, K, R, S, P, Q, sh, sw, ph,
                            pw, dh, dw, relu, s);
}

BIGDL_EXPORT int bigdl_conv_i8_fwd3(const void* x, const void* w, int ldw, const float* sx, float sxs, const float* swt,
                                    const float* bias, void* y, void* yq, float out_scale, int ldy, int Nb, int H,
                                    int W, int C, int K, int R, int S, int P, int Q, int sh, int sw, int ph, int pw,
                                    int dh, int dw, int relu, int x_u8, int y_u8, hipStream_t s);

BIGDL_EXPORT int bigdl_conv_i8_fwd2(const void* x, const void* w, int ldw, const float* sx, float sxs, const float* swt,
                                    const float* bias, void* y, void* yq, float out_scale, int ldy, int Nb, int H,
                                    int W, int C, int K, int R, int S, int P, int Q, int sh, int sw, int ph, int pw,
                                    int dh, int dw, int relu, hipStream_t s) {
  return bigdl_conv_i8_fwd3(x, w, ldw, sx, sxs, swt, bias, y, yq, out_scale, ldy, Nb, H, W, C, K, R, S, P, Q, sh, sw, ph,
                            pw, dh, dw, relu, 0, 0, s);
}

BIGDL_EXPORT int bigdl_conv_i8_fwd4(const void* x, const void* w, int ldw, const float* sx, float sxs, const float* swt,
                                    const float* bias, void* y, void* yq, float out_scale, int ldy, int Nb, int H,
                                    int W, int C, int K, int R, int S, int P, int Q, int sh, int sw, int ph, int pw,
                                    int dh, int dw, int relu, int x_u8, int y_u8, const void* res, int res_kind,
                                    int ldr, float res_scale, float res_zero, hipStream_t s);

// default 2 (tools/i8_shortk_bench.py, batch 256: 64→256 at 56² with the residual 266 → 230 µs,
// 128→512 at 28² 103 → 92.5; the int8 ResNet-50 forward 4.37-4.39 → 4.23 ms per batch in 3 interleaved
// repeats, VGG16 unchanged — profiles/r6_int8.txt)
static int g_i8_shortk = [] {
  const char* e = getenv("BIGDL_I8_SHORTK");
  return e ? atoi(e) : 2;
}();

// the short-K tile variant (measurement hook: tools/i8_shortk_bench.py); returns the previous one
BIGDL_EXPORT int bigdl_conv_i8_set_shortk(int v) {
  const int old = g_i8_shortk;
  if (v >= 0 && v <= 2) g_i8_shortk = v;
  return old;
}

BIGDL_EXPORT int bigdl_conv_i8_fwd3(const void* x, const void* w, int ldw, const float* sx, float sxs, const float* swt,
                                    const float* bias, void* y, void* yq, float out_scale, int ldy, int Nb, int H,
                                    int W, int C, int K, int R, int S, int P, int Q, int sh, int sw, int ph, int pw,
                                    int dh, int dw, int relu, int x_u8, int y_u8, hipStream_t s) {
  return bigdl_conv_i8_fwd4(x, w, ldw, sx, sxs, swt, bias, y, yq, out_scale, ldy, Nb, H, W, C, K, R, S, P, Q, sh, sw,
                            ph, pw, dh, dw, relu, x_u8, y_u8, nullptr, 0, 0, 1.f, 0.f, s);
}

// res (res_kind 1: int8 [M][ldr], value (q + res_zero)·res_scale; 2: bf16 [M][ldr]): added to the
// dequantised output before the ReLU (ldr % 4 == 0, 8-B aligned rows for bf16)
BIGDL_EXPORT int bigdl_conv_i8_fwd4(const void* x, const void* w, int ldw, const float* sx, float sxs, const float* swt,
                                    const float* bias, void* y, void* yq, float out_scale, int ldy, int Nb, int H,
                                    int W, int C, int K, int R, int S, int P, int Q, int sh, int sw, int ph, int pw,
                                    int dh, int dw, int relu, int x_u8, int y_u8, const void* res, int res_kind,
                                    int ldr, float res_scale, float res_zero, hipStream_t s) {
  // x_u8: x holds 16 bytes of 0x80 after its last byte (and the bias carries the offset term);
  // y_u8: yq is dense (ldy == K) with room for that tail, or a channel slice of a wider tensor
  // (ldy > K: a zero-copy concat whose owner writes the tail)
  if (y_u8 && !yq) return (int)hipErrorInvalidValue;
  if (res_kind < 0 || res_kind > 2 || (res_kind && (!res || ldr < K || ldr % 4 || ((uintptr_t)res & 7))))
    return (int)hipErrorInvalidValue;
  if (!x || !w || (!sx && !(sxs > 0.f)) || !swt || (!y && !yq) || Nb <= 0 || K <= 0 || K % 8 || P <= 0 || Q <= 0)
    return (int)hipErrorInvalidValue;
  if (yq && (K % 16 || ldy % 16 || ((uintptr_t)yq & 15) || !(out_scale > 0.f))) return (int)hipErrorInvalidValue;
  // C % 128 != 0 (C % 16 == 0, e.g. Inception's 480 / 528 / 832-channel concats): every tap takes
  // ⌈C / 128⌉ k-tiles and the weight rows are zero-padded per tap to that many 128-byte tiles
  const int tpt = C == 64 ? 2 : (C % 16 == 0 ? 1 : 0);
  if (!tpt || R * S > 64 || R <= 0 || S <= 0) return (int)hipErrorInvalidValue;
  const int KT = tpt == 2 ? (R * S + 1) / 2 : R * S * ((C + 127) / 128);
  if (ldw != KT * 128 || ldy < K || ldy % 8 || ((uintptr_t)x & 15) || ((uintptr_t)w & 15) || ((uintptr_t)y & 15))
    return (int)hipErrorInvalidValue;
  if ((size_t)Nb * H * W * C >= 0x80000000ull || (size_t)K * ldw >= 0x80000000ull) return (int)hipErrorInvalidValue;
  const long long Ml = (long long)Nb * P * Q;
  if (Ml > 0x7fffffffLL) return (int)hipErrorInvalidValue;
  ConvI8Params p{};
  p.x = (const int8_t*)x; p.w = (const int8_t*)w; p.sx = sx; p.swt = swt; p.bias = bias; p.y = (bf16_t*)y;
  p.Nb = Nb; p.H = H; p.W = W; p.C = C; p.K = K; p.R = R; p.S = S; p.P = P; p.Q = Q;
  p.sh = sh; p.sw = sw; p.ph = ph; p.pw = pw; p.dh = dh; p.dw = dw;
  p.M = (int)Ml; p.KT = KT; p.ldw = ldw; p.ldy = ldy; p.relu = relu;
  p.sxs = sxs; p.yq = (int8_t*)yq; p.out_inv = yq ? 1.f / out_scale : 1.f;
  p.x_u8 = x_u8; p.y_u8 = y_u8;
  p.res = res; p.res_kind = res_kind; p.ldr = ldr; p.res_scale = res_scale; p.res_zero = res_zero;
  // 256 × 128 tiles; K ≤ 64 (VGG's 64-channel 224² convs, a quarter of the int8 net's time) takes a
  // 256 × 64 tile instead of leaving half of every 128-wide tile's MFMA work and staging idle
  const int BN = K <= 64 ? 64 : 128;
  const bool short_k = KT <= 2 && BN == 128;  // short reductions: small tiles, several blocks per CU
  // short-K tile (g_i8_shortk): 0 = 128 × 128, 2-deep ring, 2 blocks/CU; 1 = 64 × 128, 2-deep ring,
  // 3 blocks/CU; 2 = as 1, and for a single k-tile no ring (32 KB of LDS, 5 blocks/CU)
  int sk = short_k ? g_i8_shortk : 0;
  if (sk == 2 && KT != 1) sk = 0;  // variant 2 differs from 0 on single-k-tile launches only
  const int BM = short_k ? (sk ? 64 : 128) : 256;
  p.tiles_n = (K + BN - 1) / BN;
  const long long tiles = (long long)((p.M + BM - 1) / BM) * p.tiles_n;
  if (tiles > 0x7fffffff) return (int)hipErrorInvalidValue;
  const dim3 g((unsigned)tiles);
  if (short_k) {
    if (sk == 2) {
      if (tpt == 2) hipLaunchKernelGGL((k_conv_i8<64, 128, 2, 2, 2, 1, 5>), g, dim3(256), 0, s, p);
      else hipLaunchKernelGGL((k_conv_i8<64, 128, 2, 2, 1, 1, 5>), g, dim3(256), 0, s, p);
    } else if (sk == 1) {
      if (tpt == 2) hipLaunchKernelGGL((k_conv_i8<64, 128, 2, 2, 2, 2, 3>), g, dim3(256), 0, s, p);
      else hipLaunchKernelGGL((k_conv_i8<64, 128, 2, 2, 1, 2, 3>), g, dim3(256), 0, s, p);
    } else {
      if (tpt == 2) hipLaunchKernelGGL((k_conv_i8<128, 128, 2, 2, 2, 2>), g, dim3(256), 0, s, p);
      else hipLaunchKernelGGL((k_conv_i8<128, 128, 2, 2, 1, 2>), g, dim3(256), 0, s, p);
    }
    BIGDL_CHECK_LAUNCH();
  }
  if (BN == 64) {
    if (tpt == 2) hipLaunchKernelGGL((k_conv_i8<256, 64, 4, 2, 2>), g, dim3(512), 0, s, p);
    else hipLaunchKernelGGL((k_conv_i8<256, 64, 4, 2, 1>), g, dim3(512), 0, s, p);
  } else {
    if (tpt == 2) hipLaunchKernelGGL((k_conv_i8<256, 128, 4, 2, 2>), g, dim3(512), 0, s, p);
    else hipLaunchKernelGGL((k_conv_i8<256, 128, 4, 2, 1>), g, dim3(512), 0, s, p);
  }
  BIGDL_CHECK_LAUNCH();
}
