// Implicit-GEMM convolution on MFMA (K1 forward, K2 stride-1 backward-data), NHWC bf16 -> bf16,
// fp32 accumulation.  Reference: SpatialConvolution.updateOutput (im2col + MKL sgemm per sample,
// DL/nn/SpatialConvolution.scala:253-362, NNPrimitive.im2colFloat :108); here no im2col is ever
// materialised — the A operand is gathered straight from the NHWC activation.
//
// GEMM view:   D[n = out channel][m = output pixel] = Σ_k W[n][k] · X̂[m][k],  k = (r, s, c)
//   A operand (MFMA rows)  = weights, KRSC  → row n contiguous in k
//   B operand (MFMA cols)  = im2col rows gathered on the fly, NHWC → 8 channels per 16-B chunk
//   so each lane's accumulator holds 4 consecutive OUTPUT CHANNELS of one pixel (D layout of
//   mfma_f32_16x16x32_bf16: row=(lane>>4)*4+j, col=lane&15) → 8-byte NHWC stores.
//
// Tiling: block 128 pixels × BN channels × BK (64, or 32 for shallow reductions), 256 threads =
// 4 waves (2 × 2), each wave (BN/2) × 64 = (BN/32) × 4 MFMA 16×16×32 tiles.  Global→LDS through registers (the gather needs
// per-row zero padding, so no global_load_lds), double-buffered LDS, one barrier per k-tile, the
// next tile's loads issued before the current tile's MFMAs (T14 split).  LDS rows are 128 B with
// a 16-B-chunk XOR swizzle (chunk ^ (row & 7)) so the ds_read_b128 fragment reads of 16 distinct
// rows are conflict-free (cdna_hip_programming.md T2).  Blocks are remapped so each XCD gets a
// contiguous range of tiles (T1; bijective for any grid size).
#include "conv_params.h"

// raising the wave priority around the MFMA phase (the 256² GEMM template's idiom) measured 4 %
// slower on the ResNet-50 conv set at this 128² 2–3-blocks/CU structure: off by default
#ifndef BIGDL_CONV_SETPRIO
#define BIGDL_CONV_SETPRIO 0
#endif

// k-tile depth is a kernel parameter (64 or 32).  A fragment read (ds_read_b128) is serviced in four
// 16-lane groups ({0–3,12–15,20–27}, {4–11,16–19,28–31} and the same +32, MI355X_MICROARCH.md §LDS):
// a group holds rows r..r+15 of the tile, half of them at chunk c and half at chunk c^1, and the XOR
// swizzle must put its 16 reads in 16 distinct 16-B slots of the 256-B bank window.
// 64-wide rows (128 B, 2 rows per window): chunk ^ (row & 7).
// 32-wide rows (64 B, 4 rows per window): chunk ^ ((row >> 2) & 2).  (The former
// chunk ^ ((row >> 2) & 3) put rows r and r + 4 of the same group on one slot: 8 LDS cycles per
// fragment read instead of 4 — found with a lane-group bank model of both formulas.)
template <int BK>
__device__ __forceinline__ int swz(int row, int chunk) {
  if constexpr (BK == 64) return row * BK + ((chunk ^ (row & 7)) << 3);
  else return row * BK + ((chunk ^ ((row >> 2) & 2)) << 3);
}


// MODE 1 (FAST): C % BK == 0 and R·S ≤ 64 — every k-tile lies inside one filter tap, so the tap /
// channel position of a k-tile is wave-uniform (scalar registers, no per-lane division) and the
// padding test of a staged row is one bit of a per-row tap-validity mask built once in the prologue.
// MODE 2 (C4): 4-channel input (the RGB stem padded 3 → 4, not 8: 1.33× instead of 2.67× padded
// MACs and half the input bytes) — a 16-B chunk holds two consecutive taps, gathered as two 8-B
// loads with their own padding tests.  MODE 0: any C % 8 == 0.  MODE 3 (POINTWISE): a 1×1
// filter with no padding (C % BK == 0) — every staged row is in bounds, the k-tile is a plain
// channel offset, no tap mask at all (the bottleneck 1×1 convs and their dgrads, half the FLOPs).
template <int BN, int MODE, int BM, int BK, bool D3 = false, bool AT = false>
__global__ void __launch_bounds__(256, BM == 256 ? 1 : (BK == 32 && !AT ? 3 : 2)) k_conv_fwd(ConvParams p) {
  static_assert(!D3 || MODE == 0 || MODE == 1, "3-D: generic or tap-uniform gather only");
  static_assert(!AT || MODE == 3, "BN-backward prologue: pointwise mode only");
  constexpr bool PW = MODE == 3;
  constexpr bool FAST = MODE == 1 || PW;
  constexpr int ROWS = BM + BN;
  constexpr int CPK = BK / 8;    // 16-B chunks per staged row
  constexpr int RPS = 256 / CPK; // rows staged per pass of the block
  constexpr int TN = BN / 32;  // MFMA tiles along channels per wave
  constexpr int TM = BM / 32;  // MFMA tiles along pixels per wave (BM / 2 pixels)
  constexpr int A_CHUNKS = BM * BK / 8 / 256;  // activation chunks per thread (4 or 8)
  constexpr int B_CHUNKS = BN * BK / 8 / 256;  // weight chunks per thread (4 or 2)
  constexpr int STAGE = ROWS * BK;
  constexpr int EPI = BM * BN + 4 * (256 / (BN / 8)) * BN;  // epilogue tile + Σ/Σ² reduction rows
  __shared__ __attribute__((aligned(16))) bf16_t lds[2 * STAGE > EPI ? 2 * STAGE : EPI];

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wave_m = wid & 1, wave_n = wid >> 1;
  const long long grp = blockIdx.y;  // grouped conv: this block's group (0 otherwise)
  if (grp) {
    p.x += grp * p.gx;
    p.w += grp * p.gw;
    p.y += grp * p.gy;
    if (p.bias) p.bias += grp * p.gy;
  }
  const int tile = xcd_remap(blockIdx.x, gridDim.x);
  const int tm = tile / p.tiles_n, tn = tile - tm * p.tiles_n;
  const int m0 = tm * BM, n0 = tn * BN;
  // the BN-statistics shift of this lane's channels, fetched before the main loop so the epilogue
  // does not wait on a dependent global load per tile (shifted statistics, rstats epilogue)
  float kpre[TN][4];
#pragma unroll
  for (int i = 0; i < TN; ++i)
#pragma unroll
    for (int e = 0; e < 4; ++e) kpre[i][e] = 0.f;
  if (BM == SBM && p.stats && p.stat_shift) {
#pragma unroll
    for (int i = 0; i < TN; ++i) {
      const int nk = n0 + wave_n * (BN / 2) + i * 16 + (lane >> 4) * 4;
#pragma unroll
      for (int e = 0; e < 4; ++e) kpre[i][e] = nk + e < p.K ? p.stat_shift[nk + e] : 0.f;
    }
  }
  const int col8 = tid & (CPK - 1);  // this thread's 16-B chunk column inside a k tile

  // Operand loads are raw buffer loads: the descriptor's num_records bounds-check returns zeros
  // for an out-of-range offset, so conv padding, the M / K tails and the channel tail need no
  // branches (a per-element "load or zero" select makes hipcc branch and drain vmcnt per load,
  // cdna_hip_programming.md §5 item 4(c)).  OOB = an offset past the end of the tensor.
  const uint32_t x_bytes = (uint32_t)(((size_t)p.Nb * (D3 ? p.T : 1) * p.H * p.W * p.ldx - grp * p.gx) * 2);
  const uint32_t w_bytes = (uint32_t)((size_t)p.K * p.ldw * 2);
  const __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc((void*)p.x, 0, (int)x_bytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t wr = __builtin_amdgcn_make_buffer_rsrc((void*)p.w, 0, (int)w_bytes, 0x00020000);
  constexpr uint32_t OOB = 0xFFFFFFF0u;
  // AT: the BN input rides along with the A operand (same offsets); coefficient tiles [3][BK] for
  // two k-tiles in flight (slot = LDS stage of the tile)
  const __amdgpu_buffer_rsrc_t axr =
      __builtin_amdgcn_make_buffer_rsrc((void*)(AT ? p.ax : p.x), 0, (int)x_bytes, 0x00020000);
  __shared__ __attribute__((aligned(16))) float acf[AT ? 2 : 1][3][AT ? BK : 4];

  // per-row gather state for the activation rows this thread stages
  int a_img[A_CHUNKS], a_h[A_CHUNKS], a_w[A_CHUNKS];
  int a_t[D3 ? A_CHUNKS : 1];  // 3-D: first input frame of the row's window (may be < 0: padding)
  // a pointwise stride-1 conv reads input pixel m for output pixel m: skip the (n, p, q) split
  const bool pw_direct = PW && p.sh == 1 && p.sw == 1;
#pragma unroll
  for (int i = 0; i < A_CHUNKS; ++i) {
    int m = m0 + tid / CPK + RPS * i;
    if constexpr (D3) a_t[i] = -(1 << 28);
    if (pw_direct) {
      a_img[i] = m < p.M ? m : -1;
      a_h[i] = 0;
      a_w[i] = 0;
    } else if (m < p.M) {
      int n = m / (p.P * p.Q);
      int pq = m - n * p.P * p.Q;
      int pp = pq / p.Q, qq = pq - pp * p.Q;
      if constexpr (D3) {
        const int img = n;  // (sample, output frame)
        n = img / p.To;
        a_t[i] = (img - n * p.To) * p.st - p.pt;
        a_img[i] = n * p.T * p.H * p.W;
      } else {
        a_img[i] = n * p.H * p.W;
      }
      a_h[i] = pp * p.sh - p.ph;
      a_w[i] = qq * p.sw - p.pw;
    } else {
      a_img[i] = -1;
      a_h[i] = -(1 << 28);
      a_w[i] = 0;
    }
  }
  uint32_t b_row[B_CHUNKS];
#pragma unroll
  for (int i = 0; i < B_CHUNKS; ++i) {
    const int n = n0 + tid / CPK + RPS * i;
    b_row[i] = n < p.K ? (uint32_t)n * (uint32_t)p.ldw * 2u : 0x80000000u;  // + any k stays out of range
  }

  const int KT = (p.Kg + BK - 1) / BK;

  // FAST-path per-row state: base element offset of the (r=0, s=0) tap and its tap-validity mask
  int rbase[A_CHUNKS];
  uint64_t vmask[A_CHUNKS];
  if constexpr (FAST) {
#pragma unroll
    for (int i = 0; i < A_CHUNKS; ++i) {
      if constexpr (D3) rbase[i] = ((a_img[i] + (a_t[i] * p.H + a_h[i]) * p.W + a_w[i]) * p.ldx) + col8 * 8;
      else rbase[i] = ((a_img[i] + a_h[i] * p.W + a_w[i]) * p.ldx) + col8 * 8;
      uint64_t msk = 0;
      if (PW) {
        msk = a_img[i] >= 0 ? 1ull : 0ull;
      } else if (a_img[i] >= 0) {
        for (int d = 0; d < (D3 ? p.KT : 1); ++d) {
          if constexpr (D3) {
            if ((unsigned)(a_t[i] + d * p.dtd) >= (unsigned)p.T) continue;
          }
          for (int r = 0; r < p.R; ++r) {
            const int h = a_h[i] + r * p.dh;
            if ((unsigned)h >= (unsigned)p.H) continue;
            for (int sx = 0; sx < p.S; ++sx) {
              const int w = a_w[i] + sx * p.dw;
              if ((unsigned)w < (unsigned)p.W) msk |= 1ull << ((d * p.R + r) * p.S + sx);
            }
          }
        }
      }
      vmask[i] = msk;
    }
  }

  // ``live`` = false issues the same loads with out-of-range offsets (they return zeros and touch no
  // memory): keeping every load unconditional keeps hipcc's vmcnt counting exact — a conditionally
  // issued group makes it wait as if the group were absent, draining the pipeline every k-tile.
  // FAST-path k-tile iterator (wave-uniform, scalar registers): live tiles are requested in
  // increasing order, so the (tap, channel) position advances by BK per live call instead of two
  // scalar divisions per k-tile (the round-1 PMC showed ~2.5 SALU per MFMA from them).
  int it_c0 = 0, it_s = 0, it_tap = 0, it_off = 0;  // channel in tap, s, tap index, element offset
  int it_r = 0;                                       // 3-D: filter row inside the depth tap
  auto load_tile = [&](int kt, bool live, uint4 (&ra)[A_CHUNKS], uint4 (&rb)[B_CHUNKS]) {
    const uint32_t dead = live ? 0u : 0x80000000u;
    if constexpr (FAST) {
      const int kb = live ? kt * BK : 0;      // wave-uniform
      const int tap = (PW || !live) ? 0 : it_tap;  // a dead call's offsets are forced out of range below
      const int cl = PW ? kb : it_c0;  // logical channel of the tile (cdup: the duplicated part re-reads hi)
      const int tap_off = (PW ? 0 : it_off) + ((p.cdup && cl >= p.cdup) ? cl - p.cdup : cl);
      if (!PW && live) {
        it_c0 += BK;
        if (it_c0 == p.C) {
          it_c0 = 0;
          ++it_tap;
          if (++it_s == p.S) {
            it_s = 0;
            if (D3 && ++it_r == p.R) {  // next depth tap: back to row 0, column 0, one frame on
              it_r = 0;
              it_off += (p.dtd * p.H * p.W - (p.R - 1) * p.dh * p.W - (p.S - 1) * p.dw) * p.ldx;
            } else {
              it_off += (p.dh * p.W - (p.S - 1) * p.dw) * p.ldx;
            }
          } else {
            it_off += p.dw * p.ldx;
          }
        }
      }
#pragma unroll
      for (int i = 0; i < A_CHUNKS; ++i) {
        const bool ok = PW ? (vmask[i] != 0) : ((vmask[i] >> tap) & 1ull);
        const uint32_t off = (ok ? (uint32_t)(rbase[i] + tap_off) * 2u : OOB) | dead;
        ra[i] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(xr, off, 0, 0));
      }
#pragma unroll
      for (int i = 0; i < B_CHUNKS; ++i) {
        const uint32_t off = (b_row[i] + (uint32_t)(kb + col8 * 8) * 2u) | dead;  // OOB rows stay out of range
        rb[i] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(wr, off, 0, 0));
      }
    } else if constexpr (MODE == 2) {
      const int k = kt * BK + col8 * 8;
      const bool kin0 = live && k < p.Kg, kin1 = live && k + 4 < p.Kg;
      const int t0 = k >> 2;
      int r0 = t0 / p.S, s0 = t0 - (t0 / p.S) * p.S;
      int r1 = r0, s1 = s0 + 1;
      if (s1 == p.S) { s1 = 0; ++r1; }
#pragma unroll
      for (int i = 0; i < A_CHUNKS; ++i) {
        const int h0 = a_h[i] + r0 * p.dh, w0 = a_w[i] + s0 * p.dw;
        const int h1 = a_h[i] + r1 * p.dh, w1 = a_w[i] + s1 * p.dw;
        const bool ok0 = kin0 && (unsigned)h0 < (unsigned)p.H && (unsigned)w0 < (unsigned)p.W;
        const bool ok1 = kin1 && (unsigned)h1 < (unsigned)p.H && (unsigned)w1 < (unsigned)p.W;
        const uint32_t off0 = ok0 ? (uint32_t)((a_img[i] + h0 * p.W + w0) * 4) * 2u : OOB;
        const uint32_t off1 = ok1 ? (uint32_t)((a_img[i] + h1 * p.W + w1) * 4) * 2u : OOB;
        const uint2 lo = __builtin_bit_cast(uint2, __builtin_amdgcn_raw_buffer_load_b64(xr, off0, 0, 0));
        const uint2 hi = __builtin_bit_cast(uint2, __builtin_amdgcn_raw_buffer_load_b64(xr, off1, 0, 0));
        ra[i] = make_uint4(lo.x, lo.y, hi.x, hi.y);
      }
      const bool kw = live && k < p.ldw;
#pragma unroll
      for (int i = 0; i < B_CHUNKS; ++i) {
        const uint32_t off = kw && b_row[i] != OOB ? b_row[i] + (uint32_t)k * 2u : OOB;
        rb[i] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(wr, off, 0, 0));
      }
    } else {
      const int k = kt * BK + col8 * 8;
      int tap = 0, c = k, r = 0, sx = 0, d = 0;
      const bool kin = live && k < p.Kg;
      if (kin) {
        tap = k / p.C;
        c = k - tap * p.C;
        if (p.cdup && c >= p.cdup) c -= p.cdup;
        if constexpr (D3) {
          d = tap / (p.R * p.S);
          tap -= d * p.R * p.S;
        }
        r = tap / p.S;
        sx = tap - r * p.S;
      }
#pragma unroll
      for (int i = 0; i < A_CHUNKS; ++i) {
        const int h = a_h[i] + r * p.dh, w = a_w[i] + sx * p.dw;
        bool ok = kin && (unsigned)h < (unsigned)p.H && (unsigned)w < (unsigned)p.W;
        int pix = a_img[i] + h * p.W + w;
        if constexpr (D3) {
          const int tt = a_t[i] + d * p.dtd;
          ok = ok && (unsigned)tt < (unsigned)p.T;
          pix += tt * p.H * p.W;
        }
        const uint32_t off = ok ? (uint32_t)(pix * p.ldx + c) * 2u : OOB;
        ra[i] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(xr, off, 0, 0));
      }
#pragma unroll
      for (int i = 0; i < B_CHUNKS; ++i) {
        const uint32_t off = kin && b_row[i] != OOB ? b_row[i] + (uint32_t)k * 2u : OOB;
        rb[i] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(wr, off, 0, 0));
      }
    }
  };
  // AT: BN-input chunks at the A offsets (issued unconditionally like the A loads) and one float4 of
  // the k-tile's coefficients for the first 3·BK/4 threads
  auto load_aux = [&](int kt, bool live, uint4 (&xa)[A_CHUNKS], float4& cf) {
    if constexpr (AT) {
      const uint32_t dead = live ? 0u : 0x80000000u;
      const int kb = live ? kt * BK : 0;
#pragma unroll
      for (int i = 0; i < A_CHUNKS; ++i) {
        const uint32_t off = (vmask[i] != 0 ? (uint32_t)(rbase[i] + kb) * 2u : OOB) | dead;
        xa[i] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(axr, off, 0, 0));
      }
      if (tid < 3 * BK / 4) {
        const int arr = tid / (BK / 4), q = tid - arr * (BK / 4);
        cf = live ? *reinterpret_cast<const float4*>(p.acoef + (size_t)arr * p.C + kb + 4 * q)
                  : make_float4(0.f, 0.f, 0.f, 0.f);
      }
    }
  };
  // AT: rewrite the A chunks as the BN input gradient (zero for rows past M), then stage as usual;
  // also park the NEXT k-tile's coefficients in the other slot (read after the next barrier)
  auto transform_a = [&](int buf, uint4 (&ra)[A_CHUNKS], const uint4 (&xa)[A_CHUNKS], const float4& cfn) {
    if constexpr (AT) {
      float Av[8], Bv[8], Cv[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        Av[e] = acf[buf][0][col8 * 8 + e];
        Bv[e] = acf[buf][1][col8 * 8 + e];
        Cv[e] = acf[buf][2][col8 * 8 + e];
      }
#pragma unroll
      for (int i = 0; i < A_CHUNKS; ++i) {
        float g[8], xv[8], o[8];
        unpack8(ra[i], g);
        unpack8(xa[i], xv);
#pragma unroll
        for (int e = 0; e < 8; ++e) o[e] = vmask[i] != 0 ? fmaf(Av[e], g[e], fmaf(Bv[e], xv[e], Cv[e])) : 0.f;
        uint32_t w4[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) w4[e] = (uint32_t)f2bf(o[2 * e]) | ((uint32_t)f2bf(o[2 * e + 1]) << 16);
        ra[i] = make_uint4(w4[0], w4[1], w4[2], w4[3]);
      }
      if (tid < 3 * BK / 4) {
        const int arr = tid / (BK / 4), q = tid - arr * (BK / 4);
        *reinterpret_cast<float4*>(&acf[buf ^ 1][arr][4 * q]) = cfn;
      }
    }
  };

  auto store_tile = [&](int buf, const uint4 (&ra)[A_CHUNKS], const uint4 (&rb)[B_CHUNKS]) {
#pragma unroll
    for (int i = 0; i < A_CHUNKS; ++i) {
      int row = tid / CPK + RPS * i;
      *reinterpret_cast<uint4*>(&lds[buf * STAGE + swz<BK>(row, col8)]) = ra[i];
    }
#pragma unroll
    for (int i = 0; i < B_CHUNKS; ++i) {
      int row = BM + tid / CPK + RPS * i;
      *reinterpret_cast<uint4*>(&lds[buf * STAGE + swz<BK>(row, col8)]) = rb[i];
    }
  };

  v4f acc[TN][TM];
#pragma unroll
  for (int i = 0; i < TN; ++i)
#pragma unroll
    for (int j = 0; j < TM; ++j) acc[i][j] = v4f{0.f, 0.f, 0.f, 0.f};

  const int fr = lane & 15, fq = lane >> 4;
  auto compute = [&](int buf) {
#if BIGDL_CONV_SETPRIO
    __builtin_amdgcn_s_setprio(1);
#endif
#pragma unroll
    for (int kk = 0; kk < BK / 32; ++kk) {
      const int chunk = kk * 4 + fq;
      v8s af[TN], bfr[TM];
#pragma unroll
      for (int i = 0; i < TN; ++i) {
        int row = BM + wave_n * (BN / 2) + i * 16 + fr;
        af[i] = *reinterpret_cast<const v8s*>(&lds[buf * STAGE + swz<BK>(row, chunk)]);
      }
#pragma unroll
      for (int j = 0; j < TM; ++j) {
        int row = wave_m * (BM / 2) + j * 16 + fr;
        bfr[j] = *reinterpret_cast<const v8s*>(&lds[buf * STAGE + swz<BK>(row, chunk)]);
      }
#pragma unroll
      for (int i = 0; i < TN; ++i)
#pragma unroll
        for (int j = 0; j < TM; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
    }
#if BIGDL_CONV_SETPRIO
    __builtin_amdgcn_s_setprio(0);
#endif
  };

  // Two register sets, loads issued two k-tiles ahead of their use: tile t+2 is requested while
  // tile t is multiplied and is written to LDS only after tile t+1's MFMAs, so HBM / L2 latency
  // hides under two compute phases (one barrier per k-tile; the loop is unrolled by two so both
  // register sets stay statically indexed — runtime-indexed vectors would go to scratch).
  uint4 ra0[A_CHUNKS], rb0[B_CHUNKS], ra1[A_CHUNKS], rb1[B_CHUNKS];
  uint4 xa0[AT ? A_CHUNKS : 1], xa1[AT ? A_CHUNKS : 1];
  float4 cf0 = make_float4(0.f, 0.f, 0.f, 0.f), cf1 = cf0;
  load_tile(0, true, ra0, rb0);
  if constexpr (AT) load_aux(0, true, xa0, cf0);
  load_tile(1, KT > 1, ra1, rb1);
  if constexpr (AT) {
    load_aux(1, KT > 1, xa1, cf1);
    if (tid < 3 * BK / 4) {  // tile 0's coefficients → slot 0 before the first transform
      const int arr = tid / (BK / 4), q = tid - arr * (BK / 4);
      *reinterpret_cast<float4*>(&acf[0][arr][4 * q]) = cf0;
    }
    __syncthreads();
    transform_a(0, ra0, xa0, cf1);
  }
  store_tile(0, ra0, rb0);
  __syncthreads();
  int kt = 0;
  for (; kt + 2 <= KT; kt += 2) {
    // lds[0] = tile kt; set 1 = tile kt+1 (in flight)
    load_tile(kt + 2, kt + 2 < KT, ra0, rb0);
    if constexpr (AT) load_aux(kt + 2, kt + 2 < KT, xa0, cf0);
    compute(0);
    if constexpr (AT) transform_a(1, ra1, xa1, cf0);
    store_tile(1, ra1, rb1);
    __syncthreads();
    load_tile(kt + 3, kt + 3 < KT, ra1, rb1);
    if constexpr (AT) load_aux(kt + 3, kt + 3 < KT, xa1, cf1);
    compute(1);
    if (kt + 2 < KT) {
      if constexpr (AT) transform_a(0, ra0, xa0, cf1);
      store_tile(0, ra0, rb0);
    }
    __syncthreads();
  }
  if (kt < KT) {  // odd KT: the last tile sits in lds[0]
    compute(0);
    __syncthreads();
  }

  if (p.y32) {  // fp32 output (uniform branch): 4 consecutive channels of one pixel per accumulator
    if (p.stats && !p.bnx32) {
      // BN statistics of the fp32 output (the fp32-compute conv → BN case; host-checked: no bias, ReLU or
      // residual, replicated atomic sums): shifted by the prefetched running mean, summed over the lane's
      // TM pixels, folded over the 16 pixel lanes of a DPP row, then one atomic per wave and channel into
      // replica tm % R (ConvParams::stats_atomic)
#pragma unroll
      for (int i = 0; i < TN; ++i) {
        float s4[4] = {0.f, 0.f, 0.f, 0.f}, q4[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int j = 0; j < TM; ++j) {
          const float live = (m0 + wave_m * (BM / 2) + j * 16 + fr < p.M) ? 1.f : 0.f;
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const float a = live * (acc[i][j][e] - kpre[i][e]);
            s4[e] += a;
            q4[e] = fmaf(a, a, q4[e]);
          }
        }
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          s4[e] += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(s4[e]), 0x128, 0xF, 0xF, false));
          q4[e] += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(q4[e]), 0x128, 0xF, 0xF, false));
          s4[e] += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(s4[e]), 0x124, 0xF, 0xF, false));
          q4[e] += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(q4[e]), 0x124, 0xF, 0xF, false));
          s4[e] += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(s4[e]), 0x122, 0xF, 0xF, false));
          q4[e] += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(q4[e]), 0x122, 0xF, 0xF, false));
          s4[e] += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(s4[e]), 0x121, 0xF, 0xF, false));
          q4[e] += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(q4[e]), 0x121, 0xF, 0xF, false));
        }
        const int n = n0 + wave_n * (BN / 2) + i * 16 + fq * 4;
        if (fr == 0 && n < p.K) {
          const int rep = tm % p.stats_atomic;
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            atomicAdd(&p.stats[(size_t)rep * p.K + n + e], s4[e]);
            atomicAdd(&p.stats[((size_t)p.stats_atomic + rep) * p.K + n + e], q4[e]);
          }
        }
      }
    }
#pragma unroll
    for (int i = 0; i < TN; ++i) {
      const int n = n0 + wave_n * (BN / 2) + i * 16 + fq * 4;
      if (n >= p.K) continue;  // K % 4 == 0 (host-checked): a 4-channel group is all in or all out
      // fp32 BN backward (p.bnx32): Σg', Σg'·(x − μ) of the stored gradient masked by the BN's ReLU
      float gs[4] = {0.f, 0.f, 0.f, 0.f}, gq[4] = {0.f, 0.f, 0.f, 0.f}, mu[4] = {0.f, 0.f, 0.f, 0.f};
      float sc4[4] = {0.f, 0.f, 0.f, 0.f}, sh4[4] = {0.f, 0.f, 0.f, 0.f};
      if (p.bnx32) {
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          mu[e] = p.bn_mean[n + e];
          if (!p.bn_bits && p.bn_sc) { sc4[e] = p.bn_sc[n + e]; sh4[e] = p.bn_sh[n + e]; }
        }
      }
      float b4[4] = {0.f, 0.f, 0.f, 0.f};
      if (p.bias) {
#pragma unroll
        for (int e = 0; e < 4; ++e) b4[e] = p.bias[n + e];
      }
#pragma unroll
      for (int j = 0; j < TM; ++j) {
        const int m = m0 + wave_m * (BM / 2) + j * 16 + fr;
        if (m >= p.M) continue;
        float4 v = make_float4(acc[i][j][0] + b4[0], acc[i][j][1] + b4[1], acc[i][j][2] + b4[2], acc[i][j][3] + b4[3]);
        if (p.res32) {
          const float4 r = *reinterpret_cast<const float4*>(p.res32 + (size_t)m * p.ldy + n);
          v = make_float4(v.x + r.x, v.y + r.y, v.z + r.z, v.w + r.w);
        }
        if (p.relu) v = make_float4(fmaxf(v.x, 0.f), fmaxf(v.y, 0.f), fmaxf(v.z, 0.f), fmaxf(v.w, 0.f));
        if (p.bnx32) {  // the stored gradient is the ReLU-masked g' (the BN backward's and the shortcut's input)
          const float4 xv = *reinterpret_cast<const float4*>(p.bnx32 + (size_t)m * p.K + n);
          const float xa[4] = {xv.x, xv.y, xv.z, xv.w}, va[4] = {v.x, v.y, v.z, v.w};
          unsigned mb = 0xFu;
          if (p.bn_bits) {
            mb = (p.bn_bits[(size_t)m * (p.K >> 3) + (n >> 3)] >> (n & 7)) & 0xFu;
          } else if (p.bn_sc) {
            mb = 0;
#pragma unroll
            for (int e = 0; e < 4; ++e) mb |= (fmaf(xa[e], sc4[e], sh4[e]) > 0.f ? 1u : 0u) << e;
          }
          float ga[4];
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            ga[e] = (mb >> e) & 1u ? va[e] : 0.f;
            gs[e] += ga[e];
            gq[e] = fmaf(ga[e], xa[e] - mu[e], gq[e]);
          }
          v = make_float4(ga[0], ga[1], ga[2], ga[3]);
        }
        *reinterpret_cast<float4*>(p.y32 + (size_t)m * p.ldy + n) = v;
      }
      if (p.bnx32) {  // fold the 16 pixel lanes of the DPP row, one atomic per wave and channel
#pragma unroll
        for (int e = 0; e < 4; ++e) {
#define BIGDL_ROW_FOLD(CTL)                                                                              \
  gs[e] += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(gs[e]), CTL, 0xF, 0xF, false));     \
  gq[e] += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(gq[e]), CTL, 0xF, 0xF, false));
          BIGDL_ROW_FOLD(0x128)
          BIGDL_ROW_FOLD(0x124)
          BIGDL_ROW_FOLD(0x122)
          BIGDL_ROW_FOLD(0x121)
#undef BIGDL_ROW_FOLD
        }
        if (fr == 0) {
          const int rep = tm % p.stats_atomic;
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            atomicAdd(&p.stats[(size_t)rep * p.K + n + e], gs[e]);
            atomicAdd(&p.stats[((size_t)p.stats_atomic + rep) * p.K + n + e], gq[e]);
          }
        }
      }
    }
    return;
  }

  // Epilogue, staged through LDS so every global access is a full 16-B chunk of a pixel row:
  //  1. each lane parks its 4-channel fragments (+bias) as bf16 in a [BM][BN+8] tile (the +8 pad
  //     spreads the 16 pixel rows a ds_write_b64 covers over distinct banks);
  //  2. the block walks the tile row-major, 8 channels per thread: optional residual add (same
  //     16-B chunk of `res`), ReLU, one global_store_dwordx4, and optional per-channel Σy / Σy²
  //     partials for a following BatchNormalization (the conv then replaces the BN stats pass).
  // Staging layout: rows of BN bf16 (no pad); the 16-B chunk c of row r lives at chunk c ^ (r & CMASK).
  // A fragment write (16 rows × one 8-B half-chunk) lands in 16 distinct chunk slots (at most 2-way
  // bank conflicts), and the store loop reads every chunk back with ONE ds_read_b128 — the 8-B-unit
  // swizzle this replaces needed a compare and four selects per chunk to undo odd-row swaps.
  constexpr int LDR = BN;
  constexpr int CMASK = (BN / 8 - 1) & 15;
  bf16_t* et = &lds[0];
  // BN statistics straight from the fp32 accumulators (the plain conv → BN case: no bias, residual,
  // ReLU or BN-backward prologue): each lane sums its TM pixels per channel, two DPP row rotations
  // fold the 16 pixel lanes of a row to 4, and lanes fr < 4 park [2 wave_m × 4] partials per channel
  // in LDS behind the staging tile — ~2 VALU per output instead of unpack + 4 per output in the
  // store loop (round-2 PMC: the expand 1×1 convs issued 8.7 VALU per MFMA, mostly here).
  constexpr int SRED = 8;
  const bool rstats = (BM == SBM) && p.stats && !p.res && !p.relu && !p.bnx && !p.bias && !p.scatter;
  float* red8 = reinterpret_cast<float*>(&et[BM * LDR]);  // [2][SRED][BN]: Σ then Σ²
  if (rstats) {
#pragma unroll
    for (int i = 0; i < TN; ++i) {
      float s4[4] = {0.f, 0.f, 0.f, 0.f}, q4[4] = {0.f, 0.f, 0.f, 0.f};
      float k4[4] = {kpre[i][0], kpre[i][1], kpre[i][2], kpre[i][3]};
#pragma unroll
      for (int j = 0; j < TM; ++j) {
        // rows past M (the last tile's padding) hold acc = 0 and must stay 0 after the shift
        const float live = (m0 + wave_m * (BM / 2) + j * 16 + fr < p.M) ? 1.f : 0.f;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const float a = fmaf(-live, k4[e], acc[i][j][e]);
          s4[e] += a;
          q4[e] = fmaf(a, a, q4[e]);
        }
      }
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        s4[e] += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(s4[e]), 0x128, 0xF, 0xF, false));
        q4[e] += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(q4[e]), 0x128, 0xF, 0xF, false));
        s4[e] += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(s4[e]), 0x124, 0xF, 0xF, false));
        q4[e] += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(q4[e]), 0x124, 0xF, 0xF, false));
      }
      if (fr < 4) {
        const int nl = wave_n * (BN / 2) + i * 16 + fq * 4;
        const int g = wave_m * 4 + fr;
        *reinterpret_cast<float4*>(&red8[g * BN + nl]) = make_float4(s4[0], s4[1], s4[2], s4[3]);
        *reinterpret_cast<float4*>(&red8[(SRED + g) * BN + nl]) = make_float4(q4[0], q4[1], q4[2], q4[3]);
      }
    }
  }
  if (p.bias) {
#pragma unroll
    for (int i = 0; i < TN; ++i) {
      const int n = n0 + wave_n * (BN / 2) + i * 16 + fq * 4;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float b = (n + e < p.K) ? p.bias[n + e] : 0.f;
#pragma unroll
        for (int j = 0; j < TM; ++j) acc[i][j][e] += b;
      }
    }
  }
#pragma unroll
  for (int i = 0; i < TN; ++i) {
    const int nl = wave_n * (BN / 2) + i * 16 + fq * 4;
#pragma unroll
    for (int j = 0; j < TM; ++j) {
      const int ml = wave_m * (BM / 2) + j * 16 + fr;
      uint32_t lo = (uint32_t)f2bf(acc[i][j][0]) | ((uint32_t)f2bf(acc[i][j][1]) << 16);
      uint32_t hi = (uint32_t)f2bf(acc[i][j][2]) | ((uint32_t)f2bf(acc[i][j][3]) << 16);
      *reinterpret_cast<uint2*>(&et[ml * LDR + (((nl >> 3) ^ (ml & CMASK)) << 3) + (nl & 4)]) = make_uint2(lo, hi);
    }
  }
  __syncthreads();
  conv_store_pass<BM, BN, 256>(p, et, tid, m0, n0, tm, rstats);
}

// Environment pin of a tile parameter (A/B measurements): returns a or b if the variable names one
// of them, else 0 (= use the heuristic).
static int conv_env_override(const char* name, int a, int b) {
  const char* e = getenv(name);
  const int v = e ? atoi(e) : 0;
  return (v == a || v == b) ? v : 0;
}

// Tile choice passed with a launch (0 = the shape heuristic in conv_fwd_launch): the compile phase's
// kernel selection (nn/compiled.py autotune times every candidate per conv geometry and launches
// that conv with the winner).  Valid: BN ∈ {64, 128}, BK ∈ {32, 64}, BM ∈ {128, 256}, BM 256 ⇒ BK 64.
// BK = 1 selects the 32x32x16 / LDS-DMA family (conv_mfma32.hip, k-tile 64): BM × BN ∈ {128 × 128,
// 256 × 64, 256 × 128, 256 × 256}; it needs C % 64 == 0 and falls back to the 16x16x32 family otherwise.
constexpr int kX8 = 1;
static bool tile_ok(int bn, int bk, int bm) {
  if (bk == kX8) return (bm == 128 && bn == 128) || (bm == 256 && (bn == 64 || bn == 128 || bn == 256));
  return !((bn && bn != 64 && bn != 128) || (bk && bk != 32 && bk != 64) || (bm && bm != 128 && bm != 256) ||
           (bm == 256 && bk == 32));
}

BIGDL_EXPORT int bigdl_conv_tile_ok(int bn, int bk, int bm) { return tile_ok(bn, bk, bm) ? 0 : (int)hipErrorInvalidValue; }

template <int BN, int BM, int BK>
static void launch_fwd(int mode, dim3 grid, hipStream_t s, const ConvParams& p) {
  if (mode == 3)
    hipLaunchKernelGGL((k_conv_fwd<BN, 3, BM, BK>), grid, dim3(256), 0, s, p);
  else if (mode == 1)
    hipLaunchKernelGGL((k_conv_fwd<BN, 1, BM, BK>), grid, dim3(256), 0, s, p);
  else if (mode == 2)
    hipLaunchKernelGGL((k_conv_fwd<BN, 2, BM, BK>), grid, dim3(256), 0, s, p);
  else
    hipLaunchKernelGGL((k_conv_fwd<BN, 0, BM, BK>), grid, dim3(256), 0, s, p);
}

// Host launchers.  Requirements (checked): C % 8 == 0 (any K; residual / statistics need K % 8), 16-B aligned x/w/y/res.
// ``stats`` (optional) receives 2·G·K floats, G = bigdl_conv_num_row_tiles(Nb·P·Q).
BIGDL_EXPORT int bigdl_conv_num_row_tiles(long long M) { return (int)((M + SBM - 1) / SBM); }

static int conv_fwd_launch(const void* x, const void* w, const float* bias, const void* res, void* y,
                           float* stats, int Nb, int H, int W, int C, int K, int R, int S, int P, int Q,
                           int sh, int sw, int ph, int pw, int dh, int dw, int relu, int osh, int osw,
                           int ooh, int oow, int oH, int oW, const void* bnx, const float* bn_sc,
                           const float* bn_sh, const float* bn_mean, const void* bn_mask, int ldy,
                           hipStream_t s, int ldw = 0, const float* stat_shift = nullptr, int res_sh = 0,
                           int res_sw = 0, int res_H = 0, int res_W = 0, const void* bn_bits = nullptr,
                           int ldx = 0, int groups = 1, const void* ax = nullptr, const float* acoef = nullptr,
                           float* y32 = nullptr, int tile_bn = 0, int tile_bk = 0, int tile_bm = 0,
                           int stats_atomic = 0, const float* res32 = nullptr, int cdup = 0,
                           const float* bnx32 = nullptr, int8_t* yq = nullptr, float yq_scale = 0.f,
                           int yq_u8 = 0) {
  const bool c4 = C == 4;
  if (yq && (y32 || stats || bnx || res || ldy != K || K % 8 || ((uintptr_t)yq & 7) || !(yq_scale > 0.f) ||
             osh != 1 || osw != 1 || ooh != 0 || oow != 0 || oH != P || oW != Q || groups != 1))
    return (int)hipErrorInvalidValue;
  if (cdup && (cdup < 0 || cdup % 8 || 2 * cdup > C || c4 || ax || groups != 1 || !y32)) return (int)hipErrorInvalidValue;
  if (!tile_ok(tile_bn, tile_bk, tile_bm)) return (int)hipErrorInvalidValue;
  if (y32 && (K % 4 || ldy % 4 || ((uintptr_t)y32 & 15) || res || bnx || ax || groups != 1 || osh != 1 ||
              osw != 1 || ooh != 0 || oow != 0 || oH != P || oW != Q))
    return (int)hipErrorInvalidValue;
  // fp32-output statistics: replicated atomic sums only, of the plain conv output
  if (y32 && stats && (stats_atomic <= 0 || bias || relu || (res32 && !bnx32) || ldy != K || tile_bm == 256))
    return (int)hipErrorInvalidValue;
  if (bnx32 && (!y32 || !stats || !bn_mean || ((uintptr_t)bnx32 & 15) || (bn_sc != nullptr) != (bn_sh != nullptr)))
    return (int)hipErrorInvalidValue;
  if (ldx == 0) ldx = C - cdup;
  if (groups < 1 || ldx < C - cdup || (ldx != C && (c4 || ldx % 8 || ((uintptr_t)x & 15)))) return (int)hipErrorInvalidValue;
  // grouped: C / K are per group; x pixels are ldx apart with group g at channel g·C; y rows ldy
  // apart with group g at channel g·K; w holds the groups' [K][R][S][C] blocks back to back
  if (groups > 1 && (c4 || res || stats || bnx || ldx < groups * C || ldy < groups * K || K % 8 ||
                     osh != 1 || osw != 1 || ooh != 0 || oow != 0 || oH != P || oW != Q))
    return (int)hipErrorInvalidValue;
  // any K: partial 8-channel chunks are stored per element in the epilogue
  if ((C % 8 && !c4) || Nb <= 0 || K <= 0) return (int)hipErrorInvalidValue;
  if (c4 && (ldw < R * S * C || ldw % 8 || dh != 1 || dw != 1)) return (int)hipErrorInvalidValue;
  if (!y32 && (ldy < K || (ldy != K && (ldy % 8 || K % 8 || ((uintptr_t)y & 15))))) return (int)hipErrorInvalidValue;
  if (y32 && ldy < K) return (int)hipErrorInvalidValue;
  if ((res || stats) && K % 8) return (int)hipErrorInvalidValue;
  // 32-bit buffer offsets: both operands must stay below 2 GiB
  if (!c4) ldw = R * S * C;
  if ((size_t)Nb * H * W * ldx * 2 >= 0x80000000ull || (size_t)groups * K * ldw * 2 >= 0x80000000ull)
    return (int)hipErrorInvalidValue;
  ConvParams p{};  // value-initialised: a field a launcher forgets is null / 0, never stack garbage
  p.T = p.KT = p.st = p.dtd = p.To = 1;
  p.ldx = ldx;
  p.cdup = cdup;
  p.ax = (const bf16_t*)ax;
  p.acoef = acoef;
  if ((ax != nullptr) != (acoef != nullptr) || (ax && ((uintptr_t)ax & 15))) return (int)hipErrorInvalidValue;
  p.gx = C;
  p.gw = (long long)K * (c4 ? ldw : R * S * C);
  p.gy = K;
  p.x = (const bf16_t*)x;
  p.w = (const bf16_t*)w;
  p.bias = bias;
  p.y = (bf16_t*)y;
  p.y32 = y32;
  if (res32 && (!y32 || ((uintptr_t)res32 & 15))) return (int)hipErrorInvalidValue;
  p.res32 = res32;
  p.bnx32 = bnx32;
  p.res = (const bf16_t*)res;
  p.stats = stats;
  p.stats_atomic = stats ? stats_atomic : 0;
  p.yq = yq;
  p.yq_inv = yq ? 1.f / yq_scale : 0.f;
  p.yq_u8 = yq ? yq_u8 : 0;
  p.res_sh = res ? res_sh : 0;
  p.res_sw = res ? res_sw : 0;
  p.res_H = res_H;
  p.res_W = res_W;
  if (p.res_sh && (p.res_sw <= 0 || res_H * p.res_sh < P || res_W * p.res_sw < Q || res_H <= 0 || res_W <= 0))
    return (int)hipErrorInvalidValue;
  p.stat_shift = stats ? stat_shift : nullptr;
  p.Nb = Nb; p.H = H; p.W = W; p.C = C; p.K = K; p.R = R; p.S = S; p.P = P; p.Q = Q;
  p.sh = sh; p.sw = sw; p.ph = ph; p.pw = pw; p.dh = dh; p.dw = dw;
  long long Ml = (long long)Nb * P * Q;
  if (Ml > 0x7fffffffLL) return (int)hipErrorInvalidValue;
  p.M = (int)Ml;
  p.Kg = R * S * C;
  p.ldw = ldw;
  p.relu = relu;
  p.scatter = (osh != 1 || osw != 1 || ooh != 0 || oow != 0 || oH != P || oW != Q) ? 1 : 0;
  p.osh = osh; p.osw = osw; p.ooh = ooh; p.oow = oow; p.oH = oH; p.oW = oW;
  if (p.scatter && stats) return (int)hipErrorInvalidValue;
  if (p.scatter && p.res_sh) return (int)hipErrorInvalidValue;
  p.ldy = ldy;
  if (ldy != K && (p.scatter || bnx)) return (int)hipErrorInvalidValue;
  p.bnx = (const bf16_t*)bnx;
  p.bn_sc = bn_sc;
  p.bn_sh = bn_sh;
  p.bn_mean = bn_mean;
  p.bn_mask = (const bf16_t*)bn_mask;
  p.bn_bits = (const uint8_t*)bn_bits;
  if (bn_bits && ((!bn_mask && !bnx32) || K % 8)) return (int)hipErrorInvalidValue;
  if (bnx && (!stats || !bn_mean || relu || bias || p.scatter)) return (int)hipErrorInvalidValue;
  if (bnx && !bn_mask && (!bn_sc || !bn_sh || res)) return (int)hipErrorInvalidValue;
  if (bn_mask && !bnx) return (int)hipErrorInvalidValue;
  // the 64 → 64 3×3 stride-1 shape (ResNet-50 stage 1): the persistent halo-patch kernel, whatever
  // tile the launch carries (it stages each input pixel once instead of once per tap)
  if (!ax && !c4 && !cdup && groups == 1 && !yq) {
    const int e = conv_patch_launch(p, s);
    if (e != (int)hipErrorNotSupported) return e;
  }
  // 32x32x16 / LDS-DMA family: pinned by the launch's tile (BK = kX8) or, with no tile given, by
  // BIGDL_CONV_X8=1 (256 × 128 tile; 256 × 64 for K ≤ 64).  Shapes it does not cover (C % 64 != 0,
  // the BN-backward prologue, the C = 4 stem) take the 16x16x32 family with the heuristic tile.
  {
    static const int x8_env = [] { const char* e = getenv("BIGDL_CONV_X8"); return e ? atoi(e) : 0; }();
    int xbn = 0, xbm = 0;
    if (tile_bk == kX8) {
      xbn = tile_bn;
      xbm = tile_bm;
      tile_bn = tile_bk = tile_bm = 0;
    } else if (!tile_bk && !tile_bn && !tile_bm && x8_env) {
      xbm = 256;
      xbn = K <= 64 ? 64 : (x8_env == 2 && K >= 256 ? 256 : 128);  // 2: the 256 × 256 tile where K allows
    }
    if (xbm && !ax && !c4 && !cdup && !yq) {
      const int xmode = (R == 1 && S == 1 && ph == 0 && pw == 0) ? 3 : 1;
      p.tiles_n = (K + xbn - 1) / xbn;
      p.tiles_m = (p.M + SBM - 1) / SBM;
      const long long xt = (long long)((p.M + xbm - 1) / xbm) * p.tiles_n;
      if (conv_x8_ok(xmode, xbm, xbn, p) && xt <= 0x7fffffff && groups == 1)
        return conv_x8_launch(p, xmode, xbm, xbn, dim3((unsigned)xt, (unsigned)groups), s);
    }
  }
  const int bn_env = tile_bn ? tile_bn : conv_env_override("BIGDL_CONV_BN", 64, 128);
  const int BN = bn_env ? bn_env : (K <= 64 ? 64 : 128);
  p.tiles_n = (K + BN - 1) / BN;
  p.tiles_m = (p.M + SBM - 1) / SBM;
  // Tile shape: 128 pixels × BN × BK.  BK = 32 halves the LDS stage (48 KiB incl. the epilogue) and
  // the register prefetch so 3 blocks share a CU; BM = 256 (128 × 64 per wave) trades occupancy for
  // less LDS traffic per MFMA.  BIGDL_CONV_BM / BIGDL_CONV_BK pin a shape for A/B measurements.
  // Measured on the ResNet-50 shapes (profiles/r1_conv_bk_ab.txt): BK = 32 wins on every reduction
  // of ≤ 512 (the 1×1 convs; more blocks in flight hide the short k-loop's prologue/epilogue),
  // BK = 64 on the deeper ones (3×3, C ≥ 1024).
  const int bk_env = tile_bk ? tile_bk : conv_env_override("BIGDL_CONV_BK", 32, 64);
  // (The 3×3 convs with Kg ≤ 1152 run 3–5 % faster alone at BK = 32 — profiles/r2_conv3x3_tile_ab.txt —
  // but the whole step, with wgrad overlapping on a side stream, measured 23.5 vs 23.1 ms: kept at 64.)
  int bk = bk_env ? bk_env : (p.Kg <= 512 ? 32 : 64);
  // a channel count that is a multiple of 32 but not 64 (Inception's 96 / 480 / 528-style reductions)
  // keeps the tap-uniform FAST path at BK = 32 instead of the per-chunk generic gather at BK = 64
  if (!bk_env && bk == 64 && C % 64 != 0 && C % 32 == 0) bk = 32;
  const int bm = tile_bm ? tile_bm
                          : (conv_env_override("BIGDL_CONV_BM", 128, 256) ? conv_env_override("BIGDL_CONV_BM", 128, 256) : 128);
  if (!bk_env && bk == 64 && cdup % 64 != 0 && cdup % 32 == 0) bk = 32;
  // the tap-uniform gather maps a whole k-tile through cdup: a tile must not straddle a part boundary
  const bool fast = (C % bk == 0) && R * S <= 64 && cdup % bk == 0;
  const int mode = c4 ? 2 : (fast && R == 1 && S == 1 && ph == 0 && pw == 0 ? 3 : (fast ? 1 : 0));
  if (ax && (mode != 3 || groups != 1 || bm != 128)) return (int)hipErrorInvalidValue;  // prologue: pointwise only
  long long tiles = (long long)((p.M + bm - 1) / bm) * p.tiles_n;
  if (tiles > 0x7fffffff || groups > 65535) return (int)hipErrorInvalidValue;
  const dim3 g((unsigned)tiles, (unsigned)groups);
  if (ax) {
    if (bk == 32) {
      if (BN == 64) hipLaunchKernelGGL((k_conv_fwd<64, 3, 128, 32, false, true>), g, dim3(256), 0, s, p);
      else hipLaunchKernelGGL((k_conv_fwd<128, 3, 128, 32, false, true>), g, dim3(256), 0, s, p);
    } else {
      if (BN == 64) hipLaunchKernelGGL((k_conv_fwd<64, 3, 128, 64, false, true>), g, dim3(256), 0, s, p);
      else hipLaunchKernelGGL((k_conv_fwd<128, 3, 128, 64, false, true>), g, dim3(256), 0, s, p);
    }
    BIGDL_CHECK_LAUNCH();
  }
  if (bm == 256)
    BN == 64 ? launch_fwd<64, 256, 64>(mode, g, s, p) : launch_fwd<128, 256, 64>(mode, g, s, p);
  else if (bk == 32)
    BN == 64 ? launch_fwd<64, 128, 32>(mode, g, s, p) : launch_fwd<128, 128, 32>(mode, g, s, p);
  else
    BN == 64 ? launch_fwd<64, 128, 64>(mode, g, s, p) : launch_fwd<128, 128, 64>(mode, g, s, p);
  BIGDL_CHECK_LAUNCH();
}

BIGDL_EXPORT int bigdl_conv_fwd_full(const void* x, const void* w, const float* bias, const void* res, void* y,
                                     float* stats, int Nb, int H, int W, int C, int K, int R, int S, int P, int Q,
                                     int sh, int sw, int ph, int pw, int dh, int dw, int relu, int osh, int osw,
                                     int ooh, int oow, int oH, int oW, const void* bnx, const float* bn_sc,
                                     const float* bn_sh, const float* bn_mean, const void* bn_mask, int tbn,
                                     int tbk, int tbm, hipStream_t s) {
  return conv_fwd_launch(x, w, bias, res, y, stats, Nb, H, W, C, K, R, S, P, Q, sh, sw, ph, pw, dh, dw, relu, osh,
                         osw, ooh, oow, oH, oW, bnx, bn_sc, bn_sh, bn_mean, bn_mask, K, s, 0, nullptr, 0, 0, 0, 0,
                         nullptr, 0, 1, nullptr, nullptr, nullptr, tbn, tbk, tbm);
}

// bigdl_conv_fwd_full2 with the statistics mode (stats_atomic: 1 = the partial sums are ADDED into
// stats[2][K], see ConvParams::stats_atomic) — the dgrad + BN-backward-prologue launch of the fused
// ResNet path.
BIGDL_EXPORT int bigdl_conv_fwd_bnbwd(const void* x, const void* w, const void* res, void* y, float* stats,
                                      int stats_atomic, int Nb, int H, int W, int C, int K, int R, int S, int P, int Q,
                                      int sh, int sw, int ph, int pw, int dh, int dw, const void* bnx,
                                      const float* bn_sc, const float* bn_sh, const float* bn_mean,
                                      const void* bn_mask, const void* bn_bits, int res_sh, int res_sw, int res_H,
                                      int res_W, int tbn, int tbk, int tbm, hipStream_t s) {
  if (res_sh < 0 || res_sw < 0 || (res_sh > 0) != (res_sw > 0) || (res_sh && !res)) return (int)hipErrorInvalidValue;
  return conv_fwd_launch(x, w, nullptr, res, y, stats, Nb, H, W, C, K, R, S, P, Q, sh, sw, ph, pw, dh, dw, 0, 1, 1, 0,
                         0, P, Q, bnx, bn_sc, bn_sh, bn_mean, bn_mask, K, s, 0, nullptr, res_sh, res_sw, res_H, res_W,
                         bn_bits, 0, 1, nullptr, nullptr, nullptr, tbn, tbk, tbm, stats_atomic);
}

// bigdl_conv_fwd_full (no bias / ReLU / scatter) with the dgrad extensions: a STRIDED residual
// (res_sh > 0, see ConvParams::res_sh; res is [Nb][res_H][res_W][K]) and/or the block-tail ReLU mask
// as bits (bn_bits, with bn_mask given as the fallback source of the same mask).
BIGDL_EXPORT int bigdl_conv_fwd_full2(const void* x, const void* w, const void* res, void* y, float* stats, int Nb,
                                      int H, int W, int C, int K, int R, int S, int P, int Q, int sh, int sw, int ph,
                                      int pw, int dh, int dw, const void* bnx, const float* bn_sc, const float* bn_sh,
                                      const float* bn_mean, const void* bn_mask, const void* bn_bits, int res_sh,
                                      int res_sw, int res_H, int res_W, int tbn, int tbk, int tbm, hipStream_t s) {
  if (res_sh < 0 || res_sw < 0 || (res_sh > 0) != (res_sw > 0) || (res_sh && !res)) return (int)hipErrorInvalidValue;
  return conv_fwd_launch(x, w, nullptr, res, y, stats, Nb, H, W, C, K, R, S, P, Q, sh, sw, ph, pw, dh, dw, 0, 1, 1, 0,
                         0, P, Q, bnx, bn_sc, bn_sh, bn_mean, bn_mask, K, s, 0, nullptr, res_sh, res_sw, res_H, res_W,
                         bn_bits, 0, 1, nullptr, nullptr, nullptr, tbn, tbk, tbm);
}

// bigdl_conv_fwd_full2 with a BatchNorm-backward prologue on the A operand (pointwise convs: the
// stride-1 backward-data of a 1×1 conv): x is g' (the gradient at a BN output), ax the BN input, acoef
// [3][C] the BN's input-gradient coefficients (gx = A·g' + B·ax + Cc).
BIGDL_EXPORT int bigdl_conv_fwd_full3(const void* x, const void* ax, const float* acoef, const void* w, const void* res,
                                      void* y, float* stats, int Nb, int H, int W, int C, int K, int R, int S, int P,
                                      int Q, int sh, int sw, int ph, int pw, int dh, int dw, const void* bnx,
                                      const float* bn_sc, const float* bn_sh, const float* bn_mean,
                                      const void* bn_mask, const void* bn_bits, int res_sh, int res_sw, int res_H,
                                      int res_W, hipStream_t s) {
  if (!ax || !acoef) return (int)hipErrorInvalidValue;
  if (res_sh < 0 || res_sw < 0 || (res_sh > 0) != (res_sw > 0) || (res_sh && !res)) return (int)hipErrorInvalidValue;
  return conv_fwd_launch(x, w, nullptr, res, y, stats, Nb, H, W, C, K, R, S, P, Q, sh, sw, ph, pw, dh, dw, 0, 1, 1, 0,
                         0, P, Q, bnx, bn_sc, bn_sh, bn_mean, bn_mask, K, s, 0, nullptr, res_sh, res_sw, res_H, res_W,
                         bn_bits, 0, 1, ax, acoef);
}

// Grouped convolution in ONE launch (SpatialConvolution.scala:93-98 nGroup): x [Nb][H][W][ldx] with
// group g's Cg input channels at channel g·Cg, w = groups × [Kg][R][S][Cg], y [Nb][P][Q][ldy] with
// group g's Kg outputs at channel g·Kg; the group is blockIdx.y.  Cg % 8 == 0, Kg % 8 == 0.
BIGDL_EXPORT int bigdl_conv_fwd_grouped(const void* x, const void* w, const float* bias, void* y, int Nb, int H, int W,
                                        int ldx, int Cg, int Kg, int groups, int R, int S, int P, int Q, int sh,
                                        int sw, int ph, int pw, int dh, int dw, int relu, int ldy, hipStream_t s) {
  return conv_fwd_launch(x, w, bias, nullptr, y, nullptr, Nb, H, W, Cg, Kg, R, S, P, Q, sh, sw, ph, pw, dh, dw, relu, 1,
                         1, 0, 0, P, Q, nullptr, nullptr, nullptr, nullptr, nullptr, ldy, s, 0, nullptr, 0, 0, 0, 0,
                         nullptr, ldx, groups);
}

// 3-D convolution (VolumetricConvolution.scala) on the same implicit-GEMM kernel: x [Nb][T][H][W][C],
// w [K][KT][R][S][C], y [Nb][To][P][Q][K] (+ fp32 bias, ReLU).  C % 8 == 0.
BIGDL_EXPORT int bigdl_conv3d_fwd(const void* x, const void* w, const float* bias, void* y, int Nb, int T, int H, int W,
                                  int C, int K, int KT, int R, int S, int To, int P, int Q, int st, int sh, int sw,
                                  int pt, int ph, int pw, int dtd, int dh, int dw, int relu, hipStream_t s) {
  if (C % 8 || Nb <= 0 || K <= 0 || T <= 0 || KT <= 0 || To <= 0 || st <= 0 || dtd <= 0 || R <= 0 || S <= 0)
    return (int)hipErrorInvalidValue;
  if (P <= 0 || Q <= 0) return (int)hipErrorInvalidValue;
  if ((size_t)Nb * T * H * W * C * 2 >= 0x80000000ull || (size_t)K * KT * R * S * C * 2 >= 0x80000000ull ||
      (size_t)Nb * To * P * Q * K * 2 >= 0x80000000ull)
    return (int)hipErrorInvalidValue;
  if (((uintptr_t)x & 15) || ((uintptr_t)w & 15) || ((uintptr_t)y & 15)) return (int)hipErrorInvalidValue;
  ConvParams p{};
  p.x = (const bf16_t*)x; p.w = (const bf16_t*)w; p.bias = bias; p.y = (bf16_t*)y;
  p.Nb = Nb;  // samples; the kernel's row split yields (sample, output frame) pairs from M / (P·Q)
  p.H = H; p.W = W; p.C = C; p.K = K; p.R = R; p.S = S; p.P = P; p.Q = Q;
  p.sh = sh; p.sw = sw; p.ph = ph; p.pw = pw; p.dh = dh; p.dw = dw;
  p.T = T; p.KT = KT; p.st = st; p.pt = pt; p.dtd = dtd; p.To = To;
  p.ldx = C;
  const long long Ml = (long long)Nb * To * P * Q;
  if (Ml > 0x7fffffffLL) return (int)hipErrorInvalidValue;
  p.M = (int)Ml;
  p.Kg = KT * R * S * C;
  p.ldw = p.Kg;
  p.ldy = K;
  p.relu = relu;
  p.osh = p.osw = 1; p.oH = P; p.oW = Q;
  const int BN = K <= 64 ? 64 : 128;
  p.tiles_n = (K + BN - 1) / BN;
  p.tiles_m = (p.M + SBM - 1) / SBM;
  const int bk = p.Kg <= 512 ? 32 : 64;
  const bool fast = C % bk == 0 && KT * R * S <= 64;  // the tap-uniform gather keeps a 64-bit tap mask
  const long long tiles = (long long)((p.M + 127) / 128) * p.tiles_n;
  if (tiles > 0x7fffffff) return (int)hipErrorInvalidValue;
  const dim3 g((unsigned)tiles);
#define BIGDL_C3(BN_, MODE_, BK_) hipLaunchKernelGGL((k_conv_fwd<BN_, MODE_, 128, BK_, true>), g, dim3(256), 0, s, p)
  if (bk == 32) {
    if (fast) { if (BN == 64) BIGDL_C3(64, 1, 32); else BIGDL_C3(128, 1, 32); }
    else { if (BN == 64) BIGDL_C3(64, 0, 32); else BIGDL_C3(128, 0, 32); }
  } else {
    if (fast) { if (BN == 64) BIGDL_C3(64, 1, 64); else BIGDL_C3(128, 1, 64); }
    else { if (BN == 64) BIGDL_C3(64, 0, 64); else BIGDL_C3(128, 0, 64); }
  }
#undef BIGDL_C3
  BIGDL_CHECK_LAUNCH();
}

// Forward conv with an fp32 NHWC output [Nb][P][Q][ldy] (+ fp32 bias, ReLU): the bf16x3 fp32 path
// (precision.hip splits the fp32 operands into bf16 hi / lo parts concatenated along C).  K % 4 == 0.
BIGDL_EXPORT int bigdl_conv_fwd_f32out(const void* x, const void* w, const float* bias, float* y32, int Nb, int H,
                                       int W, int C, int K, int R, int S, int P, int Q, int sh, int sw, int ph, int pw,
                                       int dh, int dw, int relu, int ldy, hipStream_t s) {
  if (!y32) return (int)hipErrorInvalidValue;
  return conv_fwd_launch(x, w, bias, nullptr, nullptr, nullptr, Nb, H, W, C, K, R, S, P, Q, sh, sw, ph, pw, dh, dw,
                         relu, 1, 1, 0, 0, P, Q, nullptr, nullptr, nullptr, nullptr, nullptr, ldy, s, 0, nullptr, 0, 0,
                         0, 0, nullptr, 0, 1, nullptr, nullptr, y32);
}

// bigdl_conv_fwd_f32out + an fp32 residual [M][ldy] summed in the epilogue (res32 16-B aligned)
BIGDL_EXPORT int bigdl_conv_fwd_f32out_res(const void* x, const void* w, const float* bias, const float* res32,
                                           float* y32, int Nb, int H, int W, int C, int K, int R, int S, int P, int Q,
                                           int sh, int sw, int ph, int pw, int dh, int dw, int relu, int ldy,
                                           hipStream_t s) {
  if (!y32 || !res32) return (int)hipErrorInvalidValue;
  return conv_fwd_launch(x, w, bias, nullptr, nullptr, nullptr, Nb, H, W, C, K, R, S, P, Q, sh, sw, ph, pw, dh, dw,
                         relu, 1, 1, 0, 0, P, Q, nullptr, nullptr, nullptr, nullptr, nullptr, ldy, s, 0, nullptr, 0, 0,
                         0, 0, nullptr, 0, 1, nullptr, nullptr, y32, 0, 0, 0, 0, res32);
}

// bigdl_conv_fwd_f32out_res on the two-part bf16x3 activation: x = [Nb][H][W][2·cp] holding [hi | lo],
// read as the 3·cp logical channels [hi | hi | lo] (ConvParams::cdup = cp); C = 3·cp; res32 optional
BIGDL_EXPORT int bigdl_conv_fwd_f32out2(const void* x, const void* w, const float* bias, const float* res32,
                                        float* y32, int Nb, int H, int W, int C, int cdup, int K, int R, int S, int P,
                                        int Q, int sh, int sw, int ph, int pw, int dh, int dw, int relu, int ldy,
                                        hipStream_t s) {
  if (!y32 || cdup <= 0 || C != 3 * cdup) return (int)hipErrorInvalidValue;
  return conv_fwd_launch(x, w, bias, nullptr, nullptr, nullptr, Nb, H, W, C, K, R, S, P, Q, sh, sw, ph, pw, dh, dw,
                         relu, 1, 1, 0, 0, P, Q, nullptr, nullptr, nullptr, nullptr, nullptr, ldy, s, 0, nullptr, 0, 0,
                         0, 0, nullptr, 2 * cdup, 1, nullptr, nullptr, y32, 0, 0, 0, 0, res32, cdup);
}

// bigdl_conv_fwd_f32out2 whose epilogue also ADDS the BN statistics Σ(y − shift), Σ(y − shift)² of its
// fp32 output into R replicas (stats [2][R][K], zero on entry; ConvParams::stats_atomic = R) for the
// following fp32 BN (bigdl_bn32_fwd_train_partials).  No bias / ReLU / residual.
BIGDL_EXPORT int bigdl_conv_fwd_f32out2_stats(const void* x, const void* w, float* y32, float* stats, int R_rep,
                                              const float* shift, int Nb, int H, int W, int C, int cdup, int K, int R,
                                              int S, int P, int Q, int sh, int sw, int ph, int pw, int dh, int dw,
                                              hipStream_t s) {
  if (!y32 || !stats || R_rep <= 0 || cdup <= 0 || C != 3 * cdup || K % 8) return (int)hipErrorInvalidValue;
  static const int bm_env = conv_env_override("BIGDL_CONV_BM", 128, 256);
  if (bm_env == 256) return (int)hipErrorInvalidValue;  // the statistics need 128-row tiles (kpre prefetch)
  return conv_fwd_launch(x, w, nullptr, nullptr, nullptr, stats, Nb, H, W, C, K, R, S, P, Q, sh, sw, ph, pw, dh, dw,
                         0, 1, 1, 0, 0, P, Q, nullptr, nullptr, nullptr, nullptr, nullptr, K, s, 0, shift, 0, 0,
                         0, 0, nullptr, 2 * cdup, 1, nullptr, nullptr, y32, 0, 0, 0, R_rep, nullptr, cdup);
}

// fp32 data gradient (two-part split, as bigdl_conv_fwd_f32out2) whose epilogue also ADDS the BN-backward
// statistics Σg', Σg'·(x − mean) of its output g (after the optional residual) into R replicas of stats
// ([2][R][K], zero on entry): x = bnx32 [M][K] is the BN input, the ReLU mask comes from bits ([M][K/8],
// the forward's mask) or from scale·x + shift > 0 (sc / sh, a BN + ReLU with no residual).
BIGDL_EXPORT int bigdl_conv_fwd_f32out2_bnbwd(const void* x, const void* w, const float* res32, float* y32,
                                              float* stats, int R_rep, const float* bnx32, const float* mean,
                                              const void* bits, const float* sc, const float* sh, int Nb, int H,
                                              int W, int C, int cdup, int K, int R, int S, int P, int Q, int sh_,
                                              int sw_, int ph, int pw, int dh, int dw, hipStream_t s) {
  if (!y32 || !stats || !bnx32 || !mean || R_rep <= 0 || cdup <= 0 || C != 3 * cdup || K % 8 || (!bits && !sc))
    return (int)hipErrorInvalidValue;
  return conv_fwd_launch(x, w, nullptr, nullptr, nullptr, stats, Nb, H, W, C, K, R, S, P, Q, sh_, sw_, ph, pw, dh, dw,
                         0, 1, 1, 0, 0, P, Q, nullptr, sc, sh, mean, nullptr, K, s, 0, nullptr, 0, 0, 0, 0, bits,
                         2 * cdup, 1, nullptr, nullptr, y32, 0, 0, 0, R_rep, res32, cdup, bnx32);
}

// bigdl_conv_fwd_ldy / bigdl_conv_fwd_stats_shift with an explicit tile (bn, bk, bm; 0 = heuristic).
BIGDL_EXPORT int bigdl_conv_fwd_ldy_t(const void* x, const void* w, const float* bias, const void* res, void* y,
                                      float* stats, int Nb, int H, int W, int C, int K, int R, int S, int P, int Q,
                                      int sh, int sw, int ph, int pw, int dh, int dw, int relu, int ldy, int bn, int bk,
                                      int bm, hipStream_t s) {
  return conv_fwd_launch(x, w, bias, res, y, stats, Nb, H, W, C, K, R, S, P, Q, sh, sw, ph, pw, dh, dw, relu, 1, 1, 0,
                         0, P, Q, nullptr, nullptr, nullptr, nullptr, nullptr, ldy, s, 0, nullptr, 0, 0, 0, 0, nullptr,
                         0, 1, nullptr, nullptr, nullptr, bn, bk, bm);
}

BIGDL_EXPORT int bigdl_conv_fwd_stats_shift_t(const void* x, const void* w, const float* bias, void* y, float* stats,
                                              const float* shift, int Nb, int H, int W, int C, int K, int R, int S,
                                              int P, int Q, int sh, int sw, int ph, int pw, int dh, int dw, int bn,
                                              int bk, int bm, int stats_atomic, hipStream_t s) {
  return conv_fwd_launch(x, w, bias, nullptr, y, stats, Nb, H, W, C, K, R, S, P, Q, sh, sw, ph, pw, dh, dw, 0, 1, 1, 0,
                         0, P, Q, nullptr, nullptr, nullptr, nullptr, nullptr, K, s, 0, shift, 0, 0, 0, 0, nullptr, 0,
                         1, nullptr, nullptr, nullptr, bn, bk, bm, stats_atomic);
}

// Forward conv writing rows `ldy` elements apart (a channel slice of a wider NHWC tensor).
BIGDL_EXPORT int bigdl_conv_fwd_ldy(const void* x, const void* w, const float* bias, const void* res, void* y,
                                    float* stats, int Nb, int H, int W, int C, int K, int R, int S, int P, int Q,
                                    int sh, int sw, int ph, int pw, int dh, int dw, int relu, int ldy, hipStream_t s) {
  return conv_fwd_launch(x, w, bias, res, y, stats, Nb, H, W, C, K, R, S, P, Q, sh, sw, ph, pw, dh, dw, relu, 1, 1, 0,
                         0, P, Q, nullptr, nullptr, nullptr, nullptr, nullptr, ldy, s);
}

BIGDL_EXPORT int bigdl_conv_fwd_scatter(const void* x, const void* w, const float* bias, const void* res, void* y,
                                        float* stats, int Nb, int H, int W, int C, int K, int R, int S, int P,
                                        int Q, int sh, int sw, int ph, int pw, int dh, int dw, int relu, int osh,
                                        int osw, int ooh, int oow, int oH, int oW, int tbn, int tbk, int tbm,
                                        hipStream_t s) {
  return bigdl_conv_fwd_full(x, w, bias, res, y, stats, Nb, H, W, C, K, R, S, P, Q, sh, sw, ph, pw, dh, dw, relu, osh,
                             osw, ooh, oow, oH, oW, nullptr, nullptr, nullptr, nullptr, nullptr, tbn, tbk, tbm, s);
}

BIGDL_EXPORT int bigdl_conv_fwd_ex(const void* x, const void* w, const float* bias, const void* res, void* y,
                                   float* stats, int Nb, int H, int W, int C, int K, int R, int S, int P, int Q,
                                   int sh, int sw, int ph, int pw, int dh, int dw, int relu, int tbn, int tbk, int tbm,
                                   hipStream_t s) {
  return bigdl_conv_fwd_scatter(x, w, bias, res, y, stats, Nb, H, W, C, K, R, S, P, Q, sh, sw, ph, pw, dh, dw, relu, 1,
                                1, 0, 0, P, Q, tbn, tbk, tbm, s);
}

BIGDL_EXPORT int bigdl_conv_fwd(const void* x, const void* w, const float* bias, void* y, int Nb, int H, int W, int C,
                                int K, int R, int S, int P, int Q, int sh, int sw, int ph, int pw, int dh, int dw,
                                int relu, hipStream_t s) {
  return bigdl_conv_fwd_ex(x, w, bias, nullptr, y, nullptr, Nb, H, W, C, K, R, S, P, Q, sh, sw, ph, pw, dh, dw, relu,
                           0, 0, 0, s);
}

// Forward conv + shifted BN statistics partials (``shift``: per-output-channel K, see ConvParams).
BIGDL_EXPORT int bigdl_conv_fwd_stats_shift(const void* x, const void* w, const float* bias, void* y, float* stats,
                                            const float* shift, int Nb, int H, int W, int C, int K, int R, int S,
                                            int P, int Q, int sh, int sw, int ph, int pw, int dh, int dw,
                                            hipStream_t s) {
  return conv_fwd_launch(x, w, bias, nullptr, y, stats, Nb, H, W, C, K, R, S, P, Q, sh, sw, ph, pw, dh, dw, 0, 1, 1, 0,
                         0, P, Q, nullptr, nullptr, nullptr, nullptr, nullptr, K, s, 0, shift);
}

BIGDL_EXPORT int bigdl_conv_fwd_c4_stats_shift(const void* x, const void* w, int ldw, const float* bias, void* y,
                                               float* stats, const float* shift, int Nb, int H, int W, int K, int R,
                                               int S, int P, int Q, int sh, int sw, int ph, int pw, int stats_atomic,
                                               hipStream_t s) {
  return conv_fwd_launch(x, w, bias, nullptr, y, stats, Nb, H, W, 4, K, R, S, P, Q, sh, sw, ph, pw, 1, 1, 0, 1, 1, 0,
                         0, P, Q, nullptr, nullptr, nullptr, nullptr, nullptr, K, s, ldw, shift, 0, 0, 0, 0, nullptr, 0, 1,
                         nullptr, nullptr, nullptr, 0, 0, 0, stats_atomic);
}

// 4-channel (RGB-padded) input with weight rows ldw elements apart (ldw % 8 == 0, zero beyond R·S·4).
BIGDL_EXPORT int bigdl_conv_fwd_c4(const void* x, const void* w, int ldw, const float* bias, const void* res, void* y,
                                   float* stats, int Nb, int H, int W, int K, int R, int S, int P, int Q, int sh, int sw,
                                   int ph, int pw, int relu, hipStream_t s) {
  return conv_fwd_launch(x, w, bias, res, y, stats, Nb, H, W, 4, K, R, S, P, Q, sh, sw, ph, pw, 1, 1, relu, 1, 1, 0, 0,
                         P, Q, nullptr, nullptr, nullptr, nullptr, nullptr, K, s, ldw);
}

// The C4 stem with an int8 output (bias, ReLU, then static quantisation with q_scale; u8: the unsigned
// offset code and its 0x80 tail): the calibrated int8 chain's first layer in one pass.
BIGDL_EXPORT int bigdl_conv_fwd_c4_q(const void* x, const void* w, int ldw, const float* bias, void* yq, float q_scale,
                                     int u8, int Nb, int H, int W, int K, int R, int S, int P, int Q, int sh, int sw,
                                     int ph, int pw, int relu, hipStream_t s) {
  if (!yq) return (int)hipErrorInvalidValue;
  return conv_fwd_launch(x, w, bias, nullptr, nullptr, nullptr, Nb, H, W, 4, K, R, S, P, Q, sh, sw, ph, pw, 1, 1, relu,
                         1, 1, 0, 0, P, Q, nullptr, nullptr, nullptr, nullptr, nullptr, K, s, ldw, nullptr, 0, 0, 0, 0,
                         nullptr, 0, 1, nullptr, nullptr, nullptr, 0, 0, 0, 0, nullptr, 0, nullptr, (int8_t*)yq, q_scale,
                         u8);
}

// NHWC channel zero-pad (the RGB stem: 3 → 4 channels, one 8-B store per pixel): dst[p][0:C] = src[p],
// dst[p][C:Cp] = 0.  One thread per pixel; C ≤ Cp ≤ 8.
__global__ void __launch_bounds__(256) k_pad_channels(const bf16_t* __restrict__ src, bf16_t* __restrict__ dst, long long npix,
                                                     int C, int Cp) {
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < npix; i += (long long)gridDim.x * blockDim.x) {
    bf16_t v[8];
#pragma unroll
    for (int c = 0; c < 8; ++c) v[c] = c < C ? src[i * C + c] : (bf16_t)0;
    if (Cp == 4) {
      *reinterpret_cast<uint2*>(dst + i * 4) = make_uint2((uint32_t)v[0] | ((uint32_t)v[1] << 16),
                                                          (uint32_t)v[2] | ((uint32_t)v[3] << 16));
    } else if (Cp == 8) {
      *reinterpret_cast<uint4*>(dst + i * 8) = make_uint4((uint32_t)v[0] | ((uint32_t)v[1] << 16),
                                                          (uint32_t)v[2] | ((uint32_t)v[3] << 16),
                                                          (uint32_t)v[4] | ((uint32_t)v[5] << 16),
                                                          (uint32_t)v[6] | ((uint32_t)v[7] << 16));
    } else {
      for (int c = 0; c < Cp; ++c) dst[i * Cp + c] = v[c];
    }
  }
}

BIGDL_EXPORT int bigdl_pad_channels(const void* src, void* dst, long long npix, int C, int Cp, hipStream_t s) {
  if (npix <= 0 || C <= 0 || C > Cp || Cp > 8) return (int)hipErrorInvalidValue;
  if ((Cp == 4 && ((uintptr_t)dst & 7)) || (Cp == 8 && ((uintptr_t)dst & 15))) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(k_pad_channels, dim3(bigdl_grid(npix, 256, 16384)), dim3(256), 0, s, (const bf16_t*)src,
                     (bf16_t*)dst, npix, C, Cp);
  BIGDL_CHECK_LAUNCH();
}
