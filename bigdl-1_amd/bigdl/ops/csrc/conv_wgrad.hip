// Convolution weight gradient on MFMA (K3): dW[n][k] += scale · Σ_m dY[m][n] · X̂[m][k],
// m = output pixel (N·P·Q), k = (r, s, c) — reference SpatialConvolution.accGradParameters
// (DL/nn/SpatialConvolution.scala:435-505, a per-sample gemm into gradWeight).
//
// Both operands arrive pixel-major (NHWC rows).  Tiles are staged in LDS exactly as loaded
// ([pixel][channel], 16-B chunks) and the MFMA fragments, which need 8 consecutive PIXELS per
// lane, are read with gfx950's ds_read_b64_tr_b16 transposed read (cdna_hip_programming.md T10):
// lane 4q+p of a 16-lane group addresses row q, columns 4p..4p+3 of a 4×16 block and receives
// column (lane) of the 4 rows.  The LDS image is XOR-swizzled on 32-B segments so each 32-lane half
// (8 rows × 32 B) hits all 64 banks exactly once.
// The reduction over pixels is split across blockIdx.y; partial tiles are added straight into the
// fp32 gradient (KRSC, the arena's physical layout) with no-return float atomics (Guideline 12).
#include "common.h"

typedef short v4s __attribute__((ext_vector_type(4)));
typedef short v8s __attribute__((ext_vector_type(8)));
typedef float v4f __attribute__((ext_vector_type(4)));

struct FastDiv {
  uint32_t d, m, s;
};

static FastDiv make_fastdiv(uint32_t d) {
  FastDiv f;
  uint32_t l = 0;
  while ((1ull << l) < d) ++l;
  f.d = d;
  f.m = (uint32_t)((((1ull << 32) * ((1ull << l) - d)) / d) + 1);
  f.s = l;
  return f;
}

__device__ __forceinline__ uint32_t fdiv(uint32_t n, const FastDiv& f) {
  uint32_t t = __umulhi(n, f.m);
  return (t + n) >> f.s;
}

struct WgradParams {
  const bf16_t* x;   // [Nb][H][W][C]
  const bf16_t* dy;  // [Nb][P][Q][K]
  float* dw;         // [K][R][S][C] fp32, accumulated
  float scale;
  int Nb, H, W, C, K, R, S, P, Q, sh, sw, ph, pw, dh, dw_;
  int M, Kg, tiles_k, tiles_n, m_per_split;
  FastDiv fPQ, fQ;
  // 3-D (D3 instantiations): x [Nb][T][H][W][C], dy [Nb][To][P][Q][K], dw [K][KT][R][S][C]
  int T, KT, st, pt, dtd, To;
  FastDiv fRS, fTo;
  // pixel strides of x / dy in elements (C / K unless channel slices of wider tensors) and the
  // grouped-conv per-group offsets (group = blockIdx.z) of x, dy (channels) and dw (elements)
  int ldx, ldk;
  long long gx, gdy, gdw;
  // BatchNorm-backward prologue on dY (AT instantiations): dy is g' at a BN output, dy2 the BN input
  // (same layout), dcoef [3][K]: the kernel uses A·g' + B·dy2 + Cc (the BN input gradient)
  const bf16_t* dy2;
  const float* dcoef;
  // measurement knob only (BIGDL_DEBUG_WGRAD_NO_ATOMICS=1): skip the split-K atomic epilogue, which
  // leaves dW WRONG — an upper bound of what a cheaper cross-split reduction could save
  int skip_epi;
  // 1×1, stride 1, no padding (2-D): X̂ row m is input pixel m — the gather needs no index math
  int pw1;
  // PRO instantiations: [scale | shift] of the BN + ReLU applied to x on load ([2][C])
  const float* pro;
  // 1: the split-K partial tile is staged in LDS (fp32) and added with wave-instructions covering
  // 256 contiguous bytes of a dW row (the fast atomic shape, MI355X_MICROARCH.md 'Global float
  // atomics'); 0: straight from the accumulators (four 64-B row segments per instruction)
  int epi_lds;
};

constexpr int BP = 64;  // split granularity (pixels); the k-tile depth BPT is 64 or 32

// byte offset inside a [BP rows][WIDTH bf16] tile for a 16-B chunk / 8-B quad
template <int WIDTH>
__device__ __forceinline__ int tr_swz_dword(int row, int dword) {
  if constexpr (WIDTH == 128) {
    int seg = (row & 3) | (((row >> 3) & 1) << 2);
    return row * 64 + (dword ^ (seg << 3));
  } else {
    int seg = ((row >> 1) & 1) | (((row >> 3) & 1) << 1);
    return row * 32 + (dword ^ (seg << 3));
  }
}

// C4: 4-channel input (RGB stem padded 3 → 4): an X̂ chunk of 8 k-values is two consecutive taps,
// gathered as two 8-B loads with separate padding tests (see conv_igemm.hip MODE 2).
// F32: fp32 operands (the bf16x3 fp32 compute mode, csrc/precision.hip): each 8-channel chunk is loaded as
// two 16-B fp32 pieces, split in registers into bf16 hi = rne(v) and lo = rne(v − hi) tiles (LDS holds
// both), and every fragment pair feeds three MFMAs (dY_hi·X_hi + dY_lo·X_hi + dY_hi·X_lo) — one launch
// reading 4 B per element instead of three over a materialised [hi | lo] split.
// PRO (F32 only): x is the INPUT of a training BN + ReLU whose (never written) output the conv consumed:
// X̂ = relu(x·pro[c] + pro[C + c]) per loaded chunk, padded taps 0 (ops/fp32x3.py deferred BN).
template <int TILE_N, int TILE_K, int BPT, bool C4 = false, bool D3 = false, bool AT = false, bool PW1 = false,
          bool F32 = false, bool PRO = false>
__global__ void __launch_bounds__(256, BPT == 32 && !AT ? (F32 ? 2 : 3) : 2) k_conv_wgrad(WgradParams p) {
  static_assert(!PRO || (F32 && !C4 && !D3 && !AT), "BN prologue on X: fp32 8-channel chunks only");
  static_assert(!(F32 && (D3 || AT)), "fp32 operands: 2-D, 8-channel (or C4) chunks, no BN prologue");
  static_assert(!(PW1 && (C4 || D3)), "pointwise gather: 2-D, 8-channel chunks");
  static_assert(!(C4 && D3), "3-D wgrad gathers 8-channel chunks");
  static_assert(!(AT && (C4 || D3)), "BN-backward prologue: 2-D, 8-channel chunks");
  constexpr int DY_CH = BPT * TILE_N / 8 / 256;  // 16-B chunks per thread for the dY tile
  constexpr int X_CH = BPT * TILE_K / 8 / 256;   // for the X̂ tile
  constexpr int TMN = TILE_N / 32;              // MFMA tiles per wave along n
  constexpr int TMK = TILE_K / 32;              // along k
  constexpr int DY_WORDS = BPT * TILE_N / 2;     // dwords per tile
  constexpr int X_WORDS = BPT * TILE_K / 2;
  constexpr int LO = DY_WORDS + X_WORDS;          // F32: the lo tiles follow the hi tiles
  constexpr int ES = F32 ? 4 : 2;                 // operand element bytes
  constexpr int PC = F32 ? 2 : 1;                 // 16-B pieces per 8-channel chunk
  __shared__ __attribute__((aligned(16))) uint32_t lds[2][LO * (F32 ? 2 : 1)];

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wave_n = wid & 1, wave_k = wid >> 1;
  const long long grp = blockIdx.z;
  if (grp) {
    p.x += grp * p.gx;
    p.dy += grp * p.gdy;
    p.dw += grp * p.gdw;
  }
  // tile mapping (XCD-contiguous ranges of the tile grid)
  const int nwg = gridDim.x, bid = blockIdx.x;
  const int xcd = bid & 7, qq = nwg >> 3, rr = nwg & 7;
  const int tile = (xcd < rr ? xcd * (qq + 1) : rr * (qq + 1) + (xcd - rr) * qq) + (bid >> 3);
  const int tnI = tile / p.tiles_k, tkI = tile - tnI * p.tiles_k;
  const int n0 = tnI * TILE_N, k0 = tkI * TILE_K;
  const int mbeg = blockIdx.y * p.m_per_split;
  int mend = mbeg + p.m_per_split;
  if (mend > p.M) mend = p.M;
  if (mbeg >= mend) return;

  // this thread's fixed chunk columns
  constexpr int DY_CPR = TILE_N / 8;  // chunks per row
  constexpr int X_CPR = TILE_K / 8;
  const int dy_col = tid % DY_CPR, dy_row0 = tid / DY_CPR;
  const int x_col = tid % X_CPR, x_row0 = tid / X_CPR;
  constexpr int DY_RSTEP = 256 / DY_CPR, X_RSTEP = 256 / X_CPR;
  // X̂ column → (tap, c) once
  const int kx = k0 + x_col * 8;
  const bool kx_ok = kx < p.Kg;
  int tap = kx_ok ? kx / p.C : 0;
  const int cx = kx - tap * p.C;
  int dx = 0;  // 3-D: depth tap of this column
  if constexpr (D3) {
    dx = (int)fdiv((uint32_t)tap, p.fRS);
    tap -= dx * p.R * p.S;
  }
  const int rx = tap / p.S, sx = tap - (tap / p.S) * p.S;
  // C4: the chunk's second tap (tap + 1, wrapping to the next filter row)
  const bool kx1_ok = kx + 4 < p.Kg;
  int rx1 = rx, sx1 = sx + 1;
  if (sx1 == p.S) { sx1 = 0; ++rx1; }
  const int ndy = n0 + dy_col * 8;
  const bool ndy_ok = ndy < p.K;
  float psc[PRO ? 8 : 1], psh[PRO ? 8 : 1];  // PRO: this thread's X̂ column channels cx .. cx + 7
  if constexpr (PRO) {
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      psc[e] = kx_ok ? p.pro[cx + e] : 0.f;
      psh[e] = kx_ok ? p.pro[p.C + cx + e] : 0.f;
    }
  }

  // Raw buffer loads (OOB offsets → zeros, no branches) into two register sets; tile t+2 is
  // requested while tile t is multiplied (loads always issued — beyond the range with a dead
  // offset — so hipcc's vmcnt counts stay exact; see conv_igemm.hip).
  const uint32_t x_bytes = (uint32_t)(((size_t)p.Nb * (D3 ? p.T : 1) * p.H * p.W * p.ldx - grp * p.gx) * ES);
  const uint32_t dy_bytes = (uint32_t)(((size_t)p.M * p.ldk - grp * p.gdy) * ES);
  const __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc((void*)p.x, 0, (int)x_bytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t yr = __builtin_amdgcn_make_buffer_rsrc((void*)p.dy, 0, (int)dy_bytes, 0x00020000);
  constexpr uint32_t DEAD = 0x80000000u;
  const __amdgpu_buffer_rsrc_t y2r =
      __builtin_amdgcn_make_buffer_rsrc((void*)(AT ? p.dy2 : p.dy), 0, (int)dy_bytes, 0x00020000);
  float cA[AT ? 8 : 1], cB[AT ? 8 : 1], cC[AT ? 8 : 1];  // this thread's dY column coefficients
  if constexpr (AT) {
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const bool in = ndy_ok;
      cA[e] = in ? p.dcoef[ndy + e] : 0.f;
      cB[e] = in ? p.dcoef[p.K + ndy + e] : 0.f;
      cC[e] = in ? p.dcoef[2 * p.K + ndy + e] : 0.f;
    }
  }

  auto load = [&](int mt, bool live, uint4 (&rdy)[DY_CH * PC], uint4 (&rx_)[X_CH * PC], uint4 (&r2)[AT ? DY_CH : 1],
                  uint32_t& okm) {
    const uint32_t dead = live ? 0u : DEAD;
    okm = 0;
#pragma unroll
    for (int i = 0; i < DY_CH; ++i) {
      const int m = mt + dy_row0 + i * DY_RSTEP;
      const bool ok = ndy_ok && m < mend;
      const uint32_t off = (ok ? ((uint32_t)m * (uint32_t)p.ldk + (uint32_t)ndy) * (uint32_t)ES : DEAD) | dead;
      rdy[PC * i] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(yr, off, 0, 0));
      if constexpr (F32) rdy[PC * i + 1] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(yr, off + 16u, 0, 0));
      if constexpr (AT) r2[i] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(y2r, off, 0, 0));
    }
    if constexpr (PW1) {  // pointwise: pixel m of the output is pixel m of the input
#pragma unroll
      for (int i = 0; i < X_CH; ++i) {
        const int m = mt + x_row0 + i * X_RSTEP;
        const bool ok = kx_ok && m < mend;
        if (PRO && ok) okm |= 1u << i;
        const uint32_t off = (ok ? ((uint32_t)m * (uint32_t)p.ldx + (uint32_t)cx) * (uint32_t)ES : DEAD) | dead;
        rx_[PC * i] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(xr, off, 0, 0));
        if constexpr (F32) rx_[PC * i + 1] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(xr, off + 16u, 0, 0));
      }
      return;
    }
#pragma unroll
    for (int i = 0; i < X_CH; ++i) {
      const int m = mt + x_row0 + i * X_RSTEP;
      const uint32_t mm = (uint32_t)(m < mend ? m : mbeg);
      uint32_t n = fdiv(mm, p.fPQ);
      const uint32_t pq = mm - n * (uint32_t)(p.P * p.Q);
      const uint32_t pp = fdiv(pq, p.fQ);
      const uint32_t q = pq - pp * (uint32_t)p.Q;
      const int h = (int)pp * p.sh - p.ph + rx * p.dh;
      const int w = (int)q * p.sw - p.pw + sx * p.dw_;
      bool ok = kx_ok && m < mend && (unsigned)h < (unsigned)p.H && (unsigned)w < (unsigned)p.W;
      const uint32_t pq_n = n;
      if constexpr (D3) {  // n = (sample, output frame) → input frame plane index sample·T + t
        const uint32_t ns = fdiv(pq_n, p.fTo);
        const int tt = (int)(pq_n - ns * (uint32_t)p.To) * p.st - p.pt + dx * p.dtd;
        ok = ok && (unsigned)tt < (unsigned)p.T;
        n = ns * (uint32_t)p.T + (uint32_t)(tt < 0 ? 0 : tt);
      }
      if constexpr (C4) {
        const int h1 = (int)pp * p.sh - p.ph + rx1, w1 = (int)q * p.sw - p.pw + sx1;
        const bool ok1 = kx1_ok && m < mend && (unsigned)h1 < (unsigned)p.H && (unsigned)w1 < (unsigned)p.W;
        // one pixel of the 4-channel input: 8 B (bf16) or 16 B (fp32, one piece per tap)
        const uint32_t off0 = (ok ? (uint32_t)((n * p.H + h) * p.W + w) * (4u * ES) : DEAD) | dead;
        const uint32_t off1 = (ok1 ? (uint32_t)((n * p.H + h1) * p.W + w1) * (4u * ES) : DEAD) | dead;
        if constexpr (F32) {
          rx_[2 * i] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(xr, off0, 0, 0));
          rx_[2 * i + 1] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(xr, off1, 0, 0));
        } else {
          const uint2 lo = __builtin_bit_cast(uint2, __builtin_amdgcn_raw_buffer_load_b64(xr, off0, 0, 0));
          const uint2 hi = __builtin_bit_cast(uint2, __builtin_amdgcn_raw_buffer_load_b64(xr, off1, 0, 0));
          rx_[i] = make_uint4(lo.x, lo.y, hi.x, hi.y);
        }
      } else {
        if (PRO && ok) okm |= 1u << i;
        const uint32_t off = (ok ? ((uint32_t)((n * p.H + h) * p.W + w) * (uint32_t)p.ldx + (uint32_t)cx) * (uint32_t)ES : DEAD) | dead;
        rx_[PC * i] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(xr, off, 0, 0));
        if constexpr (F32) rx_[PC * i + 1] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(xr, off + 16u, 0, 0));
      }
    }
  };
  // F32: 8 fp32 (two 16-B pieces) → the hi and lo bf16 chunks
  auto split8 = [&](const uint4 a, const uint4 b, uint4& h, uint4& l) {
    const uint32_t u[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
    uint32_t hw[4], lw[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const float v0 = __uint_as_float(u[2 * e]), v1 = __uint_as_float(u[2 * e + 1]);
      const bf16_t h0 = f2bf(v0), h1 = f2bf(v1);
      hw[e] = (uint32_t)h0 | ((uint32_t)h1 << 16);
      lw[e] = (uint32_t)f2bf(v0 - bf2f(h0)) | ((uint32_t)f2bf(v1 - bf2f(h1)) << 16);
    }
    h = make_uint4(hw[0], hw[1], hw[2], hw[3]);
    l = make_uint4(lw[0], lw[1], lw[2], lw[3]);
  };
  // PRO: relu(x·sc + sh) of a loaded 8-channel chunk (two 16-B pieces), 0 for a padded / dead row
  auto pro8 = [&](uint4& a, uint4& b, bool ok) {
    uint32_t u[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
#pragma unroll
    for (int e = 0; e < 8; ++e)
      u[e] = ok ? __float_as_uint(fmaxf(fmaf(__uint_as_float(u[e]), psc[e], psh[e]), 0.f)) : 0u;
    a = make_uint4(u[0], u[1], u[2], u[3]);
    b = make_uint4(u[4], u[5], u[6], u[7]);
  };
  auto store = [&](int buf, int mt, const uint4 (&rdy)[DY_CH * PC], const uint4 (&rx_)[X_CH * PC],
                   const uint4 (&r2)[AT ? DY_CH : 1], uint32_t okm) {
    if constexpr (F32) {
#pragma unroll
      for (int i = 0; i < DY_CH; ++i) {
        const int row = dy_row0 + i * DY_RSTEP;
        uint4 h, l;
        split8(rdy[2 * i], rdy[2 * i + 1], h, l);
        *reinterpret_cast<uint4*>(&lds[buf][tr_swz_dword<TILE_N>(row, dy_col * 4)]) = h;
        *reinterpret_cast<uint4*>(&lds[buf][LO + tr_swz_dword<TILE_N>(row, dy_col * 4)]) = l;
      }
#pragma unroll
      for (int i = 0; i < X_CH; ++i) {
        const int row = x_row0 + i * X_RSTEP;
        uint4 h, l;
        if constexpr (PRO) {
          uint4 a = rx_[2 * i], b = rx_[2 * i + 1];
          pro8(a, b, (okm >> i) & 1u);
          split8(a, b, h, l);
        } else {
          split8(rx_[2 * i], rx_[2 * i + 1], h, l);
        }
        *reinterpret_cast<uint4*>(&lds[buf][DY_WORDS + tr_swz_dword<TILE_K>(row, x_col * 4)]) = h;
        *reinterpret_cast<uint4*>(&lds[buf][LO + DY_WORDS + tr_swz_dword<TILE_K>(row, x_col * 4)]) = l;
      }
      return;
    }
#pragma unroll
    for (int i = 0; i < DY_CH; ++i) {
      int row = dy_row0 + i * DY_RSTEP;
      uint4 v = rdy[i];
      if constexpr (AT) {  // dY := the BN input gradient; rows past the split end stay zero
        const bool ok = ndy_ok && mt + row < mend;
        float g[8], xv[8];
        unpack8(rdy[i], g);
        unpack8(r2[i], xv);
        uint32_t w4[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const float o0 = ok ? fmaf(cA[2 * e], g[2 * e], fmaf(cB[2 * e], xv[2 * e], cC[2 * e])) : 0.f;
          const float o1 = ok ? fmaf(cA[2 * e + 1], g[2 * e + 1], fmaf(cB[2 * e + 1], xv[2 * e + 1], cC[2 * e + 1])) : 0.f;
          w4[e] = (uint32_t)f2bf(o0) | ((uint32_t)f2bf(o1) << 16);
        }
        v = make_uint4(w4[0], w4[1], w4[2], w4[3]);
      }
      *reinterpret_cast<uint4*>(&lds[buf][tr_swz_dword<TILE_N>(row, dy_col * 4)]) = v;
    }
#pragma unroll
    for (int i = 0; i < X_CH; ++i) {
      int row = x_row0 + i * X_RSTEP;
      *reinterpret_cast<uint4*>(&lds[buf][DY_WORDS + tr_swz_dword<TILE_K>(row, x_col * 4)]) = rx_[PC * i];
    }
  };

  v4f acc[TMN][TMK];
#pragma unroll
  for (int i = 0; i < TMN; ++i)
#pragma unroll
    for (int j = 0; j < TMK; ++j) acc[i][j] = v4f{0.f, 0.f, 0.f, 0.f};

  const int g = (lane >> 4) & 3;  // 16-lane group → pixels 8g..8g+7 of a 32-pixel k-step
  const int t = lane & 15, q4 = t >> 2, p4 = t & 3;
  // fragment of 8 consecutive pixels (transposed read) at tile word offset `base` (0: hi, LO: lo tiles)
  auto frag_n = [&](int buf, int base, int i, int kk) -> v8s {
    const int col = wave_n * (TILE_N / 2) + i * 16 + 4 * p4;  // channel of this lane's quad
    const int r0 = kk * 32 + 8 * g + q4;
    v4s lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
        (__attribute__((address_space(3))) v4s*)&lds[buf][base + tr_swz_dword<TILE_N>(r0, col >> 1)]);
    v4s hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
        (__attribute__((address_space(3))) v4s*)&lds[buf][base + tr_swz_dword<TILE_N>(r0 + 4, col >> 1)]);
    return v8s{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  };
  auto frag_k = [&](int buf, int base, int j, int kk) -> v8s {
    const int col = wave_k * (TILE_K / 2) + j * 16 + 4 * p4;
    const int r0 = kk * 32 + 8 * g + q4;
    v4s lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
        (__attribute__((address_space(3))) v4s*)&lds[buf][base + DY_WORDS + tr_swz_dword<TILE_K>(r0, col >> 1)]);
    v4s hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
        (__attribute__((address_space(3))) v4s*)&lds[buf][base + DY_WORDS + tr_swz_dword<TILE_K>(r0 + 4, col >> 1)]);
    return v8s{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  };
  auto compute = [&](int buf) {
#pragma unroll
    for (int kk = 0; kk < BPT / 32; ++kk) {
      v8s af[TMN], bfr[TMK];
#pragma unroll
      for (int i = 0; i < TMN; ++i) af[i] = frag_n(buf, 0, i, kk);
#pragma unroll
      for (int j = 0; j < TMK; ++j) bfr[j] = frag_k(buf, 0, j, kk);
      if constexpr (F32) {
        v8s afl[TMN], bfl[TMK];
#pragma unroll
        for (int i = 0; i < TMN; ++i) afl[i] = frag_n(buf, LO, i, kk);
#pragma unroll
        for (int j = 0; j < TMK; ++j) bfl[j] = frag_k(buf, LO, j, kk);
#pragma unroll
        for (int i = 0; i < TMN; ++i)
#pragma unroll
          for (int j = 0; j < TMK; ++j) {
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(afl[i], bfr[j], acc[i][j], 0, 0, 0);
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfl[j], acc[i][j], 0, 0, 0);
          }
      } else {
#pragma unroll
        for (int i = 0; i < TMN; ++i)
#pragma unroll
          for (int j = 0; j < TMK; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
      }
    }
  };

  uint4 dy0[DY_CH * PC], x0[X_CH * PC], dy1[DY_CH * PC], x1[X_CH * PC];
  uint4 z0[AT ? DY_CH : 1], z1[AT ? DY_CH : 1];
  uint32_t ok0 = 0, ok1 = 0;
  const int NT = (mend - mbeg + BPT - 1) / BPT;
  load(mbeg, true, dy0, x0, z0, ok0);
  load(mbeg + BPT, NT > 1, dy1, x1, z1, ok1);
  store(0, mbeg, dy0, x0, z0, ok0);
  __syncthreads();
  int it = 0;
  for (; it + 2 <= NT; it += 2) {
    load(mbeg + (it + 2) * BPT, it + 2 < NT, dy0, x0, z0, ok0);
    compute(0);
    store(1, mbeg + (it + 1) * BPT, dy1, x1, z1, ok1);
    __syncthreads();
    load(mbeg + (it + 3) * BPT, it + 3 < NT, dy1, x1, z1, ok1);
    compute(1);
    if (it + 2 < NT) store(0, mbeg + (it + 2) * BPT, dy0, x0, z0, ok0);
    __syncthreads();
  }
  if (it < NT) {
    compute(0);
  }

  // epilogue: D[row = n][col = k]; lane holds rows (lane>>4)*4 + e of column lane&15
  if (p.skip_epi) return;
  if (p.epi_lds) {
    // rows per pass: a multiple of 16 dividing TILE_N whose padded fp32 image fits the ring's LDS
    constexpr int LDK = TILE_K + 16;  // +16 floats: the 4 rows of one write land on distinct banks
    constexpr int LDS_F = (int)(sizeof(lds) / 4);
    constexpr int ROWS = (TILE_N * LDK <= LDS_F) ? TILE_N : (TILE_N / 2 * LDK <= LDS_F) ? TILE_N / 2
                         : (TILE_N / 4 * LDK <= LDS_F) ? TILE_N / 4 : 16;
    static_assert(ROWS * LDK <= LDS_F && TILE_N % ROWS == 0 && ROWS % 16 == 0, "wgrad epilogue staging");
    float* st = reinterpret_cast<float*>(&lds[0][0]);
    __syncthreads();  // the last k-tile's fragment reads are done with the ring
#pragma unroll
    for (int pass = 0; pass < TILE_N / ROWS; ++pass) {
#pragma unroll
      for (int i = 0; i < TMN; ++i) {
        const int rb = wave_n * (TILE_N / 2) + i * 16;  // this (wave, i)'s 16 rows
        if (rb < pass * ROWS || rb >= (pass + 1) * ROWS) continue;
#pragma unroll
        for (int j = 0; j < TMK; ++j) {
          const int c = wave_k * (TILE_K / 2) + j * 16 + (lane & 15);
#pragma unroll
          for (int e = 0; e < 4; ++e) st[(rb - pass * ROWS + (lane >> 4) * 4 + e) * LDK + c] = acc[i][j][e];
        }
      }
      __syncthreads();
#pragma unroll 4
      for (int idx = tid; idx < ROWS * TILE_K; idx += 256) {
        const int r = idx / TILE_K, c = idx - r * TILE_K;
        const int n = n0 + pass * ROWS + r, k = k0 + c;
        if (n < p.K && k < p.Kg) atomicAdd(p.dw + (size_t)n * p.Kg + k, p.scale * st[r * LDK + c]);
      }
      if (pass + 1 < TILE_N / ROWS) __syncthreads();
    }
    return;
  }
#pragma unroll
  for (int i = 0; i < TMN; ++i) {
#pragma unroll
    for (int j = 0; j < TMK; ++j) {
      const int k = k0 + wave_k * (TILE_K / 2) + j * 16 + (lane & 15);
      if (k >= p.Kg) continue;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int n = n0 + wave_n * (TILE_N / 2) + i * 16 + (lane >> 4) * 4 + e;
        if (n < p.K) atomicAdd(p.dw + (size_t)n * p.Kg + k, p.scale * acc[i][j][e]);
      }
    }
  }
}

// 3-D weight gradient (VolumetricConvolution.scala accGradParameters): dw [K][KT][R][S][C] +=
// scale · Σ x̂ᵀ·dy over (sample, output frame, p, q).  C % 8 == 0, K % 8 == 0.
BIGDL_EXPORT int bigdl_conv3d_wgrad(const void* x, const void* dy, float* dw, float scale, int Nb, int T, int H, int W,
                                    int C, int K, int KT, int R, int S, int To, int P, int Q, int st, int sh, int sw,
                                    int pt, int ph, int pw, int dtd, int dh, int dwd, hipStream_t s) {
  if (C % 8 || K % 8 || Nb <= 0 || T <= 0 || To <= 0 || KT <= 0 || R <= 0 || S <= 0) return (int)hipErrorInvalidValue;
  if ((size_t)Nb * T * H * W * C * 2 >= 0x80000000ull || (size_t)Nb * To * P * Q * K * 2 >= 0x80000000ull)
    return (int)hipErrorInvalidValue;
  if (((uintptr_t)x & 15) || ((uintptr_t)dy & 15)) return (int)hipErrorInvalidValue;
  WgradParams p{};
  p.x = (const bf16_t*)x; p.dy = (const bf16_t*)dy; p.dw = dw; p.scale = scale;
  p.Nb = Nb; p.H = H; p.W = W; p.C = C; p.K = K; p.R = R; p.S = S; p.P = P; p.Q = Q;
  p.sh = sh; p.sw = sw; p.ph = ph; p.pw = pw; p.dh = dh; p.dw_ = dwd;
  p.T = T; p.KT = KT; p.st = st; p.pt = pt; p.dtd = dtd; p.To = To;
  p.ldx = C; p.ldk = K;
  p.M = Nb * To * P * Q;
  p.Kg = KT * R * S * C;
  p.fPQ = make_fastdiv((uint32_t)(P * Q));
  p.fQ = make_fastdiv((uint32_t)Q);
  p.fRS = make_fastdiv((uint32_t)(R * S));
  p.fTo = make_fastdiv((uint32_t)To);
  const int TN = K <= 64 ? 64 : 128;
  p.tiles_n = (K + TN - 1) / TN;
  p.tiles_k = (p.Kg + 127) / 128;
  const int tiles = p.tiles_n * p.tiles_k;
  long long splits = g_bigdl_deterministic ? 1 : (512 + tiles - 1) / tiles;
  const long long max_by_work = (p.M + 8 * BP - 1) / (8 * BP);
  if (splits > max_by_work) splits = max_by_work;
  if (splits < 1) splits = 1;
  if (splits > 65535) splits = 65535;
  int mps = (int)((p.M + splits - 1) / splits);
  mps = (mps + BP - 1) / BP * BP;
  p.m_per_split = mps;
  const dim3 grid(tiles, (p.M + mps - 1) / mps);
  if (TN == 64) hipLaunchKernelGGL((k_conv_wgrad<64, 128, 64, false, true>), grid, dim3(256), 0, s, p);
  else hipLaunchKernelGGL((k_conv_wgrad<128, 128, 64, false, true>), grid, dim3(256), 0, s, p);
  BIGDL_CHECK_LAUNCH();
}

// dw += scale · wgrad.  Requirements (checked): C % 8 == 0, K % 8 == 0, 16-B aligned x/dy.
// Grouped (groups > 1): C / K are per group, x / dy pixels ldx / ldk apart with group g at channel
// g·C / g·K, dw = groups × [K][R][S][C] blocks; the group is blockIdx.z.
static int wgrad_launch(const void* x, const void* dy, float* dw, float scale, int Nb, int H, int W, int C, int K,
                        int R, int S, int P, int Q, int sh, int sw, int ph, int pw, int dh, int dwd, int splits,
                        hipStream_t s, int ldx, int ldk, int groups, const void* dy2 = nullptr,
                        const float* dcoef = nullptr, int bp_pin = 0) {
  const bool c4 = C == 4;
  if ((C % 8 && !c4) || K % 8 || Nb <= 0) return (int)hipErrorInvalidValue;
  if (c4 && (dh != 1 || dwd != 1)) return (int)hipErrorInvalidValue;
  if (groups < 1 || groups > 65535 || ldx < groups * C || ldk < groups * K) return (int)hipErrorInvalidValue;
  if ((ldx != C || ldk != K) && (c4 || ldx % 8 || ldk % 8)) return (int)hipErrorInvalidValue;
  if ((size_t)Nb * H * W * ldx * 2 >= 0x80000000ull || (size_t)Nb * P * Q * ldk * 2 >= 0x80000000ull)
    return (int)hipErrorInvalidValue;  // 32-bit buffer offsets
  WgradParams p{};
  static const int skip_env = [] { const char* ev = getenv("BIGDL_DEBUG_WGRAD_NO_ATOMICS"); return ev ? atoi(ev) : 0; }();
  p.skip_epi = skip_env;
  const char* epi_env = getenv("BIGDL_WGRAD_EPI");  // per launch: tests switch it in-process
  p.epi_lds = epi_env ? atoi(epi_env) : 0;
  p.ldx = ldx; p.ldk = ldk;
  if ((dy2 != nullptr) != (dcoef != nullptr) || (dy2 && (c4 || groups != 1 || ((uintptr_t)dy2 & 15))))
    return (int)hipErrorInvalidValue;
  p.dy2 = (const bf16_t*)dy2;
  p.dcoef = dcoef;
  p.gx = C; p.gdy = K; p.gdw = (long long)K * R * S * C;
  p.x = (const bf16_t*)x;
  p.dy = (const bf16_t*)dy;
  p.dw = dw;
  p.scale = scale;
  p.Nb = Nb; p.H = H; p.W = W; p.C = C; p.K = K; p.R = R; p.S = S; p.P = P; p.Q = Q;
  p.sh = sh; p.sw = sw; p.ph = ph; p.pw = pw; p.dh = dh; p.dw_ = dwd;
  p.M = Nb * P * Q;
  p.Kg = R * S * C;
  p.fPQ = make_fastdiv((uint32_t)(P * Q));
  p.fQ = make_fastdiv((uint32_t)Q);
  p.pw1 = (R == 1 && S == 1 && sh == 1 && sw == 1 && ph == 0 && pw == 0 && P == H && Q == W && !c4) ? 1 : 0;
  const int TN = K <= 64 ? 64 : 128;
  const int TK = (p.Kg <= 64 && !c4) ? 64 : 128;  // the C4 kernels are instantiated with 128-wide k tiles only
  p.tiles_n = (K + TN - 1) / TN;
  p.tiles_k = (p.Kg + TK - 1) / TK;
  const int tiles = p.tiles_n * p.tiles_k;
  if (g_bigdl_deterministic) splits = 1;  // one block per output tile: no racing atomics
  if (splits <= 0) {
    // splits <= 0: aim for -splits blocks in total (default 512 = two resident blocks per CU), but
    // ≥ 8 k-tiles of pixels per block.  Every split adds its full K×Kg partial with fp32 atomics
    // (≈1.3 TB/s chip-wide, MI355X_MICROARCH.md 'Global float atomics'), so fewer, longer splits win
    // once the grid fills the chip.
    const long long target = splits < 0 ? -(long long)splits : 512;
    long long want = (target + (long long)tiles * groups - 1) / ((long long)tiles * groups);
    long long max_by_work = (p.M + 8 * BP - 1) / (8 * BP);
    splits = (int)(want < max_by_work ? want : max_by_work);
    if (splits < 1) splits = 1;
    if (splits > 65535) splits = 65535;
  }
  int mps = (p.M + splits - 1) / splits;
  mps = (mps + BP - 1) / BP * BP;
  p.m_per_split = mps;
  splits = (p.M + mps - 1) / mps;
  dim3 grid(tiles, splits, groups);
  // Pixel depth of a k-tile: 32 (half the LDS / prefetch registers, 3 blocks per CU) wins on the
  // small weight grids (≤ 16 tiles, K ≥ 128: few tiles, long split reductions), 64 elsewhere
  // (profiles/r1_conv_bk_ab.txt).  BIGDL_WGRAD_BP=32|64 pins it for A/B measurements.
  // A launch may pin it (the compile phase's kernel selection, bigdl_conv_wgrad_t).
  static const int bp_env = [] { const char* ev = getenv("BIGDL_WGRAD_BP"); return ev ? atoi(ev) : 0; }();
  const int bp = (bp_pin == 32 || bp_pin == 64) ? bp_pin
                 : (bp_env == 32 || bp_env == 64) ? bp_env : (tiles <= 16 && K >= 128 ? 32 : 64);
  if (dy2) {  // BN-backward prologue: the 32-deep k-tile variants (register budget for the second dY)
    if (TN == 64) {
      if (TK == 64) hipLaunchKernelGGL((k_conv_wgrad<64, 64, 32, false, false, true>), grid, dim3(256), 0, s, p);
      else hipLaunchKernelGGL((k_conv_wgrad<64, 128, 32, false, false, true>), grid, dim3(256), 0, s, p);
    } else {
      if (TK == 64) hipLaunchKernelGGL((k_conv_wgrad<128, 64, 32, false, false, true>), grid, dim3(256), 0, s, p);
      else hipLaunchKernelGGL((k_conv_wgrad<128, 128, 32, false, false, true>), grid, dim3(256), 0, s, p);
    }
    BIGDL_CHECK_LAUNCH();
  }
  if (c4) {
    if (bp == 32) {
      if (TN == 64) hipLaunchKernelGGL((k_conv_wgrad<64, 128, 32, true>), grid, dim3(256), 0, s, p);
      else hipLaunchKernelGGL((k_conv_wgrad<128, 128, 32, true>), grid, dim3(256), 0, s, p);
    } else {
      if (TN == 64) hipLaunchKernelGGL((k_conv_wgrad<64, 128, 64, true>), grid, dim3(256), 0, s, p);
      else hipLaunchKernelGGL((k_conv_wgrad<128, 128, 64, true>), grid, dim3(256), 0, s, p);
    }
  } else if (p.pw1 && bp == 32) {
    if (TN == 64 && TK == 64) hipLaunchKernelGGL((k_conv_wgrad<64, 64, 32, false, false, false, true>), grid, dim3(256), 0, s, p);
    else if (TN == 64) hipLaunchKernelGGL((k_conv_wgrad<64, 128, 32, false, false, false, true>), grid, dim3(256), 0, s, p);
    else if (TK == 64) hipLaunchKernelGGL((k_conv_wgrad<128, 64, 32, false, false, false, true>), grid, dim3(256), 0, s, p);
    else hipLaunchKernelGGL((k_conv_wgrad<128, 128, 32, false, false, false, true>), grid, dim3(256), 0, s, p);
  } else if (p.pw1) {
    if (TN == 64 && TK == 64) hipLaunchKernelGGL((k_conv_wgrad<64, 64, 64, false, false, false, true>), grid, dim3(256), 0, s, p);
    else if (TN == 64) hipLaunchKernelGGL((k_conv_wgrad<64, 128, 64, false, false, false, true>), grid, dim3(256), 0, s, p);
    else if (TK == 64) hipLaunchKernelGGL((k_conv_wgrad<128, 64, 64, false, false, false, true>), grid, dim3(256), 0, s, p);
    else hipLaunchKernelGGL((k_conv_wgrad<128, 128, 64, false, false, false, true>), grid, dim3(256), 0, s, p);
  } else if (bp == 32) {
    if (TN == 64 && TK == 64) hipLaunchKernelGGL((k_conv_wgrad<64, 64, 32>), grid, dim3(256), 0, s, p);
    else if (TN == 64) hipLaunchKernelGGL((k_conv_wgrad<64, 128, 32>), grid, dim3(256), 0, s, p);
    else if (TK == 64) hipLaunchKernelGGL((k_conv_wgrad<128, 64, 32>), grid, dim3(256), 0, s, p);
    else hipLaunchKernelGGL((k_conv_wgrad<128, 128, 32>), grid, dim3(256), 0, s, p);
  } else {
    if (TN == 64 && TK == 64) hipLaunchKernelGGL((k_conv_wgrad<64, 64, 64>), grid, dim3(256), 0, s, p);
    else if (TN == 64) hipLaunchKernelGGL((k_conv_wgrad<64, 128, 64>), grid, dim3(256), 0, s, p);
    else if (TK == 64) hipLaunchKernelGGL((k_conv_wgrad<128, 64, 64>), grid, dim3(256), 0, s, p);
    else hipLaunchKernelGGL((k_conv_wgrad<128, 128, 64>), grid, dim3(256), 0, s, p);
  }
  BIGDL_CHECK_LAUNCH();
}

BIGDL_EXPORT int bigdl_conv_wgrad(const void* x, const void* dy, float* dw, float scale, int Nb, int H, int W, int C,
                                  int K, int R, int S, int P, int Q, int sh, int sw, int ph, int pw, int dh, int dwd,
                                  int splits, hipStream_t s) {
  return wgrad_launch(x, dy, dw, scale, Nb, H, W, C, K, R, S, P, Q, sh, sw, ph, pw, dh, dwd, splits, s, C, K, 1);
}

// bigdl_conv_wgrad with the k-tile pixel depth pinned (bp ∈ {32, 64}; 0 = heuristic).
BIGDL_EXPORT int bigdl_conv_wgrad_t(const void* x, const void* dy, float* dw, float scale, int Nb, int H, int W, int C,
                                    int K, int R, int S, int P, int Q, int sh, int sw, int ph, int pw, int dh, int dwd,
                                    int splits, int bp, hipStream_t s) {
  if (bp != 0 && bp != 32 && bp != 64) return (int)hipErrorInvalidValue;
  return wgrad_launch(x, dy, dw, scale, Nb, H, W, C, K, R, S, P, Q, sh, sw, ph, pw, dh, dwd, splits, s, C, K, 1, nullptr,
                      nullptr, bp);
}

// bigdl_conv_wgrad with a BatchNorm-backward prologue on dY: dy = g' at the BN output, dy2 = the BN input,
// dcoef [3][K] (dY := A·g' + B·dy2 + Cc).
BIGDL_EXPORT int bigdl_conv_wgrad_bnbwd(const void* x, const void* dy, const void* dy2, const float* dcoef, float* dw,
                                        float scale, int Nb, int H, int W, int C, int K, int R, int S, int P, int Q,
                                        int sh, int sw, int ph, int pw, int dh, int dwd, int splits, hipStream_t s) {
  if (!dy2 || !dcoef) return (int)hipErrorInvalidValue;
  return wgrad_launch(x, dy, dw, scale, Nb, H, W, C, K, R, S, P, Q, sh, sw, ph, pw, dh, dwd, splits, s, C, K, 1, dy2,
                      dcoef);
}

// Grouped weight gradient in one launch (SpatialConvolution.scala:93-98 nGroup accGradParameters).
BIGDL_EXPORT int bigdl_conv_wgrad_grouped(const void* x, const void* dy, float* dw, float scale, int Nb, int H, int W,
                                          int ldx, int Cg, int ldk, int Kg, int groups, int R, int S, int P, int Q,
                                          int sh, int sw, int ph, int pw, int dh, int dwd, hipStream_t s) {
  if (Cg == 4) return (int)hipErrorInvalidValue;
  return wgrad_launch(x, dy, dw, scale, Nb, H, W, Cg, Kg, R, S, P, Q, sh, sw, ph, pw, dh, dwd, 0, s, ldx, ldk, groups);
}

// fp32 operands (bf16x3 fp32 compute mode): x [Nb][H][W][C], dy [Nb][P][Q][K] fp32 NHWC (16-B aligned,
// C % 8 == 0, K % 8 == 0); dw [K][R][S][C] fp32 += scale · Σ dyᵀ·x̂ at bf16x3 accuracy in ONE launch.
// Pixel depth 32 per k-tile (the hi + lo tiles double the LDS image).  splits <= 0: heuristic.
// C == 4 (the padded RGB stem, x [Nb][H][W][4]): the C4 gather, an 8-index chunk = two taps × 4 channels.
static int wgrad_f32_impl(const float* x, const float* dy, float* dw, float scale, int Nb, int H, int W, int C, int K,
                          int R, int S, int P, int Q, int sh, int sw, int ph, int pw, int dh, int dwd, int splits,
                          hipStream_t s, const float* pro) {
  const bool c4 = C == 4;
  if (pro && (c4 || C % 8 || ((uintptr_t)pro & 15))) return (int)hipErrorInvalidValue;
  if ((C % 8 && !c4) || K % 8 || Nb <= 0 || !x || !dy || !dw) return (int)hipErrorInvalidValue;
  if (c4 && (dh != 1 || dwd != 1)) return (int)hipErrorInvalidValue;
  if (((uintptr_t)x & 15) || ((uintptr_t)dy & 15)) return (int)hipErrorInvalidValue;
  if ((size_t)Nb * H * W * C * 4 >= 0x80000000ull || (size_t)Nb * P * Q * K * 4 >= 0x80000000ull)
    return (int)hipErrorInvalidValue;
  WgradParams p{};
  p.ldx = C; p.ldk = K;
  p.gx = C; p.gdy = K; p.gdw = (long long)K * R * S * C;
  p.x = (const bf16_t*)x;
  p.dy = (const bf16_t*)dy;
  p.dw = dw;
  p.scale = scale;
  const char* epi_env = getenv("BIGDL_WGRAD_EPI");
  p.epi_lds = epi_env ? atoi(epi_env) : 0;
  p.Nb = Nb; p.H = H; p.W = W; p.C = C; p.K = K; p.R = R; p.S = S; p.P = P; p.Q = Q;
  p.sh = sh; p.sw = sw; p.ph = ph; p.pw = pw; p.dh = dh; p.dw_ = dwd;
  const long long Ml = (long long)Nb * P * Q;
  if (Ml > 0x7fffffffLL) return (int)hipErrorInvalidValue;
  p.M = (int)Ml;
  p.Kg = R * S * C;
  p.fPQ = make_fastdiv((uint32_t)(P * Q));
  p.fQ = make_fastdiv((uint32_t)Q);
  p.pw1 = (R == 1 && S == 1 && sh == 1 && sw == 1 && ph == 0 && pw == 0 && P == H && Q == W && !c4) ? 1 : 0;
  p.pro = pro;
  const int TN = K <= 64 ? 64 : 128;
  const int TK = (p.Kg <= 64 && !c4) ? 64 : 128;
  p.tiles_n = (K + TN - 1) / TN;
  p.tiles_k = (p.Kg + TK - 1) / TK;
  const int tiles = p.tiles_n * p.tiles_k;
  if (g_bigdl_deterministic) splits = 1;
  if (splits <= 0) {
    const long long target = splits < 0 ? -(long long)splits : 512;
    long long want = (target + tiles - 1) / tiles;
    const long long max_by_work = (p.M + 8 * BP - 1) / (8 * BP);
    splits = (int)(want < max_by_work ? want : max_by_work);
    if (splits < 1) splits = 1;
    if (splits > 65535) splits = 65535;
  }
  int mps = (p.M + splits - 1) / splits;
  mps = (mps + BP - 1) / BP * BP;
  p.m_per_split = mps;
  splits = (p.M + mps - 1) / mps;
  const dim3 grid(tiles, splits, 1);
#define BIGDL_WF32(TN_, TK_, PW_) \
  hipLaunchKernelGGL((k_conv_wgrad<TN_, TK_, 32, false, false, false, PW_, true>), grid, dim3(256), 0, s, p)
#define BIGDL_WF32P(TN_, TK_, PW_) \
  hipLaunchKernelGGL((k_conv_wgrad<TN_, TK_, 32, false, false, false, PW_, true, true>), grid, dim3(256), 0, s, p)
  if (pro) {
    if (p.pw1) {
      if (TN == 64 && TK == 64) BIGDL_WF32P(64, 64, true);
      else if (TN == 64) BIGDL_WF32P(64, 128, true);
      else if (TK == 64) BIGDL_WF32P(128, 64, true);
      else BIGDL_WF32P(128, 128, true);
    } else {
      if (TN == 64 && TK == 64) BIGDL_WF32P(64, 64, false);
      else if (TN == 64) BIGDL_WF32P(64, 128, false);
      else if (TK == 64) BIGDL_WF32P(128, 64, false);
      else BIGDL_WF32P(128, 128, false);
    }
  } else if (c4) {
    if (TN == 64) hipLaunchKernelGGL((k_conv_wgrad<64, 128, 32, true, false, false, false, true>), grid, dim3(256), 0, s, p);
    else hipLaunchKernelGGL((k_conv_wgrad<128, 128, 32, true, false, false, false, true>), grid, dim3(256), 0, s, p);
  } else if (p.pw1) {
    if (TN == 64 && TK == 64) BIGDL_WF32(64, 64, true);
    else if (TN == 64) BIGDL_WF32(64, 128, true);
    else if (TK == 64) BIGDL_WF32(128, 64, true);
    else BIGDL_WF32(128, 128, true);
  } else {
    if (TN == 64 && TK == 64) BIGDL_WF32(64, 64, false);
    else if (TN == 64) BIGDL_WF32(64, 128, false);
    else if (TK == 64) BIGDL_WF32(128, 64, false);
    else BIGDL_WF32(128, 128, false);
  }
#undef BIGDL_WF32
#undef BIGDL_WF32P
  BIGDL_CHECK_LAUNCH();
}

BIGDL_EXPORT int bigdl_conv_wgrad_f32(const float* x, const float* dy, float* dw, float scale, int Nb, int H, int W,
                                      int C, int K, int R, int S, int P, int Q, int sh, int sw, int ph, int pw, int dh,
                                      int dwd, int splits, hipStream_t s) {
  return wgrad_f32_impl(x, dy, dw, scale, Nb, H, W, C, K, R, S, P, Q, sh, sw, ph, pw, dh, dwd, splits, s, nullptr);
}

// bigdl_conv_wgrad_f32 whose x is the INPUT of a training BN + ReLU (its output deferred): X̂ =
// relu(x·pro[c] + pro[C + c]) on load, pro = [scale | shift] [2][C].
BIGDL_EXPORT int bigdl_conv_wgrad_f32_pro(const float* x, const float* pro, const float* dy, float* dw, float scale,
                                          int Nb, int H, int W, int C, int K, int R, int S, int P, int Q, int sh,
                                          int sw, int ph, int pw, int dh, int dwd, int splits, hipStream_t s) {
  if (!pro) return (int)hipErrorInvalidValue;
  return wgrad_f32_impl(x, dy, dw, scale, Nb, H, W, C, K, R, S, P, Q, sh, sw, ph, pw, dh, dwd, splits, s, pro);
}
