// fp32 implicit-GEMM convolution on the bf16 matrix cores with the operand split done IN the kernel
// ("bf16x3", csrc/precision.hip): D[n = out channel][m = output pixel] = Σ_k W[n][k] · X̂[m][k] at fp32
// accuracy as  W_hi·X_hi + W_lo·X_hi + W_hi·X_lo  (v_mfma_f32_32x32x16_bf16, fp32 accumulation).
// Reference: SpatialConvolution.updateOutput / updateGradInput in fp32 (MKL-DNN fp32 primitives,
// DL/nn/SpatialConvolution.scala:253-430); no im2col is materialised.
//
// Why a separate family: the conv_igemm / conv_mfma32 kernels take the fp32 activations as a
// materialised [hi | lo] bf16 split read as three logical parts [hi | hi | lo] (ConvParams::cdup), so
// every fp32 activation costs a split pass (or a second write by its producer) and the kernel stages
// 3 × 2 B per element through LDS for 3 MFMAs.  Here the raw fp32 activation rows go global → LDS by the
// LDS-DMA path (4 B per element, the same bytes as the split) and each wave splits its B fragments
// while reading them (v_cvt_pk_bf16_f32, round-to-nearest hi and lo: |v − hi − lo| ≤ 2^-17 |v|), so
// 2 fragment reads feed 3 MFMAs and nothing upstream has to write a split.  The weights (small, per
// step) are pre-split by the host into 32-channel [hi | lo] chunks: W2[n][kt][0:32] = hi, [32:64] = lo
// of reduction indices kt·32 … kt·32 + 31 — one 128-B LDS row per k-tile, like the activation row.
//
// Tile: BM pixels × BN channels, 8 waves (WM × WN), k-tile = 32 reduction indices (one tap, 32
// channels), a 3-deep LDS ring with counted vmcnt and raw s_barrier (as conv_mfma32.hip; the next
// stage's LDS-DMA pieces are issued between the MFMA groups of the current one).  LDS rows are 128 B with
// the XOR swizzle chunk ^ ((row >> 1) & 7) on the DMA source address and on every fragment read, which
// keeps both the bf16 (A) and the fp32 (B) fragment reads conflict-free.
//
// Epilogues (uniform branches on the launch's arguments).  The accumulators (lane l of a 32×32 block holds
// pixel l & 31 and channels 8·(r >> 2) + 4·(l >> 5) + (r & 3)) are parked as an fp32 tile in the ring's
// LDS and walked row-major, so every store / residual / BN-input access of a wave-instruction covers whole
// 4·BN-byte row segments (the register-direct form wrote 32 rows × 32 B per instruction and ran the
// expand 1×1 convs store-bound: 372 vs 208 µs with the stores skipped, 64→256 at 56², batch 256):
//   plain  : y = relu?(acc + bias + res), fp32 [M][ldy];
//   stats  : y = acc, plus Σ(y − shift), Σ(y − shift)² of the following BN added into its replicated
//            buffer [2][R][K] (fp32 atomics, one per block and channel after an LDS fold);
//   bnbwd  : the data gradient g = acc (+ res) masked by the ReLU of the BN that produced this
//            conv's input (mask bits, or recomputed as sc·x + sh > 0 from that BN's input x), stored,
//            and Σg, Σg·(x − mean) of that BN's backward added into its replicated buffer.
// Modes: 1 = tap-uniform gather (C % 32 == 0, R·S ≤ 64), 3 = pointwise (1×1, no padding), 2 = C4: the
// 4-channel (padded RGB) stem input [Nb][H][W][4] — a k-tile is 8 taps × 4 channels, each lane's 16-B
// DMA piece one tap of its row (its own padding test), so the 7×7 stem reduces over ⌈49 / 8⌉·32 = 224
// indices (the s2d image's 16 taps × 32 padded channels were 512).
#include "common.h"
#include <type_traits>

typedef short v8s __attribute__((ext_vector_type(8)));
typedef float v4f __attribute__((ext_vector_type(4)));
typedef float v16f __attribute__((ext_vector_type(16)));
typedef float v2f __attribute__((ext_vector_type(2)));
typedef __bf16 v2bf __attribute__((ext_vector_type(2)));

#define X3_WAIT(n) asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)" ::"n"(n) : "memory")
#define X3_BARRIER()                   \
  do {                                 \
    asm volatile("" ::: "memory");     \
    __builtin_amdgcn_s_barrier();      \
    asm volatile("" ::: "memory");     \
  } while (0)

typedef __attribute__((address_space(3))) void x3_lds_t;

struct X3Params {
  const float* x;      // [Nb][H][W][ldx] fp32
  const bf16_t* w;     // [K][Kg / 32][64] bf16: per 32-index k-chunk, hi then lo
  const float* bias;   // [K] or null
  const float* res;    // [M][ldy] fp32 or null (added before the ReLU / the mask)
  float* y;            // [M][ldy] fp32
  int Nb, H, W, C, K, R, S, P, Q;
  int sh, sw, ph, pw, dh, dw;
  int M, Kg, ldx, ldy;
  int relu;
  int tiles_n;
  // statistics (stats != null): [2][R_rep][K], tile tm adds into replica tm % R_rep
  float* stats;
  int R_rep;
  const float* shift;  // forward statistics shift (the BN's running mean), [K]
  // BN-backward epilogue (bnx != null): the BN input [M][K], its mean, and the ReLU mask as bits
  // ([M][K / 8], bit e of byte (m, c / 8) = channel c) or recomputed from sc · x + sh > 0
  const float* bnx;
  const float* mean;
  const uint8_t* bits;
  const float* bsc;
  const float* bsh;
  // output scatter (sub-pixel strided data gradient): output pixel (n, p, q) of this launch is pixel
  // (n, p·osh + ooh, q·osw + oow) of an [Nb][oH][oW] grid (y, res and bnx are all on that grid)
  int scatter, osh, osw, ooh, oow, oH, oW;
  // strided residual (res_sh > 0): `res` holds only the grid pixels (h, w) with h % res_sh == 0 and
  // w % res_sw == 0 as a dense [Nb][res_H][res_W][ldy] tensor (a 1×1 stride-s shortcut's input gradient)
  int res_sh, res_sw, res_H, res_W;
  // measurement knob (BIGDL_X3_DEBUG, read per launch): bit 0 = skip the output stores (leaves y WRONG)
  int dbg;
  // B-operand prologue (PRO instantiations): x is the INPUT of a training BN + ReLU whose output this
  // conv consumes; the conv reads relu(x·pro[c] + pro[C + c]) (padded taps stay 0), so the BN output is
  // never written (C ≤ X3_PRO_MAXC)
  const float* pro;
};

constexpr int X3_PRO_MAXC = 512;


// the prologue of one slice: y = relu(x·sc + sh) of a lane's 8 channels for its TMI fragment rows
// (0 for a padded tap); sc = this slice's scales in the [scale | shift] LDS copy
template <int TMI>
__device__ __forceinline__ void x3_pro_slice(v4f (&a)[TMI], v4f (&b)[TMI], const float* sc, const bool (&valid)[TMI]) {
  const v4f s0 = *reinterpret_cast<const v4f*>(sc), s1 = *reinterpret_cast<const v4f*>(sc + 4);
  const v4f h0 = *reinterpret_cast<const v4f*>(sc + X3_PRO_MAXC), h1 = *reinterpret_cast<const v4f*>(sc + X3_PRO_MAXC + 4);
#pragma unroll
  for (int j = 0; j < TMI; ++j)
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      a[j][e] = valid[j] ? fmaxf(fmaf(a[j][e], s0[e], h0[e]), 0.f) : 0.f;
      b[j][e] = valid[j] ? fmaxf(fmaf(b[j][e], s1[e], h1[e]), 0.f) : 0.f;
    }
}


// One 16-B-per-lane LDS-DMA piece (buffer_load_dwordx4 ... lds): lane l's 16 bytes land at lds + 16·l.
// (A non-template function: inside the kernel template the builtin fails host-side substitution.)
__device__ __forceinline__ void x3_glds16(__amdgpu_buffer_rsrc_t r, void* lds, uint32_t voff) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (x3_lds_t*)lds, 16, voff, 0, 0, 0);
}

__device__ __forceinline__ int x3_xcd_remap(int bid, int nwg) {
  const int xcd = bid & 7, q = nwg >> 3, r = nwg & 7;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (bid >> 3);
}

// 8 fp32 → bf16 hi and lo fragments: hi = rne(v), lo = rne(v − hi) (both v_cvt_pk_bf16_f32)
__device__ __forceinline__ void x3_split8(const v4f a, const v4f b, v8s& hi, v8s& lo) {
  const float v[8] = {a[0], a[1], a[2], a[3], b[0], b[1], b[2], b[3]};
  uint32_t hw[4], lw[4];
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    const v2bf h = __builtin_convertvector((v2f){v[2 * e], v[2 * e + 1]}, v2bf);
    const uint32_t hu = __builtin_bit_cast(uint32_t, h);
    const float r0 = v[2 * e] - __uint_as_float(hu << 16);
    const float r1 = v[2 * e + 1] - __uint_as_float(hu & 0xFFFF0000u);
    const v2bf l = __builtin_convertvector((v2f){r0, r1}, v2bf);
    hw[e] = hu;
    lw[e] = __builtin_bit_cast(uint32_t, l);
  }
  typedef uint32_t u4 __attribute__((ext_vector_type(4)));
  hi = __builtin_bit_cast(v8s, (u4){hw[0], hw[1], hw[2], hw[3]});
  lo = __builtin_bit_cast(v8s, (u4){lw[0], lw[1], lw[2], lw[3]});
}

// fold a per-lane value over the 16 lanes of its DPP row (every lane of the row ends with the sum)
__device__ __forceinline__ float x3_row_fold(float v) {
  v += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x128, 0xF, 0xF, false));
  v += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x124, 0xF, 0xF, false));
  v += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x122, 0xF, 0xF, false));
  v += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x121, 0xF, 0xF, false));
  return v;
}

template <int BM, int BN, int WM, int WN, int MODE, int NS, bool PRO = false>
__global__ void __launch_bounds__(64 * WM * WN, NS == 2 ? (BM * BN <= 128 * 64 ? 3 : 2) : 1) k_conv_x3(X3Params p) {
  static_assert(!PRO || MODE != 2, "the BN prologue reads a BN output: never the RGB stem");
  static_assert(MODE == 1 || MODE == 2 || MODE == 3, "tap-uniform / C4 / pointwise gathers only");
  constexpr bool C4 = MODE == 2;
  static_assert(NS == 2 || NS == 3, "LDS ring depth");
  constexpr bool PW = MODE == 3;
  constexpr int NT = 64 * WM * WN, NW = WM * WN;
  constexpr int BK = 32;                       // reduction indices per k-tile (one 128-B row each side)
  constexpr int STAGE = (BM + BN) * 128;
  constexpr int GA = BN / 8 / NW, GB = BM / 8 / NW;  // 8-row DMA groups per wave: weights, activations
  static_assert(GA * NW * 8 == BN && GB * NW * 8 == BM, "tile rows must split evenly over the waves");
  constexpr int L = GA + GB;
  constexpr int TMI = BM / WM / 32, TNI = BN / WN / 32;
  static_assert(TMI >= 1 && TNI >= 1, "wave tile below 32x32");
  // epilogue staging: the fp32 tile [BM][BN] (16-B chunks XOR-swizzled by row) + [2][RPP][BN] partial sums
  constexpr int CPR = BN / 4, RPP = NT / CPR;
  constexpr int EPI = BM * BN * 4 + 2 * RPP * BN * 4;
  constexpr int LDS_BYTES = NS * STAGE > EPI ? NS * STAGE : EPI;
  __shared__ __attribute__((aligned(16))) unsigned char lds[LDS_BYTES];
  __shared__ __attribute__((aligned(16))) float pro_s[PRO ? 2 * X3_PRO_MAXC : 4];  // [scale | shift]

  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wave_m = wid % WM, wave_n = wid / WM;
  const int tile = x3_xcd_remap(blockIdx.x, gridDim.x);
  const int tm = tile / p.tiles_n, tn = tile - tm * p.tiles_n;
  const int m0 = tm * BM, n0 = tn * BN;
  if constexpr (PRO) {  // visible after the main loop's first barrier
    for (int i = tid; i < p.C; i += NT) {
      pro_s[i] = p.pro[i];
      pro_s[X3_PRO_MAXC + i] = p.pro[p.C + i];
    }
  }

  const uint32_t x_bytes = (uint32_t)((size_t)p.Nb * p.H * p.W * p.ldx * 4);
  const uint32_t w_bytes = (uint32_t)((size_t)p.K * p.Kg * 4);  // 2 bf16 parts per index
  const __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc((void*)p.x, 0, (int)x_bytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t wr = __builtin_amdgcn_make_buffer_rsrc((void*)p.w, 0, (int)w_bytes, 0x00020000);
  constexpr uint32_t OOB = 0x80000000u;

  const int lrow = lane >> 3, slot = lane & 7;
  const int KT = p.Kg / BK;  // host-checked: C % 32 == 0 (C4: Kg = ⌈R·S / 8⌉·32)
  uint32_t woff[GA];
#pragma unroll
  for (int i = 0; i < GA; ++i) {
    const int row = 8 * (wid + NW * i) + lrow;
    const int chunk = slot ^ ((row >> 1) & 7);
    const int n = n0 + row;
    woff[i] = n < p.K ? (uint32_t)n * (uint32_t)p.Kg * 4u + (uint32_t)chunk * 16u : OOB;
  }
  int rbase[GB];  // fp32 elements
  uint64_t vmask[GB];
  int c4h[C4 ? GB : 1], c4w[C4 ? GB : 1], c4t[C4 ? GB : 1];  // C4: the row's window origin, its lane's tap
  const bool pw_direct = PW && p.sh == 1 && p.sw == 1;
#pragma unroll
  for (int j = 0; j < GB; ++j) {
    const int row = 8 * (wid + NW * j) + lrow;
    const int chunk = slot ^ ((row >> 1) & 7);
    const int m = m0 + row;
    int img = -1, h = 0, w = 0;
    if constexpr (C4) {
      if (m < p.M) {
        const int n = m / (p.P * p.Q);
        const int pq = m - n * p.P * p.Q;
        const int pp = pq / p.Q, qq = pq - pp * p.Q;
        img = n * p.H * p.W;
        h = pp * p.sh - p.ph;
        w = qq * p.sw - p.pw;
      }
      rbase[j] = img;  // pixel index of the image's (0, 0); -1: a row past M
      c4h[j] = h;
      c4w[j] = w;
      c4t[j] = chunk;  // the tap this lane stages in k-tile 0 (kt·8 + chunk later)
      vmask[j] = 0;
      continue;
    }
    if (m < p.M) {
      if (pw_direct) {
        img = m;
      } else {
        const int n = m / (p.P * p.Q);
        const int pq = m - n * p.P * p.Q;
        const int pp = pq / p.Q, qq = pq - pp * p.Q;
        img = n * p.H * p.W;
        h = pp * p.sh - p.ph;
        w = qq * p.sw - p.pw;
      }
    }
    rbase[j] = (img + h * p.W + w) * p.ldx + chunk * 4;
    uint64_t msk = 0;
    if (PW) {
      msk = img >= 0 ? 1ull : 0ull;
    } else if (img >= 0) {
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

  // prep: the source offsets of the next k-tile (called strictly in k order)
  int it_c0 = 0, it_s = 0, it_tap = 0, it_off = 0, p_kt = 0;
  uint32_t poff[L];
  auto prep = [&]() {
    const int kt = p_kt++;
    const uint32_t kb = (uint32_t)kt * 128u;
#pragma unroll
    for (int i = 0; i < GA; ++i) poff[i] = woff[i] + kb;
    if constexpr (C4) {
#pragma unroll
      for (int j = 0; j < GB; ++j) {
        const int t = kt * 8 + c4t[j];
        const int r = t / p.S, sx = t - r * p.S;
        const int h = c4h[j] + r * p.dh, w = c4w[j] + sx * p.dw;
        const bool ok = rbase[j] >= 0 && t < p.R * p.S && (unsigned)h < (unsigned)p.H && (unsigned)w < (unsigned)p.W;
        poff[GA + j] = ok ? (uint32_t)(rbase[j] + h * p.W + w) * 16u : OOB;
      }
      return;
    }
    const int tap = PW ? 0 : it_tap;
    const int tap_off = PW ? kt * BK : it_off + it_c0;
    if (!PW) {
      it_c0 += BK;
      if (it_c0 == p.C) {
        it_c0 = 0;
        ++it_tap;
        if (++it_s == p.S) {
          it_s = 0;
          it_off += (p.dh * p.W - (p.S - 1) * p.dw) * p.ldx;
        } else {
          it_off += p.dw * p.ldx;
        }
      }
    }
#pragma unroll
    for (int j = 0; j < GB; ++j) {
      const bool ok = PW ? (vmask[j] != 0) : ((vmask[j] >> tap) & 1ull);
      poff[GA + j] = ok ? (uint32_t)(rbase[j] + tap_off) * 4u : OOB;
    }
  };
  auto issue = [&](int i, int slotbuf) {
    unsigned char* base = lds + slotbuf * STAGE;
    if (i < GA)
      x3_glds16(wr, base + 8 * (wid + NW * i) * 128, poff[i]);
    else
      x3_glds16(xr, base + (BN + 8 * (wid + NW * (i - GA))) * 128, poff[i]);
  };

  v16f acc[TNI][TMI];
#pragma unroll
  for (int i = 0; i < TNI; ++i)
#pragma unroll
    for (int j = 0; j < TMI; ++j)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[i][j][e] = 0.f;

  const int frow = lane & 31, fh = lane >> 5;
  const int swz = (frow >> 1) & 7;
  // per slice kk (16 reduction indices): A hi chunk 2kk + fh, lo chunk 4 + 2kk + fh; B fp32 chunks
  // 4kk + 2fh and 4kk + 2fh + 1
  int fa_hi[2], fa_lo[2], fb0[2], fb1[2];
#pragma unroll
  for (int kk = 0; kk < 2; ++kk) {
    fa_hi[kk] = frow * 128 + (((2 * kk + fh) ^ swz) << 4);
    fa_lo[kk] = frow * 128 + (((4 + 2 * kk + fh) ^ swz) << 4);
    fb0[kk] = frow * 128 + (((4 * kk + 2 * fh) ^ swz) << 4);
    fb1[kk] = frow * 128 + (((4 * kk + 2 * fh + 1) ^ swz) << 4);
  }
  const int a_row0 = wave_n * (BN / WN), b_row0 = BN + wave_m * (BM / WM);
  // PRO, tap-uniform mode: which taps of this lane's B-fragment rows (pixels) are inside the image
  uint64_t fmask[PRO ? TMI : 1];
  if constexpr (PRO) {
#pragma unroll
    for (int j = 0; j < TMI; ++j) {
      uint64_t msk = ~0ull;
      const int m = m0 + (b_row0 - BN) + 32 * j + frow;
      if (!PW && m < p.M) {
        msk = 0;
        const int n = m / (p.P * p.Q);
        const int pq = m - n * p.P * p.Q;
        const int pp = pq / p.Q, qq = pq - pp * p.Q;
        const int h = pp * p.sh - p.ph, w = qq * p.sw - p.pw;
        for (int r = 0; r < p.R; ++r) {
          const int hh = h + r * p.dh;
          if ((unsigned)hh >= (unsigned)p.H) continue;
          for (int sx = 0; sx < p.S; ++sx) {
            const int ww = w + sx * p.dw;
            if ((unsigned)ww < (unsigned)p.W) msk |= 1ull << (r * p.S + sx);
          }
        }
      }
      fmask[j] = msk;
    }
  }
  int pc_c0 = 0, pc_tap = 0;  // PRO: channel offset / tap of the k-tile compute() multiplies next

  constexpr int PPK = (L + 1) / 2;  // DMA pieces of the next stage per slice
  auto compute = [&](int slotbuf, int nslot, auto issue_on) {
    const unsigned char* base = lds + slotbuf * STAGE;
    v8s ah[2][TNI], al[2][TNI];
    v4f b0[2][TMI], b1[2][TMI];
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
#pragma unroll
      for (int i = 0; i < TNI; ++i) {
        ah[kk][i] = *reinterpret_cast<const v8s*>(base + (a_row0 + 32 * i) * 128 + fa_hi[kk]);
        al[kk][i] = *reinterpret_cast<const v8s*>(base + (a_row0 + 32 * i) * 128 + fa_lo[kk]);
      }
#pragma unroll
      for (int j = 0; j < TMI; ++j) {
        b0[kk][j] = *reinterpret_cast<const v4f*>(base + (b_row0 + 32 * j) * 128 + fb0[kk]);
        b1[kk][j] = *reinterpret_cast<const v4f*>(base + (b_row0 + 32 * j) * 128 + fb1[kk]);
      }
    }
    // PRO: the deferred BN + ReLU of the input, applied to each slice right before its split (slice 1's
    // with slice 1's split, under slice 0's MFMAs); a padded tap of a row reads 0 (pointwise: none)
    const float* scp = pro_s + pc_c0 + 8 * fh;
    bool pvalid[TMI];
    if constexpr (PRO) {
#pragma unroll
      for (int j = 0; j < TMI; ++j) pvalid[j] = PW || ((fmask[j] >> pc_tap) & 1ull);
      x3_pro_slice<TMI>(b0[0], b1[0], scp, pvalid);
      pc_c0 += BK;
      if (pc_c0 == p.C) {
        pc_c0 = 0;
        ++pc_tap;
      }
    }
    // slice 0's B split is exposed; slice 1's is issued right after slice 0's MFMAs so it overlaps
    // them in the matrix pipe (the MFMA only holds vector issue for 8 of its 32 cycles)
    v8s bh[2][TMI], bl[2][TMI];
#pragma unroll
    for (int j = 0; j < TMI; ++j) x3_split8(b0[0][j], b1[0][j], bh[0][j], bl[0][j]);
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
#pragma unroll
      for (int i = 0; i < TNI; ++i) {
#pragma unroll
        for (int j = 0; j < TMI; ++j) {
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah[kk][i], bh[kk][j], acc[i][j], 0, 0, 0);
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(al[kk][i], bh[kk][j], acc[i][j], 0, 0, 0);
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah[kk][i], bl[kk][j], acc[i][j], 0, 0, 0);
        }
        if (decltype(issue_on)::value && i < PPK && kk * PPK + i < L) {
          __builtin_amdgcn_sched_barrier(0);
          issue(kk * PPK + i, nslot);
          __builtin_amdgcn_sched_barrier(0);
        }
      }
#pragma unroll
      for (int q = TNI; q < PPK; ++q)
        if (decltype(issue_on)::value && kk * PPK + q < L) issue(kk * PPK + q, nslot);
      __builtin_amdgcn_sched_barrier(0);
      if (kk == 0) {
        if constexpr (PRO) x3_pro_slice<TMI>(b0[1], b1[1], scp + 16, pvalid);
#pragma unroll
        for (int j = 0; j < TMI; ++j) x3_split8(b0[1][j], b1[1][j], bh[1][j], bl[1][j]);
        __builtin_amdgcn_sched_barrier(0);
      }
    }
  };

  // ---------------------------------------------------------------------------------- main loop
  if constexpr (NS == 2) {  // 2-deep ring: k-tile t + 1 in flight while t is multiplied
    prep();
#pragma unroll
    for (int i = 0; i < L; ++i) issue(i, 0);
    X3_WAIT(0);
    X3_BARRIER();
    int cur = 0;
    for (int t = 0; t + 1 < KT; ++t) {
      prep();
      compute(cur, cur ^ 1, std::true_type{});
      X3_WAIT(0);
      X3_BARRIER();
      cur ^= 1;
    }
    compute(cur, 0, std::false_type{});
  } else {  // 3-deep ring: t + 2 issued while t is multiplied, counted vmcnt keeps one tile in flight
    prep();
#pragma unroll
    for (int i = 0; i < L; ++i) issue(i, 0);
    if (KT > 1) {
      prep();
#pragma unroll
      for (int i = 0; i < L; ++i) issue(i, 1);
      X3_WAIT(L);
    } else {
      X3_WAIT(0);
    }
    X3_BARRIER();
    int cur = 0, nxt = 2;
    for (int t = 0; t + 2 < KT; ++t) {
      prep();
      compute(cur, nxt, std::true_type{});
      X3_WAIT(L);
      X3_BARRIER();
      cur = cur == NS - 1 ? 0 : cur + 1;
      nxt = nxt == NS - 1 ? 0 : nxt + 1;
    }
    if (KT >= 2) {
      compute(cur, 0, std::false_type{});
      X3_WAIT(0);
      X3_BARRIER();
      cur = cur == NS - 1 ? 0 : cur + 1;
    }
    compute(cur, 0, std::false_type{});
  }
  X3_BARRIER();  // every wave is done reading the ring: the epilogue reuses its LDS

  // ---------------------------------------------------------------------------------- epilogue
  // 1. park the fp32 accumulators (+ bias) as a [BM][BN] tile: 16-B chunk c of row r at c ^ (r & CMASK)
  //    (a lane group of 16 consecutive rows writes one logical chunk into 16 distinct bank slots)
  constexpr int CMASK = CPR - 1 < 31 ? CPR - 1 : 31;
  float* et = reinterpret_cast<float*>(lds);
  const int pm = lane & 31;
#pragma unroll
  for (int i = 0; i < TNI; ++i)
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const int nl = a_row0 + 32 * i + 8 * g + 4 * fh;
      float b4[4] = {0.f, 0.f, 0.f, 0.f};
      if (p.bias && n0 + nl < p.K) {
#pragma unroll
        for (int e = 0; e < 4; ++e) b4[e] = p.bias[n0 + nl + e];
      }
#pragma unroll
      for (int j = 0; j < TMI; ++j) {
        const int ml = (b_row0 - BN) + 32 * j + pm;
        *reinterpret_cast<v4f*>(&et[ml * BN + (((nl >> 2) ^ (ml & CMASK)) << 2)]) =
            (v4f){acc[i][j][4 * g] + b4[0], acc[i][j][4 * g + 1] + b4[1], acc[i][j][4 * g + 2] + b4[2],
                  acc[i][j][4 * g + 3] + b4[3]};
      }
    }
  // a full __syncthreads (LDS writes drained, then the barrier): the raw s_barrier used in the main
  // loop is preceded there by X3_WAIT's lgkmcnt(0), but here the other waves READ what this wave just
  // WROTE — on gfx950 s_barrier does not wait for the issuing wave's outstanding ds_writes, and the
  // raw form let the row pass / the statistics fold read stale LDS now and then (fp32 BN statistics
  // off by up to 65 % on a few steps of a training run: tools/convergence.py --check-bn 1)
  __syncthreads();
  // 2. row-major pass: thread (rr, cc) handles channels n0 + 4·cc … +3 of rows rr, rr + RPP, …, so every
  //    global access of a wave-instruction is RPP-row-contiguous 16-B chunks (full 4·BN-byte row segments)
  const int cc = tid % CPR, rr = tid / CPR;
  const int n = n0 + cc * 4;
  const bool nok = n < p.K;  // K % 4 == 0 (host-checked): a 4-channel chunk is all in or all out
  const bool want_stats = p.stats != nullptr;
  float k4[4] = {0.f, 0.f, 0.f, 0.f}, mu[4] = {0.f, 0.f, 0.f, 0.f}, sc4[4] = {0.f, 0.f, 0.f, 0.f},
        sh4[4] = {0.f, 0.f, 0.f, 0.f};
  if (nok) {
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      if (p.shift && !p.bnx) k4[e] = p.shift[n + e];
      if (p.bnx) {
        mu[e] = p.mean[n + e];
        if (!p.bits) { sc4[e] = p.bsc[n + e]; sh4[e] = p.bsh[n + e]; }
      }
    }
  }
  float s4[4] = {0.f, 0.f, 0.f, 0.f}, q4[4] = {0.f, 0.f, 0.f, 0.f};
  const int rmax = p.M - m0 < BM ? p.M - m0 : BM;
  if (nok) {
#pragma unroll 2
    for (int r = rr; r < rmax; r += RPP) {
      const int m = m0 + r;
      int mo = m;  // pixel of the output grid
      if (p.scatter) {
        const int img = m / (p.P * p.Q);
        const int pq = m - img * p.P * p.Q;
        const int pp = pq / p.Q, qq = pq - pp * p.Q;
        mo = (img * p.oH + pp * p.osh + p.ooh) * p.oW + qq * p.osw + p.oow;
      }
      const size_t off = (size_t)mo * p.ldy + n;
      v4f v = *reinterpret_cast<const v4f*>(&et[r * BN + ((cc ^ (r & CMASK)) << 2)]);
      if (p.res) {
        bool live = true;
        size_t roff = off;
        if (p.res_sh) {
          const int gridpix = p.scatter ? p.oH * p.oW : p.P * p.Q;
          const int gw = p.scatter ? p.oW : p.Q;
          const int img = mo / gridpix;
          const int hw = mo - img * gridpix;
          const int hh = hw / gw, ww = hw - hh * gw;
          live = hh % p.res_sh == 0 && ww % p.res_sw == 0;
          roff = ((size_t)(img * p.res_H + hh / p.res_sh) * p.res_W + ww / p.res_sw) * p.ldy + n;
        }
        if (live) v += *reinterpret_cast<const v4f*>(p.res + roff);
      }
      if (p.relu) {
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] = fmaxf(v[e], 0.f);
      }
      if (p.bnx) {
        const v4f xv = *reinterpret_cast<const v4f*>(p.bnx + (size_t)mo * p.K + n);
        unsigned mb;
        if (p.bits) {
          mb = (p.bits[(size_t)mo * (p.K >> 3) + (n >> 3)] >> (n & 7)) & 0xFu;
        } else {
          mb = 0;
#pragma unroll
          for (int e = 0; e < 4; ++e) mb |= (fmaf(xv[e], sc4[e], sh4[e]) > 0.f ? 1u : 0u) << e;
        }
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          v[e] = (mb >> e) & 1u ? v[e] : 0.f;
          s4[e] += v[e];
          q4[e] = fmaf(v[e], xv[e] - mu[e], q4[e]);
        }
      } else if (want_stats) {
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const float a = v[e] - k4[e];
          s4[e] += a;
          q4[e] = fmaf(a, a, q4[e]);
        }
      }
      if (!(p.dbg & 1)) *reinterpret_cast<v4f*>(p.y + off) = v;
    }
  }
  if (want_stats) {  // 3. fold the RPP row groups of each channel through LDS, one atomic per channel
    float* red = reinterpret_cast<float*>(lds + BM * BN * 4);  // [2][RPP][BN] behind the staged tile
    *reinterpret_cast<v4f*>(&red[rr * BN + cc * 4]) = (v4f){s4[0], s4[1], s4[2], s4[3]};
    *reinterpret_cast<v4f*>(&red[(RPP + rr) * BN + cc * 4]) = (v4f){q4[0], q4[1], q4[2], q4[3]};
    __syncthreads();  // (as above: other waves read these partials)
    const int rep = tm % p.R_rep;
    for (int t = tid; t < 2 * BN; t += NT) {
      const int which = t / BN, c = t - which * BN;
      if (n0 + c >= p.K) continue;
      float a = 0.f;
#pragma unroll 4
      for (int g = 0; g < RPP; ++g) a += red[(which * RPP + g) * BN + c];
      atomicAdd(&p.stats[((size_t)which * p.R_rep + rep) * p.K + n0 + c], a);
    }
  }
}

// ---- host side ----
// wave layout `wl`: 0 = the 2-D split (WM × WN = 4 × 2 / 2 × 2), 1 = waves over pixels only (8 × 1 /
// 4 × 1): each wave's split B fragment then feeds all BN / 32 channel blocks (half the split VALU per MFMA).
// ns2: the 2-deep ring (two 128 × 128 or three 128 × 64 blocks share a CU).
template <int MODE, bool PRO = false>
static void launch_x3(int bm, int bn, int wl, int ns2, dim3 g, hipStream_t s, const X3Params& p) {
  if (bm == 128 && bn == 64) {
    hipLaunchKernelGGL((k_conv_x3<128, 64, 4, 1, MODE, 2, PRO>), g, dim3(256), 0, s, p);
  } else if (bm == 128 && ns2) {
    if (wl) hipLaunchKernelGGL((k_conv_x3<128, 128, 4, 1, MODE, 2, PRO>), g, dim3(256), 0, s, p);
    else hipLaunchKernelGGL((k_conv_x3<128, 128, 2, 2, MODE, 2, PRO>), g, dim3(256), 0, s, p);
  } else if (bm == 128) {
    if (wl) hipLaunchKernelGGL((k_conv_x3<128, 128, 4, 1, MODE, 3, PRO>), g, dim3(256), 0, s, p);
    else hipLaunchKernelGGL((k_conv_x3<128, 128, 2, 2, MODE, 3, PRO>), g, dim3(256), 0, s, p);
  } else if (bn == 64) {
    if (wl) hipLaunchKernelGGL((k_conv_x3<256, 64, 8, 1, MODE, 3, PRO>), g, dim3(512), 0, s, p);
    else hipLaunchKernelGGL((k_conv_x3<256, 64, 4, 2, MODE, 3, PRO>), g, dim3(512), 0, s, p);
  } else {
    if (wl) hipLaunchKernelGGL((k_conv_x3<256, 128, 8, 1, MODE, 3, PRO>), g, dim3(512), 0, s, p);
    else hipLaunchKernelGGL((k_conv_x3<256, 128, 4, 2, MODE, 3, PRO>), g, dim3(512), 0, s, p);
  }
}

static bool x3_al(const void* q) { return ((uintptr_t)q & 15) == 0; }

// Tile pin for A/B measurements: BIGDL_CONV_X3_TILE = 1 (256×128), 2 (256×64), 3 (128×128).
static int x3_env_tile() {
  static const int v = [] { const char* e = getenv("BIGDL_CONV_X3_TILE"); return e ? atoi(e) : 0; }();
  return v;
}

// y[M][ldy] (fp32) = conv(x, W) with the epilogues above.  x [Nb][H][W][C] fp32 (C % 32 == 0, 16-B
// aligned), w2 the chunked [hi | lo] split of the KRSC fp32 filter (bigdl_split_bf16x2 of its
// [K·R·S·C / 32][32] view), K % 8 == 0 for statistics / bnbwd (else K % 4).  bm / bn: the tile
// (256 × 128, 256 × 64 or 128 × 128; 0 = heuristic).  osh … oW: the output scatter (1, 1, 0, 0, P, Q =
// none); res_sh … res_W: the strided residual (0 = dense); persist: unused (ABI).  Returns hipError_t.
static int conv_x3_impl(const float* x, const void* w2, const float* bias, const float* res, float* y,
                        float* stats, int R_rep, const float* shift, const float* bnx, const float* mean,
                        const void* bits, const float* bsc, const float* bsh, int Nb, int H, int W, int C,
                        int K, int R, int S, int P, int Q, int sh, int sw, int ph, int pw, int dh, int dw,
                        int relu, int ldy, int bm, int bn, int osh, int osw, int ooh, int oow, int oH,
                        int oW, int res_sh, int res_sw, int res_H, int res_W, int persist, hipStream_t s,
                        const float* pro) {
  const bool c4 = C == 4;  // the padded RGB stem: x [Nb][H][W][4]
  if (pro && (c4 || C > X3_PRO_MAXC || ((uintptr_t)pro & 15) || C % 32)) return (int)hipErrorInvalidValue;
  if (!x || !w2 || !y || Nb <= 0 || C <= 0 || K <= 0 || P <= 0 || Q <= 0 || (C % 32 && !c4) || K % 4 || ldy < K ||
      ldy % 4)
    return (int)hipErrorInvalidValue;
  if (c4 && (R * S > 64 || bnx || osh != 1 || osw != 1 || ooh != 0 || oow != 0 || oH != P || oW != Q || res_sh))
    return (int)hipErrorInvalidValue;
  if (!x3_al(x) || !x3_al(w2) || !x3_al(y) || (res && !x3_al(res)) || (bnx && !x3_al(bnx)))
    return (int)hipErrorInvalidValue;
  if (stats && (R_rep <= 0 || K % 8 || ldy != K || (!bnx && (bias || relu || res)))) return (int)hipErrorInvalidValue;
  if (bnx && (!stats || !mean || relu || bias || (!bits && (!bsc || !bsh)))) return (int)hipErrorInvalidValue;
  const bool pw1 = R == 1 && S == 1 && ph == 0 && pw == 0 && !c4;
  if (!pw1 && R * S > 64) return (int)hipErrorNotSupported;
  if ((size_t)Nb * H * W * C * 4 >= 0x80000000ull || (size_t)K * R * S * C * 4 >= 0x80000000ull)
    return (int)hipErrorInvalidValue;
  const long long Ml = (long long)Nb * P * Q;
  if (Ml > 0x7fffffffLL) return (int)hipErrorInvalidValue;
  X3Params p{};
  {
    const char* e = getenv("BIGDL_X3_DEBUG");
    p.dbg = e ? atoi(e) : 0;
  }
  p.x = x; p.w = (const bf16_t*)w2; p.bias = bias; p.res = res; p.y = y;
  p.Nb = Nb; p.H = H; p.W = W; p.C = C; p.K = K; p.R = R; p.S = S; p.P = P; p.Q = Q;
  p.sh = sh; p.sw = sw; p.ph = ph; p.pw = pw; p.dh = dh; p.dw = dw;
  p.M = (int)Ml; p.Kg = c4 ? (R * S + 7) / 8 * 32 : R * S * C; p.ldx = C; p.ldy = ldy; p.relu = relu;
  p.stats = stats; p.R_rep = stats ? R_rep : 1; p.shift = bnx ? nullptr : shift;
  p.bnx = bnx; p.mean = mean; p.bits = (const uint8_t*)bits; p.bsc = bsc; p.bsh = bsh;
  p.pro = pro;
  if (osh <= 0 || osw <= 0 || ooh < 0 || oow < 0) return (int)hipErrorInvalidValue;
  p.scatter = (osh != 1 || osw != 1 || ooh != 0 || oow != 0 || oH != P || oW != Q) ? 1 : 0;
  p.osh = osh; p.osw = osw; p.ooh = ooh; p.oow = oow; p.oH = oH; p.oW = oW;
  if (p.scatter && ((P - 1) * osh + ooh >= oH || (Q - 1) * osw + oow >= oW)) return (int)hipErrorInvalidValue;
  if (res_sh < 0 || res_sw < 0 || (res_sh > 0) != (res_sw > 0) || (res_sh && !res)) return (int)hipErrorInvalidValue;
  p.res_sh = res_sh; p.res_sw = res_sw; p.res_H = res_H; p.res_W = res_W;
  if (res_sh) {
    const int gh = p.scatter ? oH : P, gw = p.scatter ? oW : Q;
    if (res_H * res_sh < gh || res_W * res_sw < gw || (res_H - 1) * res_sh >= gh || (res_W - 1) * res_sw >= gw)
      return (int)hipErrorInvalidValue;
  }
  const int et = x3_env_tile();
  if (et == 1) { bm = 256; bn = 128; } else if (et == 2) { bm = 256; bn = 64; } else if (et == 3) { bm = 128; bn = 128; }
  if (bm == 0) {
    // measured per ResNet-50 shape (tools/bench_x3.py, profiles/r5_x3_shapes.txt): 3×3 convs run best as
    // two 128 × 128 blocks per CU (2-deep ring, waves over pixels) except the 64-channel ones (256 × 64,
    // 8 × 1); pointwise convs on 256 × 128 / 256 × 64 (4 × 2), the 7² ones as two 128 × 128 blocks per CU
    const bool pw1_ = R == 1 && S == 1 && ph == 0 && pw == 0 && !c4;
    if (c4) {
      bm = 256;
      bn = K <= 64 ? (64 | 0x100) : 128;
    } else if (!pw1_) {
      bm = K <= 64 ? 256 : 128;
      bn = K <= 64 ? (64 | 0x100) : (128 | 0x300);
    } else if (K <= 64) {
      bm = 256;
      bn = 64;
    } else if (Ml <= 2 * 12544) {
      bm = 128;
      bn = 128 | 0x300;
    } else {
      bm = 256;
      bn = 128;
    }
  }
  int wl = (bn >> 8) & 1;  // bit 8 of bn: the pixels-only wave layout
  const int ns2 = (bn >> 9) & 1;  // bit 9: the 2-deep ring (128 × 128 tile: two blocks per CU)
  bn &= 0xFF;
  if (bn == 0) bn = K <= 64 ? 64 : 128;
  if (!((bm == 256 && (bn == 64 || bn == 128)) || (bm == 128 && (bn == 128 || bn == 64)))) return (int)hipErrorInvalidValue;
  static const int wl_env = [] { const char* e = getenv("BIGDL_CONV_X3_WL"); return e ? atoi(e) : -1; }();
  if (wl_env >= 0) wl = wl_env;
  p.tiles_n = (K + bn - 1) / bn;
  const long long tiles = (Ml + bm - 1) / bm * p.tiles_n;
  if (tiles > 0x7fffffff) return (int)hipErrorInvalidValue;
  (void)persist;  // (a persistent tile-stream variant measured no gain: removed)
  if (c4) launch_x3<2>(bm, bn, wl, ns2, dim3((unsigned)tiles), s, p);
  else if (pro && pw1) launch_x3<3, true>(bm, bn, wl, ns2, dim3((unsigned)tiles), s, p);
  else if (pro) launch_x3<1, true>(bm, bn, wl, ns2, dim3((unsigned)tiles), s, p);
  else if (pw1) launch_x3<3>(bm, bn, wl, ns2, dim3((unsigned)tiles), s, p);
  else launch_x3<1>(bm, bn, wl, ns2, dim3((unsigned)tiles), s, p);
  BIGDL_CHECK_LAUNCH();
}

BIGDL_EXPORT int bigdl_conv_x3(const float* x, const void* w2, const float* bias, const float* res, float* y,
                               float* stats, int R_rep, const float* shift, const float* bnx, const float* mean,
                               const void* bits, const float* bsc, const float* bsh, int Nb, int H, int W, int C,
                               int K, int R, int S, int P, int Q, int sh, int sw, int ph, int pw, int dh, int dw,
                               int relu, int ldy, int bm, int bn, int osh, int osw, int ooh, int oow, int oH,
                               int oW, int res_sh, int res_sw, int res_H, int res_W, int persist, hipStream_t s) {
  return conv_x3_impl(x, w2, bias, res, y, stats, R_rep, shift, bnx, mean, bits, bsc, bsh, Nb, H, W, C, K, R, S, P, Q,
                      sh, sw, ph, pw, dh, dw, relu, ldy, bm, bn, osh, osw, ooh, oow, oH, oW, res_sh, res_sw, res_H,
                      res_W, persist, s, nullptr);
}

// bigdl_conv_x3 whose input x is the INPUT of a training BN + ReLU (the deferred BN output): the conv
// reads relu(x·pro[c] + pro[C + c]), pro = the BN's [scale | shift] (C % 32 == 0, C ≤ 512).
BIGDL_EXPORT int bigdl_conv_x3_pro(const float* x, const void* w2, const float* pro, const float* bias,
                                   const float* res, float* y, float* stats, int R_rep, const float* shift,
                                   const float* bnx, const float* mean, const void* bits, const float* bsc,
                                   const float* bsh, int Nb, int H, int W, int C, int K, int R, int S, int P, int Q,
                                   int sh, int sw, int ph, int pw, int dh, int dw, int relu, int ldy, int bm, int bn,
                                   int osh, int osw, int ooh, int oow, int oH, int oW, hipStream_t s) {
  if (!pro) return (int)hipErrorInvalidValue;
  return conv_x3_impl(x, w2, bias, res, y, stats, R_rep, shift, bnx, mean, bits, bsc, bsh, Nb, H, W, C, K, R, S, P, Q,
                      sh, sw, ph, pw, dh, dw, relu, ldy, bm, bn, osh, osw, ooh, oow, oH, oW, 0, 0, 0, 0, 0, s, pro);
}
