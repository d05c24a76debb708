// Implicit-GEMM convolution, large-tile family: v_mfma_f32_32x32x16_bf16, 8 waves (or 4 for the
// 128x128 tile), operands staged global -> LDS by the LDS-DMA path (buffer_load_dwordx4 ... lds),
// a 3-deep LDS ring with counted vmcnt and raw s_barrier so one k-tile stays in flight across every
// barrier (cdna_hip_programming.md §5 'Pipelining across barriers', T3/T4).  Same GEMM view and
// epilogue as conv_igemm.hip (reference: SpatialConvolution.updateOutput,
// DL/nn/SpatialConvolution.scala:253-362; no im2col is materialised):
//   D[n = out channel][m = output pixel] = Σ_k W[n][k] · X̂[m][k],   k = (r, s, c),  BK = 64.
// MFMA A = weights (rows = channels), B = gathered activations (cols = pixels): lane l of a 32x32
// accumulator holds pixel (l & 31) and channels (r & 3) + 8 (r >> 2) + 4 (l >> 5) — four runs of 4
// consecutive channels, parked as 8-B LDS writes for the shared row-major store pass.
//
// Why: the 4-wave 128x128 kernel writes every operand byte through VGPRs into LDS (ds_write_b128
// moves ≈79 B/clk/CU), which with the fragment reads left the LDS busier than the MFMA pipe; the
// DMA path skips the VGPR round trip and the larger tile halves the operand bytes per FLOP.
//
// Padding: the buffer descriptor's bounds check returns zeros for an out-of-range offset, and the
// LDS-DMA form writes those zeros to LDS — conv padding, the M tail and the channel tail need no
// branch.  The LDS image is lane-linear per wave-instruction (8 rows x 128 B); the XOR swizzle
// chunk ^ ((row >> 1) & 7) is applied on the per-lane SOURCE address and on the fragment read
// (rule 21).  It makes the 32x32x16 fragment reads conflict-free: a ds_read_b128 lane group holds 16
// rows distinct mod 16 at one chunk, and (row & 1, (row >> 1) & 7) spreads them over all 16 slots
// of the 256-B bank window.
//
// Modes (as conv_igemm.hip): 1 = tap-uniform FAST gather (C % 64 == 0, R·S ≤ 64), 3 = pointwise.
#include "conv_params.h"
#include <type_traits>

typedef float v16f __attribute__((ext_vector_type(16)));

#define X8_WAIT(n) asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)" ::"n"(n) : "memory")
#define X8_BARRIER()                   \
  do {                                 \
    asm volatile("" ::: "memory");     \
    __builtin_amdgcn_s_barrier();      \
    asm volatile("" ::: "memory");     \
  } while (0)

typedef __attribute__((address_space(3))) void lds_void_t;

// One 16-B-per-lane LDS-DMA piece (buffer_load_dwordx4 ... lds): lane l's 16 bytes land at
// lds + 16·l.  A non-template device function: inside the kernel template the builtin fails host-side
// template substitution and hipcc silently drops the kernel's launch stub.
__device__ __forceinline__ void glds16(__amdgpu_buffer_rsrc_t r, void* lds, uint32_t voff) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (lds_void_t*)lds, 16, voff, 0, 0, 0);
}

// ILV = 1: the interleaved main loop — the next k-tile's LDS-DMA pieces are issued between the
// MFMA groups of the current one (and the fragments of k-slice kk + 1 are read while slice kk's
// MFMAs run), with sched_barrier fences pinning the order; ILV = 0 issues every piece of the stage
// up front, then the 16 MFMAs.
template <int BM, int BN, int WM, int WN, int MODE, int ILV = 0>
__global__ void __launch_bounds__(64 * WM * WN, 1) k_conv_x8(ConvParams p) {
  static_assert(MODE == 1 || MODE == 3, "FAST / pointwise gathers only");
  constexpr bool PW = MODE == 3;
  constexpr int NT = 64 * WM * WN, NW = WM * WN;
  constexpr int BK = 64;
  // LDS ring depth: 3; the 256 × 256 tile (1.5× the FLOP per staged byte of 256 × 128 — the L2 → LDS
  // feed, not the MFMA, bounds these convs) has room for 2 (2 × 64 KiB, its epilogue takes all 160)
  constexpr int NS = BN == 256 ? 2 : 3;
  constexpr int STAGE = (BM + BN) * 128;       // bytes per ring slot (128-B rows)
  constexpr int GA = BN / 8 / NW, GB = BM / 8 / NW;  // 8-row DMA groups per wave: weights, activations
  static_assert(GA * NW * 8 == BN && GB * NW * 8 == BM, "tile rows must split evenly over the waves");
  constexpr int L = GA + GB;                   // DMA instructions per wave per k-tile
  constexpr int TMI = BM / WM / 32, TNI = BN / WN / 32;
  static_assert(TMI >= 1 && TNI >= 1, "wave tile below 32x32");
  constexpr int EPI = BM * BN * 2 + 2 * (NT / (BN / 8)) * BN * 4;
  constexpr int LDS_BYTES = NS * STAGE > EPI ? NS * STAGE : EPI;
  __shared__ __attribute__((aligned(16))) unsigned char lds[LDS_BYTES];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wave_m = wid % WM, wave_n = wid / WM;
  const long long grp = blockIdx.y;
  if (grp) {
    p.x += grp * p.gx;
    p.w += grp * p.gw;
    p.y += grp * p.gy;
    if (p.bias) p.bias += grp * p.gy;
  }
  const int tile = xcd_remap(blockIdx.x, gridDim.x);
  const int tm = tile / p.tiles_n, tn = tile - tm * p.tiles_n;
  const int m0 = tm * BM, n0 = tn * BN;
  // the store pass's statistics shift for this thread's 8 channels, fetched before the main loop
  float skp[8];
  {
    const int ns = n0 + (tid % (BN / 8)) * 8;
#pragma unroll
    for (int e = 0; e < 8; ++e)
      skp[e] = (p.stat_shift && p.stats && !p.bnx && ns + e < p.K) ? p.stat_shift[ns + e] : 0.f;
  }

  const uint32_t x_bytes = (uint32_t)(((size_t)p.Nb * p.H * p.W * p.ldx - grp * p.gx) * 2);
  const uint32_t w_bytes = (uint32_t)((size_t)p.K * p.ldw * 2);
  const __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc((void*)p.x, 0, (int)x_bytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t wr = __builtin_amdgcn_make_buffer_rsrc((void*)p.w, 0, (int)w_bytes, 0x00020000);
  constexpr uint32_t OOB = 0x80000000u;  // + any k offset stays past num_records (< 2 GiB)

  // per-lane DMA source state: lane l of a group covers row 8g + (l >> 3), LDS slot l & 7, which
  // holds source chunk slot ^ ((row >> 1) & 7)
  const int lrow = lane >> 3, slot = lane & 7;
  uint32_t woff[GA];
#pragma unroll
  for (int i = 0; i < GA; ++i) {
    const int row = 8 * (wid + NW * i) + lrow;
    const int chunk = slot ^ ((row >> 1) & 7);
    const int n = n0 + row;
    woff[i] = n < p.K ? (uint32_t)n * (uint32_t)p.ldw * 2u + (uint32_t)chunk * 16u : OOB;
  }
  int rbase[GB];
  uint64_t vmask[GB];
  const bool pw_direct = PW && p.sh == 1 && p.sw == 1;
#pragma unroll
  for (int j = 0; j < GB; ++j) {
    const int row = 8 * (wid + NW * j) + lrow;
    const int chunk = slot ^ ((row >> 1) & 7);
    const int m = m0 + row;
    int img = -1, h = 0, w = 0;
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
    rbase[j] = (img + h * p.W + w) * p.ldx + chunk * 8;
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

  const int KT = p.Kg / BK;  // host-checked: Kg % 64 == 0 (C % 64 == 0)
  // wave-uniform (tap, channel) iterator of the FAST gather, advanced once per staged k-tile
  int it_c0 = 0, it_s = 0, it_tap = 0, it_off = 0;
  auto stage = [&](int kt, int slotbuf) {
    unsigned char* base = lds + slotbuf * STAGE;
    const uint32_t kb2 = (uint32_t)(kt * BK) * 2u;
#pragma unroll
    for (int i = 0; i < GA; ++i) {
      glds16(wr, base + 8 * (wid + NW * i) * 128, woff[i] + kb2);
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
      unsigned char* dst = base + (BN + 8 * (wid + NW * j)) * 128;
      const bool ok = PW ? (vmask[j] != 0) : ((vmask[j] >> tap) & 1ull);
      const uint32_t off = ok ? (uint32_t)(rbase[j] + tap_off) * 2u : OOB;
      glds16(xr, dst, off);
    }
  };

  // ILV: the stage split in two — prep() advances the tap iterator and computes every piece's source
  // offset, issue(i) sends piece i (weights first, then activation row groups)
  uint32_t poff[L];
  auto prep = [&](int kt) {
    const uint32_t kb2 = (uint32_t)(kt * BK) * 2u;
#pragma unroll
    for (int i = 0; i < GA; ++i) poff[i] = woff[i] + kb2;
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
      poff[GA + j] = ok ? (uint32_t)(rbase[j] + tap_off) * 2u : OOB;
    }
  };
  auto issue = [&](int i, int slotbuf) {
    unsigned char* base = lds + slotbuf * STAGE;
    if (i < GA)
      glds16(wr, base + 8 * (wid + NW * i) * 128, poff[i]);
    else
      glds16(xr, base + (BN + 8 * (wid + NW * (i - GA))) * 128, poff[i]);
  };

  v16f acc[TNI][TMI];
#pragma unroll
  for (int i = 0; i < TNI; ++i)
#pragma unroll
    for (int j = 0; j < TMI; ++j)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[i][j][e] = 0.f;

  // fragment read offsets: row (lane & 31) of a 32-row block, chunk kk·2 + (lane >> 5); the swizzle
  // term depends on the lane only (every block starts at a multiple of 32 rows)
  const int frow = lane & 31, fh = lane >> 5;
  int foff[BK / 16];
#pragma unroll
  for (int kk = 0; kk < BK / 16; ++kk) foff[kk] = frow * 128 + (((kk * 2 + fh) ^ ((frow >> 1) & 7)) << 4);
  const int a_row0 = wave_n * (BN / WN), b_row0 = BN + wave_m * (BM / WM);

  auto compute = [&](int slotbuf) {
    const unsigned char* base = lds + slotbuf * STAGE;
#pragma unroll
    for (int kk = 0; kk < BK / 16; ++kk) {
      v8s af[TNI], bfr[TMI];
#pragma unroll
      for (int i = 0; i < TNI; ++i)
        af[i] = *reinterpret_cast<const v8s*>(base + (a_row0 + 32 * i) * 128 + foff[kk]);
#pragma unroll
      for (int j = 0; j < TMI; ++j)
        bfr[j] = *reinterpret_cast<const v8s*>(base + (b_row0 + 32 * j) * 128 + foff[kk]);
#pragma unroll
      for (int i = 0; i < TNI; ++i)
#pragma unroll
        for (int j = 0; j < TMI; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
    }
  };

  // interleaved body: fragments of slice kk+1 in flight during slice kk's MFMAs; the L pieces of
  // the next stage spread over the four slices (PPK per slice)
  constexpr int PPK = (L + 3) / 4;
  static_assert(4 * PPK >= L && BK / 16 == 4, "every piece of the next stage is issued in the four slices");
  auto compute_ilv = [&](int slotbuf, int nslot, auto issue_on) {
    const unsigned char* base = lds + slotbuf * STAGE;
    v8s af[2][TNI], bfr[2][TMI];
#pragma unroll
    for (int i = 0; i < TNI; ++i) af[0][i] = *reinterpret_cast<const v8s*>(base + (a_row0 + 32 * i) * 128 + foff[0]);
#pragma unroll
    for (int j = 0; j < TMI; ++j) bfr[0][j] = *reinterpret_cast<const v8s*>(base + (b_row0 + 32 * j) * 128 + foff[0]);
#pragma unroll
    for (int kk = 0; kk < BK / 16; ++kk) {
      const int c = kk & 1, n = c ^ 1;
      if (kk + 1 < BK / 16) {
#pragma unroll
        for (int i = 0; i < TNI; ++i)
          af[n][i] = *reinterpret_cast<const v8s*>(base + (a_row0 + 32 * i) * 128 + foff[kk + 1]);
#pragma unroll
        for (int j = 0; j < TMI; ++j)
          bfr[n][j] = *reinterpret_cast<const v8s*>(base + (b_row0 + 32 * j) * 128 + foff[kk + 1]);
      }
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int i = 0; i < TNI; ++i) {
#pragma unroll
        for (int j = 0; j < TMI; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[c][i], bfr[c][j], acc[i][j], 0, 0, 0);
        if (decltype(issue_on)::value && i < PPK && kk * PPK + i < L) {
          __builtin_amdgcn_sched_barrier(0);
          issue(kk * PPK + i, nslot);
          __builtin_amdgcn_sched_barrier(0);
        }
      }
      // a slice has fewer MFMA groups (TNI) than pieces to place (PPK, e.g. the 256x64 tile: TNI 1,
      // PPK 2): the rest of this slice's pieces go after its MFMAs — every piece is issued exactly once
#pragma unroll
      for (int q = TNI; q < PPK; ++q)
        if (decltype(issue_on)::value && kk * PPK + q < L) issue(kk * PPK + q, nslot);
      __builtin_amdgcn_sched_barrier(0);
    }
  };

  // 3-deep ring: tile t+2 is issued before tile t is multiplied; the wait after the MFMAs retires
  // only tile t+1 (counted vmcnt = L), and the barrier then publishes it to every wave and frees the
  // slot just read for the next issue.
  if constexpr (NS == 2) {
    // 2-deep ring: the whole next k-tile is requested before this one's MFMAs (all of its compute
    // time to land), then a full wait and the barrier that also frees the slot just read
    stage(0, 0);
    X8_WAIT(0);
    X8_BARRIER();
    int cur = 0;
    for (int t = 0; t + 1 < KT; ++t) {
      stage(t + 1, cur ^ 1);
      compute_ilv(cur, -1, std::false_type{});
      X8_WAIT(0);
      X8_BARRIER();
      cur ^= 1;
    }
    compute_ilv(cur, -1, std::false_type{});
    X8_BARRIER();
  } else if constexpr (ILV == 1) {
    prep(0);
#pragma unroll
    for (int i = 0; i < L; ++i) issue(i, 0);
    if (KT > 1) {
      prep(1);
#pragma unroll
      for (int i = 0; i < L; ++i) issue(i, 1);
      X8_WAIT(L);
    } else {
      X8_WAIT(0);
    }
    X8_BARRIER();
    int cur = 0, nxt = 2;
    for (int t = 0; t + 2 < KT; ++t) {
      prep(t + 2);
      compute_ilv(cur, nxt, std::true_type{});
      X8_WAIT(L);
      X8_BARRIER();
      cur = cur == NS - 1 ? 0 : cur + 1;
      nxt = nxt == NS - 1 ? 0 : nxt + 1;
    }
    if (KT >= 2) {
      compute_ilv(cur, -1, std::false_type{});
      X8_WAIT(0);
      X8_BARRIER();
      cur = cur == NS - 1 ? 0 : cur + 1;
    }
    compute_ilv(cur, -1, std::false_type{});
    X8_BARRIER();
  } else {
  stage(0, 0);
  if (KT > 1) {
    stage(1, 1);
    X8_WAIT(L);
  } else {
    X8_WAIT(0);
  }
  X8_BARRIER();
  // steady state in one branch-free body (a tail branch inside the loop makes hipcc copy every
  // accumulator at the join); the last two tiles are peeled
  int cur = 0, nxt = 2;
  for (int t = 0; t + 2 < KT; ++t) {
    stage(t + 2, nxt);
    compute(cur);
    X8_WAIT(L);
    X8_BARRIER();
    cur = cur == NS - 1 ? 0 : cur + 1;
    nxt = nxt == NS - 1 ? 0 : nxt + 1;
  }
  if (KT >= 2) {
    compute(cur);
    X8_WAIT(0);
    X8_BARRIER();
    cur = cur == NS - 1 ? 0 : cur + 1;
  }
  compute(cur);
  X8_BARRIER();  // the epilogue reuses the ring's LDS
  }

  // fp32 output (bf16x3 path): four consecutive channels per register run → float4 stores
  const int pm = lane & 31;
  if (p.y32) {
#pragma unroll
    for (int i = 0; i < TNI; ++i)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int n = n0 + a_row0 + 32 * i + 8 * g + 4 * fh;
        if (n >= p.K) continue;
        float b4[4] = {0.f, 0.f, 0.f, 0.f};
        if (p.bias)
#pragma unroll
          for (int e = 0; e < 4; ++e) b4[e] = p.bias[n + e];
#pragma unroll
        for (int j = 0; j < TMI; ++j) {
          const int m = m0 + (b_row0 - BN) + 32 * j + pm;
          if (m >= p.M) continue;
          float4 v = make_float4(acc[i][j][4 * g] + b4[0], acc[i][j][4 * g + 1] + b4[1], acc[i][j][4 * g + 2] + b4[2],
                                 acc[i][j][4 * g + 3] + b4[3]);
          if (p.res32) {
            const float4 r = *reinterpret_cast<const float4*>(p.res32 + (size_t)m * p.ldy + n);
            v = make_float4(v.x + r.x, v.y + r.y, v.z + r.z, v.w + r.w);
          }
          if (p.relu) v = make_float4(fmaxf(v.x, 0.f), fmaxf(v.y, 0.f), fmaxf(v.z, 0.f), fmaxf(v.w, 0.f));
          *reinterpret_cast<float4*>(p.y32 + (size_t)m * p.ldy + n) = v;
        }
      }
    return;
  }

  // park the tile as bf16 [BM][BN] (chunk ^ (row & CMASK) swizzle of conv_store_pass)
  constexpr int CMASK = (BN / 8 - 1) & 15;
  bf16_t* et = reinterpret_cast<bf16_t*>(lds);
#pragma unroll
  for (int i = 0; i < TNI; ++i)
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const int nl = a_row0 + 32 * i + 8 * g + 4 * fh;
      float b4[4] = {0.f, 0.f, 0.f, 0.f};
      if (p.bias)
#pragma unroll
        for (int e = 0; e < 4; ++e) b4[e] = (n0 + nl + e < p.K) ? p.bias[n0 + nl + e] : 0.f;
#pragma unroll
      for (int j = 0; j < TMI; ++j) {
        const int ml = (b_row0 - BN) + 32 * j + pm;
        const uint32_t lo = (uint32_t)f2bf(acc[i][j][4 * g] + b4[0]) | ((uint32_t)f2bf(acc[i][j][4 * g + 1] + b4[1]) << 16);
        const uint32_t hi = (uint32_t)f2bf(acc[i][j][4 * g + 2] + b4[2]) | ((uint32_t)f2bf(acc[i][j][4 * g + 3] + b4[3]) << 16);
        *reinterpret_cast<uint2*>(&et[ml * BN + (((nl >> 3) ^ (ml & CMASK)) << 3) + (nl & 4)]) = make_uint2(lo, hi);
      }
    }
  __syncthreads();
  conv_store_pass<BM, BN, NT>(p, et, tid, m0, n0, tm, false, skp);
}

// ---- host side ----
bool conv_x8_ok(int mode, int bm, int bn, const ConvParams& p) {
  if (mode != 1 && mode != 3) return false;
  if (!((bm == 256 && (bn == 64 || bn == 128 || bn == 256)) || (bm == 128 && bn == 128))) return false;
  if (p.cdup || p.C % 64 || p.Kg % 64 || p.ldx % 8 || p.ldw % 8) return false;
  if (p.T != 1 || p.KT != 1 || p.ax) return false;
  if (mode == 1 && p.R * p.S > 64) return false;
  return true;
}

template <int MODE, int ILV>
static void launch_x8(int bm, int bn, dim3 g, hipStream_t s, const ConvParams& p) {
  if (bm == 128)
    hipLaunchKernelGGL((k_conv_x8<128, 128, 2, 2, MODE, ILV>), g, dim3(256), 0, s, p);
  else if (bn == 256)
    hipLaunchKernelGGL((k_conv_x8<256, 256, 4, 2, MODE, ILV>), g, dim3(512), 0, s, p);
  else if (bn == 64)
    hipLaunchKernelGGL((k_conv_x8<256, 64, 4, 2, MODE, ILV>), g, dim3(512), 0, s, p);
  else
    hipLaunchKernelGGL((k_conv_x8<256, 128, 4, 2, MODE, ILV>), g, dim3(512), 0, s, p);
}

// BIGDL_CONV_X8_ILV=1 selects the interleaved main loop (A/B)
static int x8_ilv() {
  static const int v = [] { const char* e = getenv("BIGDL_CONV_X8_ILV"); return e ? atoi(e) : 1; }();
  return v;
}

int conv_x8_launch(const ConvParams& p, int mode, int bm, int bn, dim3 grid, hipStream_t s) {
  if (!conv_x8_ok(mode, bm, bn, p)) return (int)hipErrorNotSupported;
  if (x8_ilv()) {
    if (mode == 3) launch_x8<3, 1>(bm, bn, grid, s, p);
    else launch_x8<1, 1>(bm, bn, grid, s, p);
  } else {
    if (mode == 3) launch_x8<3, 0>(bm, bn, grid, s, p);
    else launch_x8<1, 0>(bm, bn, grid, s, p);
  }
  return (int)hipGetLastError();
}
