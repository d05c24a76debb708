// 3×3 / stride-1 / pad-1 convolution of 64 → 64 channels (ResNet-50 stage 1, its forward and its
// stride-1 data gradient) as a PERSISTENT halo-patch kernel:
//   * the whole filter (9 taps × 64 out-channels × 64 in-channels, 72 KiB bf16) is staged into the
//     LDS once per workgroup and stays resident while the workgroup walks its row tiles;
//   * a tile is 128 consecutive output pixels (NHWC order: ≤ 4 image rows at W = 56); its input is
//     the band of input rows they touch plus one halo row above and below — ≤ 6 rows × W pixels of
//     128 B (all 64 channels) — loaded ONCE by LDS-DMA (buffer_load … lds) instead of once per tap:
//     the implicit-GEMM gather of conv_igemm.hip / conv_mfma32.hip stages every input pixel 9 times,
//     and at these shapes that L2 → LDS feed (≈55 GB/s per CU measured, profiles/r5_conv_pmc.txt),
//     not the MFMA, set the time (64→64 3×3 at 56²: ~110 µs for 59 GFLOP);
//   * the next tile's band is requested into the second patch buffer before this tile's MFMAs, so
//     the DMA runs under the compute and the epilogue.
// Conv padding: the band holds whole image rows of the flattened (n·H + h) row index; a tap whose
// row or column falls outside the image reads a zero row kept in the LDS.  GEMM view as in
// conv_mfma32.hip: A = weights (rows = out-channels), B = pixels, v_mfma_f32_32x32x16_bf16, the
// XOR swizzle chunk ^ ((row >> 1) & 7) on every 128-B row (weights: row = out-channel, band: row =
// band pixel — 16 consecutive output pixels read 16 consecutive band pixels, conflict-free).  The
// epilogue is the shared conv_store_pass (bias, residual, ReLU, BN statistics, BN-backward).
// Reference: SpatialConvolution.updateOutput / updateGradInput (DL/nn/SpatialConvolution.scala:
// 253-434); the layer it serves: ResNet-50 bottleneck conv2 at 56² (DL/models/resnet/ResNet.scala).
#include "conv_params.h"
#include <type_traits>

typedef float v16f __attribute__((ext_vector_type(16)));

// vmcnt(0) expcnt(7) lgkmcnt(0) as the builtin: hipcc then knows nothing is outstanding after it (an asm
// wait is invisible to its wait-count pass, which then re-drained vmcnt — the next band — every tile)
#define PT_WAIT0() __builtin_amdgcn_s_waitcnt(0x0070)

// One 16-B-per-lane LDS-DMA piece (global_load_lds_dwordx4; lane l's 16 bytes land at ldst + 16·l) as
// inline asm (cdna_hip_programming.md §5.7 item 1): hipcc cannot tell these LDS writes from the
// fragment reads of the other band and, with the builtin, drained them (s_waitcnt vmcnt(0)) before
// the first ds_read of every tile; completion is waited for by hand (PT_WAIT0, then a barrier).
__device__ __forceinline__ void pt_dma16(const void* gsrc, const void* lds_dst) {
  const uint32_t ldst = __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)lds_dst);
  unsigned keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
               : "=&s"(keep)
               : "v"(gsrc), "s"(ldst)
               : "memory");
}

constexpr int PT_BM = 128;                              // output pixels per tile (= SBM)
constexpr int PT_NT = 256;                              // 4 waves, 32 pixels × 64 channels each
constexpr int PT_ROWS = 336;                            // band capacity in pixels (6 rows of 56)
constexpr int PT_WB = 9 * 64 * 128;                     // resident filter bytes
constexpr int PT_PB = PT_ROWS * 128;                    // one band buffer
// LDS: filter + two bands + one zero row = 159,872 B (one workgroup per CU)

__global__ void __launch_bounds__(PT_NT, 1) k_conv_patch64(ConvParams p, int ntiles, int prow) {
  // One LDS array (cdna_hip_programming.md §5 trap 4a): filter | band 0 | band 1 | zero row.
  __shared__ __attribute__((aligned(16))) unsigned char lds[PT_WB + 2 * PT_PB + 128];
  unsigned char* const wl = lds;
  unsigned char* const band0 = lds + PT_WB;
  unsigned char* const band1 = lds + PT_WB + PT_PB;
  unsigned char* const zrow = lds + PT_WB + 2 * PT_PB;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int frow = lane & 31, fh = lane >> 5;
  if (tid < 8) *reinterpret_cast<uint4*>(zrow + 16 * tid) = make_uint4(0, 0, 0, 0);

  const int HW = p.H * p.W;
  const uint32_t npix = (uint32_t)p.Nb * (uint32_t)HW;
  const int lrow = lane >> 3, slot = lane & 7;
  const char* xg = reinterpret_cast<const char*>(p.x);
  const char* wg = reinterpret_cast<const char*>(p.w);

  // the resident filter: LDS row t·64 + n = tap t, out-channel n (72 pieces of 8 rows, 18 a wave)
#pragma unroll 6
  for (int i = 0; i < 18; ++i) {
    const int piece = wid + 4 * i;
    const int row = piece * 8 + lrow;
    const int t = row >> 6, n = row & 63;
    const int chunk = slot ^ ((n >> 1) & 7);
    pt_dma16(wg + (size_t)n * p.ldw * 2 + t * 128 + chunk * 16, wl + piece * 1024);
  }
  // one tile's input band: band pixel q is flattened input pixel (first output row − 1)·W + q; a band
  // row outside the tensor is fetched from pixel 0 instead (only padded taps — the zero row — map there)
  const int npieces = (prow + 7) >> 3;
  auto load_band = [&](int tile, unsigned char* dst) {
    const int r0 = (tile * PT_BM) / p.W - 1;
    const long long g0 = (long long)r0 * p.W;
    for (int i = wid; i < npieces; i += 4) {
      const int q = i * 8 + lrow;
      const long long gp = g0 + q;
      const int chunk = slot ^ ((q >> 1) & 7);
      const long long src = (gp >= 0 && gp < (long long)npix) ? gp * 128 + chunk * 16 : chunk * 16;
      pt_dma16(xg + src, dst + i * 1024);
    }
  };

  // this thread's statistics shift (8 channels of the store pass), fetched once
  float skp[8];
  {
    const int ns = (tid & 7) * 8;
#pragma unroll
    for (int e = 0; e < 8; ++e) skp[e] = (p.stat_shift && p.stats && !p.bnx) ? p.stat_shift[ns + e] : 0.f;
  }
  // bias of this lane's accumulator channels (n = 32 i + 8 g + 4 fh + e)
  float bv[2][4][4];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int g = 0; g < 4; ++g)
#pragma unroll
      for (int e = 0; e < 4; ++e) bv[i][g][e] = p.bias ? p.bias[32 * i + 8 * g + 4 * fh + e] : 0.f;
  const int aswz = (frow >> 1) & 7;  // weight-row swizzle of this lane's fragment rows

  // one tile from band `CUR` (its successor's band is requested into the other buffer first)
  auto do_tile = [&](int tile, auto CUR) {
    unsigned char* bcur = CUR.value == 0 ? band0 : band1;
    unsigned char* bnxt = CUR.value == 0 ? band1 : band0;
    const int nxt_tile = tile + (int)gridDim.x;
    if (nxt_tile < ntiles) load_band(nxt_tile, bnxt);  // its last reader finished at the previous loop-end barrier

    const int m0 = tile * PT_BM;
    const int r0 = m0 / p.W - 1;
    const int m = m0 + 32 * wid + frow;
    const bool mlive = m < p.M;
    const int gr = m / p.W, w = m - gr * p.W, h = gr % p.H;
    const int qb = (gr - r0) * p.W + w;  // band pixel of tap (1, 1)
    const unsigned char* bp[9];
    int bsw[9];
#pragma unroll
    for (int r = 0; r < 3; ++r)
#pragma unroll
      for (int s2 = 0; s2 < 3; ++s2) {
        const int hh = h + r - 1, ww = w + s2 - 1;
        const bool ok = mlive && (unsigned)hh < (unsigned)p.H && (unsigned)ww < (unsigned)p.W;
        const int q = qb + (r - 1) * p.W + (s2 - 1);
        bp[3 * r + s2] = ok ? bcur + q * 128 : zrow;
        bsw[3 * r + s2] = ok ? ((q >> 1) & 7) : 0;
      }
    v16f acc[2];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[i][e] = 0.f;
    // 9 taps × 4 k-slices of 16 channels: a whole tap's fragments (12 reads) are requested one tap
    // ahead, so each read has a tap's 8 MFMAs (≈256 cycles) to land
    auto rd_a = [&](int t, int kk, int i) -> v8s {
      const int c = kk * 2 + fh;
      return *reinterpret_cast<const v8s*>(wl + t * 8192 + (32 * i + frow) * 128 + ((c ^ aswz) << 4));
    };
    auto rd_b = [&](int t, int kk) -> v8s {
      const int c = kk * 2 + fh;
      return *reinterpret_cast<const v8s*>(bp[t] + ((c ^ bsw[t]) << 4));
    };
    v8s fa[2][4][2], fb[2][4];
#pragma unroll
    for (int kk = 0; kk < 4; ++kk) {
      fa[0][kk][0] = rd_a(0, kk, 0);
      fa[0][kk][1] = rd_a(0, kk, 1);
      fb[0][kk] = rd_b(0, kk);
    }
#pragma unroll
    for (int t = 0; t < 9; ++t) {
      const int cb = t & 1, nb = cb ^ 1;
      __builtin_amdgcn_sched_barrier(0);
      if (t + 1 < 9) {
#pragma unroll
        for (int kk = 0; kk < 4; ++kk) {
          fa[nb][kk][0] = rd_a(t + 1, kk, 0);
          fa[nb][kk][1] = rd_a(t + 1, kk, 1);
          fb[nb][kk] = rd_b(t + 1, kk);
        }
      }
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int kk = 0; kk < 4; ++kk) {
        acc[0] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[cb][kk][0], fb[cb][kk], acc[0], 0, 0, 0);
        acc[1] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[cb][kk][1], fb[cb][kk], acc[1], 0, 0, 0);
      }
      __builtin_amdgcn_sched_barrier(0);
    }
    __syncthreads();  // every wave is done with band `CUR`: it becomes the epilogue's staging area

    // park the tile as bf16 [128][64] (chunk ^ (row & 7)) in band `CUR`, then the shared store pass
    bf16_t* et = reinterpret_cast<bf16_t*>(bcur);
    const int ml = 32 * wid + frow;
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int nl = 32 * i + 8 * g + 4 * fh;
        const uint32_t lo = (uint32_t)f2bf(acc[i][4 * g] + bv[i][g][0]) |
                            ((uint32_t)f2bf(acc[i][4 * g + 1] + bv[i][g][1]) << 16);
        const uint32_t hi = (uint32_t)f2bf(acc[i][4 * g + 2] + bv[i][g][2]) |
                            ((uint32_t)f2bf(acc[i][4 * g + 3] + bv[i][g][3]) << 16);
        *reinterpret_cast<uint2*>(&et[ml * 64 + (((nl >> 3) ^ (ml & 7)) << 3) + (nl & 4)]) = make_uint2(lo, hi);
      }
    __syncthreads();
    conv_store_pass<PT_BM, 64, PT_NT>(p, et, tid, m0, 0, tile, false, skp);
    PT_WAIT0();       // the next band has landed (and this tile's stores / loads retired)
    __syncthreads();  // … for every wave; band `CUR` is free for the tile after next
  };

  int tile = blockIdx.x;
  if (tile < ntiles) load_band(tile, band0);
  PT_WAIT0();
  __syncthreads();
  const int G = (int)gridDim.x;
  while (tile < ntiles) {
    do_tile(tile, std::integral_constant<int, 0>{});
    tile += G;
    if (tile >= ntiles) break;
    do_tile(tile, std::integral_constant<int, 1>{});
    tile += G;
  }
}

// ---- host side ----
// Band pixels a 128-pixel tile needs at width W: the output rows it touches — at most
// floor((W − 1 + 127) / W) + 1, for a tile starting in the last column — plus the two halo rows.
static int patch_rows(int W) { return ((PT_BM - 1 + W - 1) / W + 3) * W; }

bool conv_patch_ok(const ConvParams& p) {
  if (p.C != 64 || p.K != 64 || p.ldx != 64 || p.R != 3 || p.S != 3) return false;
  if (p.sh != 1 || p.sw != 1 || p.ph != 1 || p.pw != 1 || p.dh != 1 || p.dw != 1) return false;
  if (p.P != p.H || p.Q != p.W || p.scatter || p.cdup || p.ax || p.y32 || p.res32 || p.bnx32) return false;
  if (p.T != 1 || p.KT != 1 || p.ldw < 576 || p.ldw % 8 || p.ldy % 8) return false;
  if (p.W < 8 || patch_rows(p.W) > PT_ROWS) return false;
  if ((size_t)p.Nb * p.H * p.W * 128 >= 0x80000000ull) return false;
  return true;
}

// Off by default: in the ResNet-50 training step it measured slower than the implicit-GEMM kernels
// it replaces (20.90–21.00 vs 20.66–20.70 ms/step, profiles/r5_conv_patch_ab.txt — alone it wins on
// the plain forward / data gradient, 108 vs 126 µs, but its one-workgroup-per-CU epilogue with BN
// statistics or the BN-backward prologue is exposed).  BIGDL_CONV_PATCH=1 or
// bigdl_conv_patch_enable(1) turns it on.
static int g_patch = -1;
static int patch_env() {
  if (g_patch < 0) {
    const char* e = getenv("BIGDL_CONV_PATCH");
    g_patch = e ? atoi(e) : 0;
  }
  return g_patch;
}

BIGDL_EXPORT int bigdl_conv_patch_enable(int on) {
  const int old = patch_env();
  g_patch = on ? 1 : 0;
  return old;
}

int conv_patch_launch(ConvParams p, hipStream_t s) {
  if (!patch_env() || !conv_patch_ok(p)) return (int)hipErrorNotSupported;
  const int ntiles = (p.M + PT_BM - 1) / PT_BM;
  p.tiles_n = 1;
  p.tiles_m = ntiles;  // BM = SBM: one statistics row group per tile
  static int cus = [] {
    int dev = 0, n = 256;
    if (hipGetDevice(&dev) == hipSuccess) (void)hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev);
    return n > 0 ? n : 256;
  }();
  const int grid = ntiles < cus ? ntiles : cus;
  hipLaunchKernelGGL(k_conv_patch64, dim3((unsigned)grid), dim3(PT_NT), 0, s, p, ntiles, patch_rows(p.W));
  return (int)hipGetLastError();
}
