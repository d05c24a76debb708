// Backward-data weight transform: the dgrad of a conv is a forward conv of dY with the flipped,
// channel-transposed filter, W'[c][i][j][k] = W[k][rmap[i]][smap[j]][c] (stride 1: rmap = R-1-i;
// strided dgrad by sub-pixel decomposition: one flipped sub-filter per output parity class).
// Reference: SpatialConvolution.updateGradInput multiplies by the un-transposed weight through
// col2im (DL/nn/SpatialConvolution.scala:656-735); here the transpose is materialised once per step
// per layer, for every parity class in ONE launch (grid.z = class).
//
// Each block moves a 64(k) × 64(c) tile of one tap through LDS: coalesced 128-B reads along c of
// the KRSC storage, coalesced writes along k of the [C][Ro][So][K] output.
#include "common.h"

constexpr int XF_MAXC = 4;  // parity classes per launch (stride ≤ 2 in both dims)
constexpr int XF_MAXT = 8;  // taps per dimension

struct XformClass {
  int ro, so;
  int rmap[XF_MAXT], smap[XF_MAXT];
  long long out_off;
};

struct XformParams {
  const bf16_t* in;  // [K][R][S][C]
  bf16_t* out;
  int K, R, S, C, ncls;
  XformClass cls[XF_MAXC];
};

__global__ void __launch_bounds__(256) k_w_xform(XformParams p) {
  constexpr int LD = 72;  // tile row pitch in bf16 (16-B aligned rows, staggered banks)
  __shared__ __attribute__((aligned(16))) bf16_t t[64 * LD];
  const XformClass& cl = p.cls[blockIdx.z];
  const int tap = blockIdx.y;
  if (tap >= cl.ro * cl.so) return;  // block-uniform
  const int i = tap / cl.so, j = tap - (tap / cl.so) * cl.so;
  const int r = cl.rmap[i], s = cl.smap[j];
  const int tiles_c = (p.C + 63) / 64;
  const int c0 = (blockIdx.x % tiles_c) * 64, k0 = (blockIdx.x / tiles_c) * 64;
  const int tid = threadIdx.x;
  // 64 k-rows × 8 chunks of 8 channels: 16-B loads along c
#pragma unroll
  for (int it = 0; it < 2; ++it) {
    const int idx = tid + 256 * it, kl = idx >> 3, ch = idx & 7;
    const int k = k0 + kl, c = c0 + ch * 8;
    uint4 v = make_uint4(0u, 0u, 0u, 0u);
    if (k < p.K && c < p.C) v = *reinterpret_cast<const uint4*>(p.in + (((size_t)k * p.R + r) * p.S + s) * p.C + c);
    *reinterpret_cast<uint4*>(&t[kl * LD + ch * 8]) = v;
  }
  __syncthreads();
  // 64 c-rows × 8 chunks of 8 output channels k: 16-B stores along k
#pragma unroll
  for (int it = 0; it < 2; ++it) {
    const int idx = tid + 256 * it, cr = idx >> 3, kc = idx & 7;
    const int c = c0 + cr, k = k0 + kc * 8;
    if (c >= p.C || k >= p.K) continue;
    uint32_t w[4];
#pragma unroll
    for (int e = 0; e < 4; ++e)
      w[e] = (uint32_t)t[(kc * 8 + 2 * e) * LD + cr] | ((uint32_t)t[(kc * 8 + 2 * e + 1) * LD + cr] << 16);
    *reinterpret_cast<uint4*>(p.out + cl.out_off + (((size_t)c * cl.ro + i) * cl.so + j) * p.K + k) =
        make_uint4(w[0], w[1], w[2], w[3]);
  }
}

// out receives the classes back to back at out_offs[q] (elements, multiples of 8).  rmaps / smaps: class q's taps
// at [q * 8 + i].  Host arrays.
BIGDL_EXPORT int bigdl_w_dgrad_xform(const void* w, void* out, int K, int R, int S, int C, int ncls, const int* ros,
                                     const int* sos, const int* rmaps, const int* smaps, const long long* out_offs,
                                     hipStream_t s) {
  // 16-B vectors along both c (reads) and k (writes): C, K multiples of 8, 16-B aligned buffers
  if (ncls < 1 || ncls > XF_MAXC || K <= 0 || C <= 0 || C % 8 || K % 8 || ((uintptr_t)w & 15) || ((uintptr_t)out & 15))
    return (int)hipErrorInvalidValue;
  XformParams p{};
  p.in = (const bf16_t*)w;
  p.out = (bf16_t*)out;
  p.K = K; p.R = R; p.S = S; p.C = C; p.ncls = ncls;
  int taps = 0;
  for (int q = 0; q < ncls; ++q) {
    XformClass& c = p.cls[q];
    c.ro = ros[q];
    c.so = sos[q];
    if (c.ro < 1 || c.so < 1 || c.ro > XF_MAXT || c.so > XF_MAXT) return (int)hipErrorInvalidValue;
    for (int i = 0; i < XF_MAXT; ++i) {
      c.rmap[i] = i < c.ro ? rmaps[q * XF_MAXT + i] : 0;
      c.smap[i] = i < c.so ? smaps[q * XF_MAXT + i] : 0;
      if (i < c.ro && (c.rmap[i] < 0 || c.rmap[i] >= R)) return (int)hipErrorInvalidValue;
      if (i < c.so && (c.smap[i] < 0 || c.smap[i] >= S)) return (int)hipErrorInvalidValue;
    }
    c.out_off = out_offs[q];
    if (c.out_off % 8) return (int)hipErrorInvalidValue;
    if (c.ro * c.so > taps) taps = c.ro * c.so;
  }
  const dim3 grid((unsigned)(((C + 63) / 64) * ((K + 63) / 64)), (unsigned)taps, (unsigned)ncls);
  hipLaunchKernelGGL(k_w_xform, grid, dim3(256), 0, s, p);
  BIGDL_CHECK_LAUNCH();
}

// ------------------------------------------------------------------------------------------------
// Every conv's dgrad weight transform of a training step in ONE launch.  The weights change once
// per step (the optimizer update), so the per-layer launches above (one before each layer's dgrad,
// on the backward critical path) are replaced by a batched launch at the first dgrad after an
// update: a device-resident job table (built once per model, pointers stable in the parameter
// arena's bf16 shadow) and a per-job prefix of block counts; block b finds its job by a binary
// search over ≤ a few hundred prefix entries and runs the tile body of k_w_xform for that job.
// ------------------------------------------------------------------------------------------------
struct XformJob {
  XformParams p;
  int tiles;   // 64 × 64 (k, c) tiles per tap
  int taps;    // max taps over the classes
  long long first_block;
};

__global__ void __launch_bounds__(256) k_w_xform_multi(const XformJob* __restrict__ jobs, int njobs) {
  constexpr int LD = 72;
  __shared__ __attribute__((aligned(16))) bf16_t t[64 * LD];
  const long long b = blockIdx.x;
  int lo = 0, hi = njobs - 1;  // last job with first_block <= b
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (jobs[mid].first_block <= b) lo = mid;
    else hi = mid - 1;
  }
  const XformJob& jb = jobs[lo];
  const XformParams& p = jb.p;
  long long local = b - jb.first_block;
  const int q = (int)(local / ((long long)jb.tiles * jb.taps));
  local -= (long long)q * jb.tiles * jb.taps;
  const int tap = (int)(local / jb.tiles);
  const int tile = (int)(local - (long long)tap * jb.tiles);
  if (q >= p.ncls) return;  // block-uniform
  const XformClass& cl = p.cls[q];
  if (tap >= cl.ro * cl.so) return;
  const int i = tap / cl.so, j = tap - (tap / cl.so) * cl.so;
  const int r = cl.rmap[i], s = cl.smap[j];
  const int tiles_c = (p.C + 63) / 64;
  const int c0 = (tile % tiles_c) * 64, k0 = (tile / tiles_c) * 64;
  const int tid = threadIdx.x;
#pragma unroll
  for (int it = 0; it < 2; ++it) {
    const int idx = tid + 256 * it, kl = idx >> 3, ch = idx & 7;
    const int k = k0 + kl, c = c0 + ch * 8;
    uint4 v = make_uint4(0u, 0u, 0u, 0u);
    if (k < p.K && c < p.C) v = *reinterpret_cast<const uint4*>(p.in + (((size_t)k * p.R + r) * p.S + s) * p.C + c);
    *reinterpret_cast<uint4*>(&t[kl * LD + ch * 8]) = v;
  }
  __syncthreads();
#pragma unroll
  for (int it = 0; it < 2; ++it) {
    const int idx = tid + 256 * it, cr = idx >> 3, kc = idx & 7;
    const int c = c0 + cr, k = k0 + kc * 8;
    if (c >= p.C || k >= p.K) continue;
    uint32_t w[4];
#pragma unroll
    for (int e = 0; e < 4; ++e)
      w[e] = (uint32_t)t[(kc * 8 + 2 * e) * LD + cr] | ((uint32_t)t[(kc * 8 + 2 * e + 1) * LD + cr] << 16);
    *reinterpret_cast<uint4*>(p.out + cl.out_off + (((size_t)c * cl.ro + i) * cl.so + j) * p.K + k) =
        make_uint4(w[0], w[1], w[2], w[3]);
  }
}

// Host side of the batched transform: ``jobs_host`` is a byte image of njobs XformJob records
// (built by bigdl_w_xform_job; the caller copies it to ``jobs_dev``), total = Σ blocks.
BIGDL_EXPORT int bigdl_w_xform_job_size() { return (int)sizeof(XformJob); }

// Fill one job record (validated exactly like bigdl_w_dgrad_xform) at ``rec``; returns its block
// count through *nblocks.  first_block is the running prefix the caller passes in.
BIGDL_EXPORT int bigdl_w_xform_job(void* rec, const void* w, void* out, int K, int R, int S, int C, int ncls,
                                   const int* ros, const int* sos, const int* rmaps, const int* smaps,
                                   const long long* out_offs, long long first_block, long long* nblocks) {
  if (ncls < 1 || ncls > XF_MAXC || K <= 0 || C <= 0 || C % 8 || K % 8 || ((uintptr_t)w & 15) || ((uintptr_t)out & 15))
    return (int)hipErrorInvalidValue;
  XformJob jb{};
  XformParams& p = jb.p;
  p.in = (const bf16_t*)w;
  p.out = (bf16_t*)out;
  p.K = K; p.R = R; p.S = S; p.C = C; p.ncls = ncls;
  int taps = 0;
  for (int q = 0; q < ncls; ++q) {
    XformClass& c = p.cls[q];
    c.ro = ros[q];
    c.so = sos[q];
    if (c.ro < 1 || c.so < 1 || c.ro > XF_MAXT || c.so > XF_MAXT) return (int)hipErrorInvalidValue;
    for (int i = 0; i < XF_MAXT; ++i) {
      c.rmap[i] = i < c.ro ? rmaps[q * XF_MAXT + i] : 0;
      c.smap[i] = i < c.so ? smaps[q * XF_MAXT + i] : 0;
      if (i < c.ro && (c.rmap[i] < 0 || c.rmap[i] >= R)) return (int)hipErrorInvalidValue;
      if (i < c.so && (c.smap[i] < 0 || c.smap[i] >= S)) return (int)hipErrorInvalidValue;
    }
    c.out_off = out_offs[q];
    if (c.out_off % 8) return (int)hipErrorInvalidValue;
    if (c.ro * c.so > taps) taps = c.ro * c.so;
  }
  jb.tiles = ((C + 63) / 64) * ((K + 63) / 64);
  jb.taps = taps;
  jb.first_block = first_block;
  *nblocks = (long long)jb.tiles * taps * ncls;
  *reinterpret_cast<XformJob*>(rec) = jb;
  return 0;
}

BIGDL_EXPORT int bigdl_w_xform_multi(const void* jobs_dev, int njobs, long long total_blocks, hipStream_t s) {
  if (njobs <= 0 || total_blocks <= 0 || total_blocks > 0x7fffffffLL || ((uintptr_t)jobs_dev & 15))
    return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(k_w_xform_multi, dim3((unsigned)total_blocks), dim3(256), 0, s, (const XformJob*)jobs_dev,
                     njobs);
  BIGDL_CHECK_LAUNCH();
}
