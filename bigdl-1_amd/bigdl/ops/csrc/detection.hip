// Detection kernels (K28): greedy non-maximum suppression and bilinear ROI align
// (reference nn/Nms.scala, nn/RoiAlign.scala:45-330).
//
// NMS runs in two launches, both on the device so nothing but the kept count comes back to the host:
//  1. k_nms_mask — the pairwise "IoU > thresh" test of the score-sorted boxes as a bitmask, one
//     64-bit word per (row box, 64-column block).  A 64-lane workgroup owns a 64×64 tile: the tile's
//     column boxes go through LDS, each lane tests its row box against them.  Only the upper
//     triangle (column > row) is computed — the greedy scan never reads the rest.
//  2. k_nms_scan — one wave walks the boxes in score order.  The running "removed" set lives in LDS
//     (one word per 64 boxes).  A 64-box word is resolved at once: lane l holds row (64w+l)'s
//     bits inside the same word, the wave resolves the in-word suppression chain with readlane in
//     uniform control flow, then the kept rows' masks are OR-ed into the later words (lanes sweep
//     words).  Kept indices come out in score order, truncated at max_keep.
//
// ROI align is a gather: one thread per output element (roi, c, ph, pw), sr_h × sr_w bilinear
// samples per bin, arbitrary input strides (NCHW or channels-last, fp32 or bf16) and fp32 output.
// The threads' element order follows the input's fastest dimension (pw for NCHW, c for NHWC) so
// neighbouring lanes read neighbouring addresses.  The backward scatters the four-corner weights
// with fp32 atomics into an fp32 gradient (non-deterministic summation order, like the reference's
// multithreaded accumulation).
#include "common.h"

__global__ void __launch_bounds__(64) k_nms_mask(const float4* __restrict__ boxes, int n, int words, float thresh,
                                                 float plus_one, uint64_t* __restrict__ mask) {
  const int rb = blockIdx.y, cb = blockIdx.x;
  if (cb < rb) return;  // lower triangle never read
  __shared__ float4 cols[64];
  const int tid = threadIdx.x;
  const int j0 = cb * 64;
  if (j0 + tid < n) cols[tid] = boxes[j0 + tid];
  __syncthreads();
  const int i = rb * 64 + tid;
  if (i >= n) return;
  const float4 a = boxes[i];
  const float area_a = (a.z - a.x + plus_one) * (a.w - a.y + plus_one);
  const int jn = min(64, n - j0);
  uint64_t bits = 0;
  for (int t = 0; t < jn; ++t) {
    const int j = j0 + t;
    if (j <= i) continue;
    const float4 b = cols[t];
    const float w = fmaxf(fminf(a.z, b.z) - fmaxf(a.x, b.x) + plus_one, 0.f);
    const float h = fmaxf(fminf(a.w, b.w) - fmaxf(a.y, b.y) + plus_one, 0.f);
    const float inter = w * h;
    const float area_b = (b.z - b.x + plus_one) * (b.w - b.y + plus_one);
    const float iou = inter / fmaxf(area_a + area_b - inter, 1e-12f);
    if (iou > thresh) bits |= 1ull << t;
  }
  mask[(long long)i * words + cb] = bits;
}

constexpr int NMS_MAX_WORDS = 512;  // n ≤ 32768 boxes (mask ≤ 128 MiB)

__device__ __forceinline__ uint64_t readlane64(uint64_t v, int lane) {
  const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)v, lane);
  const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(v >> 32), lane);
  return ((uint64_t)hi << 32) | lo;
}

__global__ void __launch_bounds__(64) k_nms_scan(const uint64_t* __restrict__ mask, int n, int words, int max_keep,
                                                 long long* __restrict__ keep, int* __restrict__ count) {
  __shared__ uint64_t rem[NMS_MAX_WORDS];
  const int lane = threadIdx.x;
  for (int j = lane; j < words; j += 64) rem[j] = 0;
  __syncthreads();
  int cnt = 0;
  for (int w = 0; w < words; ++w) {
    uint64_t cur = rem[w];
    const int row = w * 64 + lane;
    const uint64_t dm = row < n ? mask[(long long)row * words + w] : 0ull;
    const int nb = min(64, n - w * 64);
    uint64_t kept = 0;
    for (int b = 0; b < nb; ++b) {
      if (!((cur >> b) & 1ull)) {
        kept |= 1ull << b;
        cur |= readlane64(dm, b);
      }
    }
    if (max_keep > 0) {
      while (cnt + __popcll(kept) > max_keep) kept &= ~(1ull << (63 - __clzll(kept)));
    }
    if ((kept >> lane) & 1ull) keep[cnt + __popcll(kept & ((1ull << lane) - 1ull))] = row;
    cnt += __popcll(kept);
    if (max_keep > 0 && cnt >= max_keep) break;
    for (int j = w + 1 + lane; j < words; j += 64) {
      uint64_t v = 0, kb = kept;
      while (kb) {
        const int b = __ffsll((long long)kb) - 1;
        kb &= kb - 1;
        v |= mask[(long long)(w * 64 + b) * words + j];
      }
      rem[j] |= v;
    }
    __syncthreads();
  }
  if (lane == 0) count[0] = cnt;
}

BIGDL_EXPORT int bigdl_nms(const float* boxes, int n, float thresh, float plus_one, int max_keep, void* mask,
                           long long* keep, int* count, hipStream_t s) {
  if (n <= 0 || ((uintptr_t)boxes & 15)) return (int)hipErrorInvalidValue;
  const int words = (n + 63) / 64;
  if (words > NMS_MAX_WORDS) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(k_nms_mask, dim3(words, words), dim3(64), 0, s, (const float4*)boxes, n, words, thresh, plus_one,
                     (uint64_t*)mask);
  hipLaunchKernelGGL(k_nms_scan, dim3(1), dim3(64), 0, s, (const uint64_t*)mask, n, words, max_keep, keep, count);
  BIGDL_CHECK_LAUNCH();
}

// ------------------------------------------------------------------------------------------------ ROI align
struct RoiGeom {
  float y1, x1, bin_h, bin_w;
  int srh, srw, b;
};

__device__ __forceinline__ RoiGeom roi_geom(const float* __restrict__ r, float scale, int oh, int ow, int sr,
                                            int aligned) {
  const float off = aligned ? 0.5f : 0.f;
  RoiGeom g;
  g.b = (int)r[0];
  g.x1 = r[1] * scale - off;
  g.y1 = r[2] * scale - off;
  float rw = r[3] * scale - off - g.x1, rh = r[4] * scale - off - g.y1;
  if (!aligned) {
    rw = fmaxf(rw, 1.f);
    rh = fmaxf(rh, 1.f);
  }
  g.bin_h = rh / oh;
  g.bin_w = rw / ow;
  if (sr > 0) {
    g.srh = g.srw = sr;
  } else {  // adaptive: ceil(roi / bins) samples per bin
    g.srh = max(1, (int)ceilf(fmaxf(rh, 0.f) / oh));
    g.srw = max(1, (int)ceilf(fmaxf(rw, 0.f) / ow));
  }
  return g;
}

// corner offsets (relative to the channel base) and weights of one sample; false = outside
__device__ __forceinline__ bool bilinear(float y, float x, int H, int W, long long sh, long long sw, long long o[4],
                                         float wt[4]) {
  if (y < -1.f || y > (float)H || x < -1.f || x > (float)W) return false;
  y = fminf(fmaxf(y, 0.f), (float)(H - 1));
  x = fminf(fmaxf(x, 0.f), (float)(W - 1));
  const int y0 = (int)floorf(y), x0 = (int)floorf(x);
  const int y1 = min(y0 + 1, H - 1), x1 = min(x0 + 1, W - 1);
  const float ly = y - y0, lx = x - x0, hy = 1.f - ly, hx = 1.f - lx;
  o[0] = y0 * sh + x0 * sw;
  o[1] = y0 * sh + x1 * sw;
  o[2] = y1 * sh + x0 * sw;
  o[3] = y1 * sh + x1 * sw;
  wt[0] = hy * hx;
  wt[1] = hy * lx;
  wt[2] = ly * hx;
  wt[3] = ly * lx;
  return true;
}

struct RoiArgs {
  const float* rois;  // K × 5 fp32 (batch index, x1, y1, x2, y2)
  int K, C, H, W, oh, ow, sr, aligned, c_inner;
  float scale;
  long long sn, sc, sh, sw;  // input (or input-gradient) strides, elements
  long long on, oc, oh_s, ow_s;  // output (or output-gradient) strides, elements
};

__device__ __forceinline__ void roi_index(const RoiArgs& a, long long idx, int& k, int& c, int& ph, int& pw) {
  if (a.c_inner) {
    c = (int)(idx % a.C);
    idx /= a.C;
    pw = (int)(idx % a.ow);
    idx /= a.ow;
    ph = (int)(idx % a.oh);
    k = (int)(idx / a.oh);
  } else {
    pw = (int)(idx % a.ow);
    idx /= a.ow;
    ph = (int)(idx % a.oh);
    idx /= a.oh;
    c = (int)(idx % a.C);
    k = (int)(idx / a.C);
  }
}

template <typename T>
__global__ void __launch_bounds__(256) k_roi_align_fwd(const T* __restrict__ x, float* __restrict__ y, RoiArgs a) {
  const long long total = (long long)a.K * a.C * a.oh * a.ow;
  for (long long idx = blockIdx.x * 256ll + threadIdx.x; idx < total; idx += (long long)gridDim.x * 256) {
    int k, c, ph, pw;
    roi_index(a, idx, k, c, ph, pw);
    const RoiGeom g = roi_geom(a.rois + 5 * k, a.scale, a.oh, a.ow, a.sr, a.aligned);
    const T* base = x + g.b * a.sn + c * a.sc;
    float acc = 0.f;
    for (int iy = 0; iy < g.srh; ++iy) {
      const float yy = g.y1 + ((ph * g.srh + iy) + 0.5f) / g.srh * g.bin_h;
      for (int ix = 0; ix < g.srw; ++ix) {
        const float xx = g.x1 + ((pw * g.srw + ix) + 0.5f) / g.srw * g.bin_w;
        long long o[4];
        float wt[4];
        if (!bilinear(yy, xx, a.H, a.W, a.sh, a.sw, o, wt)) continue;
        if constexpr (sizeof(T) == 4) {
          acc += wt[0] * base[o[0]] + wt[1] * base[o[1]] + wt[2] * base[o[2]] + wt[3] * base[o[3]];
        } else {
          acc += wt[0] * bf2f(base[o[0]]) + wt[1] * bf2f(base[o[1]]) + wt[2] * bf2f(base[o[2]]) +
                 wt[3] * bf2f(base[o[3]]);
        }
      }
    }
    y[k * a.on + c * a.oc + ph * a.oh_s + pw * a.ow_s] = acc / (float)(g.srh * g.srw);
  }
}

__global__ void __launch_bounds__(256) k_roi_align_bwd(const float* __restrict__ gy, float* __restrict__ gx,
                                                       RoiArgs a) {
  const long long total = (long long)a.K * a.C * a.oh * a.ow;
  for (long long idx = blockIdx.x * 256ll + threadIdx.x; idx < total; idx += (long long)gridDim.x * 256) {
    int k, c, ph, pw;
    roi_index(a, idx, k, c, ph, pw);
    const RoiGeom g = roi_geom(a.rois + 5 * k, a.scale, a.oh, a.ow, a.sr, a.aligned);
    const float go = gy[k * a.on + c * a.oc + ph * a.oh_s + pw * a.ow_s] / (float)(g.srh * g.srw);
    if (go == 0.f) continue;
    float* base = gx + g.b * a.sn + c * a.sc;
    for (int iy = 0; iy < g.srh; ++iy) {
      const float yy = g.y1 + ((ph * g.srh + iy) + 0.5f) / g.srh * g.bin_h;
      for (int ix = 0; ix < g.srw; ++ix) {
        const float xx = g.x1 + ((pw * g.srw + ix) + 0.5f) / g.srw * g.bin_w;
        long long o[4];
        float wt[4];
        if (!bilinear(yy, xx, a.H, a.W, a.sh, a.sw, o, wt)) continue;
#pragma unroll
        for (int q = 0; q < 4; ++q) atomicAdd(base + o[q], go * wt[q]);
      }
    }
  }
}

// dtype: 0 = fp32 input, 1 = bf16.  strides[0..3] input n,c,h,w; strides[4..7] output k,c,h,w.
BIGDL_EXPORT int bigdl_roi_align_fwd(const void* x, int dtype, const float* rois, float* y, int K, int C, int H, int W,
                                     int oh, int ow, float scale, int sr, int aligned, const long long* strides,
                                     hipStream_t s) {
  if (K <= 0 || C <= 0 || H <= 0 || W <= 0 || oh <= 0 || ow <= 0) return (int)hipErrorInvalidValue;
  RoiArgs a{rois, K, C, H, W, oh, ow, sr, aligned, strides[1] == 1 && C > 1, scale,
            strides[0], strides[1], strides[2], strides[3], strides[4], strides[5], strides[6], strides[7]};
  const long long total = (long long)K * C * oh * ow;
  const dim3 g(bigdl_grid(total, 256, 65536));
  if (dtype == 0)
    hipLaunchKernelGGL(k_roi_align_fwd<float>, g, dim3(256), 0, s, (const float*)x, y, a);
  else
    hipLaunchKernelGGL(k_roi_align_fwd<bf16_t>, g, dim3(256), 0, s, (const bf16_t*)x, y, a);
  BIGDL_CHECK_LAUNCH();
}

// gx: fp32 input gradient (zero-filled by the caller), strides as the forward's input strides
BIGDL_EXPORT int bigdl_roi_align_bwd(const float* gy, const float* rois, float* gx, int K, int C, int H, int W, int oh,
                                     int ow, float scale, int sr, int aligned, const long long* strides,
                                     hipStream_t s) {
  if (K <= 0 || C <= 0 || H <= 0 || W <= 0 || oh <= 0 || ow <= 0) return (int)hipErrorInvalidValue;
  RoiArgs a{rois, K, C, H, W, oh, ow, sr, aligned, strides[1] == 1 && C > 1, scale,
            strides[0], strides[1], strides[2], strides[3], strides[4], strides[5], strides[6], strides[7]};
  const long long total = (long long)K * C * oh * ow;
  hipLaunchKernelGGL(k_roi_align_bwd, dim3(bigdl_grid(total, 256, 65536)), dim3(256), 0, s, gy, gx, a);
  BIGDL_CHECK_LAUNCH();
}
