// K25: batched crop + mirror + per-channel normalise + cast, HWC (uint8 or fp32) → NHWC
// (bf16 or fp32) — the device-side tail of the image pipeline (reference: OpenCV crop / flip /
// ChannelNormalize per image, DL/transform/vision/image/augmentation/*.scala).
// One thread per output pixel, all C (≤ 4) channels; the BGR→RGB swap is an index permutation.
#include "common.h"

template <typename TIN, bool OUT_BF16>
__global__ void __launch_bounds__(256) k_img_cfn(const TIN* __restrict__ src, int B, int H, int W, int C,
                                                 const int* __restrict__ oy, const int* __restrict__ ox,
                                                 const int* __restrict__ flip, int OH, int OW, float4 mean,
                                                 float4 inv_std, int to_rgb, void* __restrict__ out) {
  const long long total = (long long)B * OH * OW;
  for (long long p = blockIdx.x * (long long)blockDim.x + threadIdx.x; p < total;
       p += (long long)gridDim.x * blockDim.x) {
    const int b = (int)(p / ((long long)OH * OW));
    const int r = (int)(p - (long long)b * OH * OW);
    const int y = r / OW, x = r - (r / OW) * OW;
    const int sx = flip[b] ? (OW - 1 - x) : x;
    const TIN* s = src + (((long long)b * H + oy[b] + y) * W + ox[b] + sx) * C;
    const float m[4] = {mean.x, mean.y, mean.z, mean.w};
    const float is[4] = {inv_std.x, inv_std.y, inv_std.z, inv_std.w};
    for (int c = 0; c < C; ++c) {
      const int sc = (to_rgb && C == 3) ? 2 - c : c;
      const float v = ((float)s[sc] - m[c]) * is[c];
      if (OUT_BF16)
        reinterpret_cast<bf16_t*>(out)[p * C + c] = f2bf(v);
      else
        reinterpret_cast<float*>(out)[p * C + c] = v;
    }
  }
}

BIGDL_EXPORT int bigdl_image_crop_flip_norm(const void* src, int src_u8, int B, int H, int W, int C, const int* oy,
                                            const int* ox, const int* flip, int OH, int OW, const float* mean,
                                            const float* stdv, int to_rgb, void* out, int out_bf16, hipStream_t s) {
  if (B <= 0 || C <= 0 || C > 4 || OH <= 0 || OW <= 0) return (int)hipErrorInvalidValue;
  float mm[4] = {0, 0, 0, 0}, iv[4] = {1, 1, 1, 1};
  for (int c = 0; c < C; ++c) {
    mm[c] = mean[c];
    iv[c] = 1.f / stdv[c];
  }
  const float4 m4 = make_float4(mm[0], mm[1], mm[2], mm[3]);
  const float4 i4 = make_float4(iv[0], iv[1], iv[2], iv[3]);
  const int grid = bigdl_grid((long long)B * OH * OW, 256, 8192);
  if (src_u8 && out_bf16)
    hipLaunchKernelGGL((k_img_cfn<uint8_t, true>), dim3(grid), dim3(256), 0, s, (const uint8_t*)src, B, H, W, C, oy,
                       ox, flip, OH, OW, m4, i4, to_rgb, out);
  else if (src_u8)
    hipLaunchKernelGGL((k_img_cfn<uint8_t, false>), dim3(grid), dim3(256), 0, s, (const uint8_t*)src, B, H, W, C, oy,
                       ox, flip, OH, OW, m4, i4, to_rgb, out);
  else if (out_bf16)
    hipLaunchKernelGGL((k_img_cfn<float, true>), dim3(grid), dim3(256), 0, s, (const float*)src, B, H, W, C, oy, ox,
                       flip, OH, OW, m4, i4, to_rgb, out);
  else
    hipLaunchKernelGGL((k_img_cfn<float, false>), dim3(grid), dim3(256), 0, s, (const float*)src, B, H, W, C, oy, ox,
                       flip, OH, OW, m4, i4, to_rgb, out);
  BIGDL_CHECK_LAUNCH();
}
