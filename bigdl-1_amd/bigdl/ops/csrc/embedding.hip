// Embedding lookup (K16): LookupTable.updateOutput gather and accGradParameters scatter-add
// (DL/nn/LookupTable.scala:170-230).  1-based indices arrive as the layer's float tensor (the
// reference's Tensor[T] of ids) or as int32 / int64.  The reference requires 1 <= id <= nIndex
// (LookupTable.scala:96-98,227-229): the forward kernel sets a device error flag (a vector atomic
// OR into a 4-byte buffer) for any id outside that range, which the host wrapper reads back
// asynchronously and raises on; the index is still clamped on the device so a bad id can never
// address outside the table.
//
// Forward: one wave per index row, 16-B vector copies (8 bf16 / 4 fp32 per lane).
// Backward: grad[id − 1][:] += scale · gy[i][:] with no-return fp32 atomics (many ids repeat —
// PTB's vocabulary has heavy hitters — and the per-row adds are independent), rows whose id equals
// paddingValue get no gradient.
#include "common.h"

template <typename I>
__device__ __forceinline__ long long row_of(const I* idx, long long i, long long n_index) {
  long long r = (long long)idx[i] - 1;
  return r < 0 ? 0 : (r >= n_index ? n_index - 1 : r);
}

template <typename I, typename T>
__global__ void __launch_bounds__(256) k_embed_fwd(const T* __restrict__ w, const I* __restrict__ idx, T* __restrict__ out,
                                                   long long n, long long n_index, int D, int* __restrict__ err,
                                                   int has_allow, float allow_v) {
  const long long i = (long long)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (i >= n) return;
  const int lane = threadIdx.x & 63;
  if (err != nullptr && lane == 0) {
    const long long raw = (long long)idx[i];
    const bool allowed = has_allow && (float)idx[i] == allow_v;  // masked padding id (maskZero)
    if (!allowed && (raw < 1 || raw > n_index || (float)idx[i] != (float)raw)) atomicOr(err, 1);
  }
  const long long r = row_of(idx, i, n_index);
  const T* src = w + r * D;
  T* dst = out + i * D;
  constexpr int V = 16 / sizeof(T);
  if (D % V == 0) {
    for (int c = lane * V; c < D; c += 64 * V)
      *reinterpret_cast<uint4*>(dst + c) = *reinterpret_cast<const uint4*>(src + c);
  } else {
    for (int c = lane; c < D; c += 64) dst[c] = src[c];
  }
}

template <typename T> __device__ __forceinline__ float tof(T v);
template <> __device__ __forceinline__ float tof<float>(float v) { return v; }
template <> __device__ __forceinline__ float tof<bf16_t>(bf16_t v) { return bf2f(v); }

template <typename I, typename T>
__global__ void __launch_bounds__(256) k_embed_bwd(float* __restrict__ gw, const I* __restrict__ idx, const T* __restrict__ gy,
                                                   long long n, long long n_index, int D, float scale, int has_pad,
                                                   float pad) {
  const long long i = (long long)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (i >= n) return;
  if (has_pad && (float)idx[i] == pad) return;
  const int lane = threadIdx.x & 63;
  const long long r = row_of(idx, i, n_index);
  float* dst = gw + r * D;
  const T* src = gy + i * D;
  for (int c = lane; c < D; c += 64) atomicAdd(dst + c, scale * tof(src[c]));
}

// Deterministic variant (bigdl.deterministic): one thread owns one column and walks the indices in
// order, so repeated ids accumulate in a fixed sequence (no atomics; D-way parallel only).
template <typename I, typename T>
__global__ void __launch_bounds__(256) k_embed_bwd_det(float* __restrict__ gw, const I* __restrict__ idx,
                                                       const T* __restrict__ gy, long long n, long long n_index, int D,
                                                       float scale, int has_pad, float pad) {
  const int c = blockIdx.x * 256 + threadIdx.x;
  if (c >= D) return;
  for (long long i = 0; i < n; ++i) {
    if (has_pad && (float)idx[i] == pad) continue;
    const long long r = row_of(idx, i, n_index);
    gw[r * D + c] += scale * tof(gy[i * D + c]);
  }
}

// itype: 0 = float32 ids, 1 = int64, 2 = int32; dtype: 0 = bf16 table/gradient, 1 = fp32
template <typename T>
static void launch_fwd(int itype, dim3 g, hipStream_t s, const void* w, const void* idx, void* out, long long n,
                       long long ni, int D, int* err, int ha, float av) {
  if (itype == 0)
    hipLaunchKernelGGL((k_embed_fwd<float, T>), g, dim3(256), 0, s, (const T*)w, (const float*)idx, (T*)out, n, ni, D,
                       err, ha, av);
  else if (itype == 1)
    hipLaunchKernelGGL((k_embed_fwd<long long, T>), g, dim3(256), 0, s, (const T*)w, (const long long*)idx, (T*)out, n,
                       ni, D, err, ha, av);
  else
    hipLaunchKernelGGL((k_embed_fwd<int, T>), g, dim3(256), 0, s, (const T*)w, (const int*)idx, (T*)out, n, ni, D,
                       err, ha, av);
}

// err: optional device int (4-B aligned) OR-ed with 1 when an id is outside [1, n_index]; an id
// equal to allow_v (has_allow: the maskZero padding id) is exempt
BIGDL_EXPORT int bigdl_embedding_fwd(const void* w, const void* idx, int itype, void* out, long long n,
                                     long long n_index, int D, int dtype, int* err, int has_allow, float allow_v,
                                     hipStream_t s) {
  if (n <= 0 || n_index <= 0 || D <= 0 || itype < 0 || itype > 2) return (int)hipErrorInvalidValue;
  if (((uintptr_t)w & 15) || ((uintptr_t)out & 15) || ((uintptr_t)err & 3)) return (int)hipErrorInvalidValue;
  dim3 g((unsigned)((n + 3) / 4));
  if (dtype == 0) launch_fwd<bf16_t>(itype, g, s, w, idx, out, n, n_index, D, err, has_allow, allow_v);
  else launch_fwd<float>(itype, g, s, w, idx, out, n, n_index, D, err, has_allow, allow_v);
  BIGDL_CHECK_LAUNCH();
}

template <typename T>
static void launch_bwd(int itype, dim3 g, hipStream_t s, float* gw, const void* idx, const void* gy, long long n,
                       long long ni, int D, float scale, int has_pad, float pad) {
  if (g_bigdl_deterministic) {
    const dim3 gd((unsigned)((D + 255) / 256));
    if (itype == 0)
      hipLaunchKernelGGL((k_embed_bwd_det<float, T>), gd, dim3(256), 0, s, gw, (const float*)idx, (const T*)gy, n, ni,
                         D, scale, has_pad, pad);
    else if (itype == 1)
      hipLaunchKernelGGL((k_embed_bwd_det<long long, T>), gd, dim3(256), 0, s, gw, (const long long*)idx,
                         (const T*)gy, n, ni, D, scale, has_pad, pad);
    else
      hipLaunchKernelGGL((k_embed_bwd_det<int, T>), gd, dim3(256), 0, s, gw, (const int*)idx, (const T*)gy, n, ni, D,
                         scale, has_pad, pad);
    return;
  }
  if (itype == 0)
    hipLaunchKernelGGL((k_embed_bwd<float, T>), g, dim3(256), 0, s, gw, (const float*)idx, (const T*)gy, n, ni, D, scale,
                       has_pad, pad);
  else if (itype == 1)
    hipLaunchKernelGGL((k_embed_bwd<long long, T>), g, dim3(256), 0, s, gw, (const long long*)idx, (const T*)gy, n, ni,
                       D, scale, has_pad, pad);
  else
    hipLaunchKernelGGL((k_embed_bwd<int, T>), g, dim3(256), 0, s, gw, (const int*)idx, (const T*)gy, n, ni, D, scale,
                       has_pad, pad);
}

BIGDL_EXPORT int bigdl_embedding_bwd(float* gw, const void* idx, int itype, const void* gy, long long n,
                                     long long n_index, int D, int dtype, float scale, int has_pad, float pad,
                                     hipStream_t s) {
  if (n <= 0 || n_index <= 0 || D <= 0 || itype < 0 || itype > 2) return (int)hipErrorInvalidValue;
  dim3 g((unsigned)((n + 3) / 4));
  if (dtype == 0) launch_bwd<bf16_t>(itype, g, s, gw, idx, gy, n, n_index, D, scale, has_pad, pad);
  else launch_bwd<float>(itype, g, s, gw, idx, gy, n, n_index, D, scale, has_pad, pad);
  BIGDL_CHECK_LAUNCH();
}
