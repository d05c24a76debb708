// Fused LogSoftMax + ClassNLL (CrossEntropyCriterion, K12+K13) and row-wise (log-)softmax.
//
// Reference: DL/nn/CrossEntropyCriterion.scala (LogSoftMax + ClassNLLCriterion), ClassNLLCriterion
// .scala:89-230 — targets are 1-BASED class indices, a target equal to paddingValue contributes
// nothing, optional per-class weights, sizeAverage divides by Σ weights (or the valid count).
// One block (256 threads = 4 waves) per row; the row is read twice (max/sum pass, then gradient).
#include "common.h"

template <typename T>
__device__ __forceinline__ float ld(const T* p, long long i);
template <>
__device__ __forceinline__ float ld<float>(const float* p, long long i) { return p[i]; }
template <>
__device__ __forceinline__ float ld<bf16_t>(const bf16_t* p, long long i) { return bf2f(p[i]); }

template <typename T>
__device__ __forceinline__ void st(T* p, long long i, float v);
template <>
__device__ __forceinline__ void st<float>(float* p, long long i, float v) { p[i] = v; }
template <>
__device__ __forceinline__ void st<bf16_t>(bf16_t* p, long long i, float v) { p[i] = f2bf(v); }

__device__ __forceinline__ float block_reduce(float v, float* red, bool is_max) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  v = is_max ? wave_max(v) : wave_sum(v);
  if (lane == 0) red[wid] = v;
  __syncthreads();
  float r = red[0];
  for (int i = 1; i < (int)(blockDim.x >> 6); ++i) r = is_max ? fmaxf(r, red[i]) : r + red[i];
  __syncthreads();
  return r;
}

// per row: lse, row loss (weighted), row weight
// TT: the target type — int32, or float (BigDL's 1-based labels as the data loader hands them over,
// read directly instead of a per-step cast)
template <typename T, typename TT = int>
__global__ void __launch_bounds__(256) k_ce_rows(const T* __restrict__ x, const TT* __restrict__ tgt,
                                                 const float* __restrict__ cw, int K, int padding,
                                                 float* __restrict__ lse, float* __restrict__ rloss,
                                                 float* __restrict__ rw) {
  __shared__ float red[8];
  const long long row = blockIdx.x;
  const T* xr = x + row * K;
  float m = -INFINITY;
  for (int i = threadIdx.x; i < K; i += blockDim.x) m = fmaxf(m, ld(xr, i));
  m = block_reduce(m, red, true);
  float s = 0.f;
  for (int i = threadIdx.x; i < K; i += blockDim.x) s += __expf(ld(xr, i) - m);
  s = block_reduce(s, red, false);
  if (threadIdx.x == 0) {
    float l = m + __logf(s);
    lse[row] = l;
    int t = (int)tgt[row];
    bool valid = t != padding && t >= 1 && t <= K;
    float w = valid ? (cw ? cw[t - 1] : 1.f) : 0.f;
    rw[row] = w;
    rloss[row] = valid ? -(ld(xr, t - 1) - l) * w : 0.f;
  }
}

// total loss and denominator (single block, deterministic order)
__global__ void k_ce_total(const float* __restrict__ rloss, const float* __restrict__ rw, long long B, int size_avg,
                           float* __restrict__ out) {
  __shared__ float red[8];
  float a = 0.f, b = 0.f;
  for (long long i = threadIdx.x; i < B; i += blockDim.x) {
    a += rloss[i];
    b += rw[i];
  }
  a = block_reduce(a, red, false);
  b = block_reduce(b, red, false);
  if (threadIdx.x == 0) {
    float denom = size_avg ? fmaxf(b, 1e-12f) : 1.f;
    out[0] = a / denom;
    out[1] = denom;
  }
}

template <typename T, typename TT = int>
__global__ void __launch_bounds__(256) k_ce_grad(const T* __restrict__ x, const TT* __restrict__ tgt,
                                                 const float* __restrict__ lse, const float* __restrict__ rw,
                                                 const float* __restrict__ tot, int K, T* __restrict__ gx) {
  const long long row = blockIdx.x;
  const T* xr = x + row * K;
  T* gr = gx + row * K;
  const float scale = rw[row] / tot[1];
  const float l = lse[row];
  const int t = (int)tgt[row] - 1;
  for (int i = threadIdx.x; i < K; i += blockDim.x) {
    float p = __expf(ld(xr, i) - l);
    st(gr, i, scale * (p - (i == t ? 1.f : 0.f)));
  }
}

template <typename TT>
static void launch_ce(const void* x, const TT* tgt, const float* cw, void* gx, long long B, int K, int padding,
                      int size_avg, int dtype, float* ws, float* out, hipStream_t s) {
  float *lse = ws, *rl = ws + B, *rw = ws + 2 * B;
  if (dtype == 1) {
    hipLaunchKernelGGL((k_ce_rows<bf16_t, TT>), dim3(B), dim3(256), 0, s, (const bf16_t*)x, tgt, cw, K, padding, lse, rl, rw);
  } else {
    hipLaunchKernelGGL((k_ce_rows<float, TT>), dim3(B), dim3(256), 0, s, (const float*)x, tgt, cw, K, padding, lse, rl, rw);
  }
  hipLaunchKernelGGL(k_ce_total, dim3(1), dim3(256), 0, s, rl, rw, B, size_avg, out);
  if (gx) {
    if (dtype == 1)
      hipLaunchKernelGGL((k_ce_grad<bf16_t, TT>), dim3(B), dim3(256), 0, s, (const bf16_t*)x, tgt, lse, rw, out, K,
                         (bf16_t*)gx);
    else
      hipLaunchKernelGGL((k_ce_grad<float, TT>), dim3(B), dim3(256), 0, s, (const float*)x, tgt, lse, rw, out, K,
                         (float*)gx);
  }
}

// dtype: 0 fp32, 1 bf16.  ws: 3·B floats; out: 2 floats (loss, denom).
BIGDL_EXPORT int bigdl_cross_entropy(const void* x, const int* tgt, const float* cw, void* gx, long long B, int K,
                                     int padding, int size_avg, int dtype, float* ws, float* out, hipStream_t s) {
  if (B <= 0 || K <= 0) return (int)hipErrorInvalidValue;
  launch_ce<int>(x, tgt, cw, gx, B, K, padding, size_avg, dtype, ws, out, s);
  BIGDL_CHECK_LAUNCH();
}

// the same with fp32 targets (1-based class indices stored as floats)
BIGDL_EXPORT int bigdl_cross_entropy_ft(const void* x, const float* tgt, const float* cw, void* gx, long long B, int K,
                                        int padding, int size_avg, int dtype, float* ws, float* out, hipStream_t s) {
  if (B <= 0 || K <= 0) return (int)hipErrorInvalidValue;
  launch_ce<float>(x, tgt, cw, gx, B, K, padding, size_avg, dtype, ws, out, s);
  BIGDL_CHECK_LAUNCH();
}

// ------------------------------------------------------------------------------------------------
// row-wise log-softmax forward / backward (LogSoftMax.scala:49-130) over the last dim
// ------------------------------------------------------------------------------------------------
template <typename T>
__global__ void __launch_bounds__(256) k_logsoftmax_fwd(const T* __restrict__ x, T* __restrict__ y, int K) {
  __shared__ float red[8];
  const long long row = blockIdx.x;
  const T* xr = x + row * K;
  float m = -INFINITY;
  for (int i = threadIdx.x; i < K; i += blockDim.x) m = fmaxf(m, ld(xr, i));
  m = block_reduce(m, red, true);
  float s = 0.f;
  for (int i = threadIdx.x; i < K; i += blockDim.x) s += __expf(ld(xr, i) - m);
  s = block_reduce(s, red, false);
  float l = m + __logf(s);
  for (int i = threadIdx.x; i < K; i += blockDim.x) st(y + row * K, i, ld(xr, i) - l);
}

template <typename T>
__global__ void __launch_bounds__(256) k_logsoftmax_bwd(const T* __restrict__ gy, const T* __restrict__ y,
                                                        T* __restrict__ gx, int K) {
  __shared__ float red[8];
  const long long row = blockIdx.x;
  float s = 0.f;
  for (int i = threadIdx.x; i < K; i += blockDim.x) s += ld(gy + row * K, i);
  s = block_reduce(s, red, false);
  for (int i = threadIdx.x; i < K; i += blockDim.x)
    st(gx + row * K, i, ld(gy + row * K, i) - __expf(ld(y + row * K, i)) * s);
}

BIGDL_EXPORT int bigdl_logsoftmax(const void* a, const void* b, void* out, long long rows, int K, int backward,
                                  int dtype, hipStream_t s) {
  if (rows <= 0 || K <= 0) return (int)hipErrorInvalidValue;
  if (!backward) {
    if (dtype == 1) hipLaunchKernelGGL(k_logsoftmax_fwd<bf16_t>, dim3(rows), dim3(256), 0, s, (const bf16_t*)a, (bf16_t*)out, K);
    else hipLaunchKernelGGL(k_logsoftmax_fwd<float>, dim3(rows), dim3(256), 0, s, (const float*)a, (float*)out, K);
  } else {
    if (dtype == 1)
      hipLaunchKernelGGL(k_logsoftmax_bwd<bf16_t>, dim3(rows), dim3(256), 0, s, (const bf16_t*)a, (const bf16_t*)b,
                         (bf16_t*)out, K);
    else
      hipLaunchKernelGGL(k_logsoftmax_bwd<float>, dim3(rows), dim3(256), 0, s, (const float*)a, (const float*)b,
                         (float*)out, K);
  }
  BIGDL_CHECK_LAUNCH();
}

// ------------------------------------------------------------------------------------------------
// K12: row-wise softmax forward / backward over the last (memory-contiguous) dim — SoftMax.scala
// (1-D/2-D rows; on the NHWC device layout a 4-D channel softmax is also a contiguous-row softmax)
//   y = exp(x − max) / Σ exp(x − max);   gx = y · (gy − Σ gy·y)
// ------------------------------------------------------------------------------------------------
template <typename T>
__global__ void __launch_bounds__(256) k_softmax_fwd(const T* __restrict__ x, T* __restrict__ y, int K) {
  __shared__ float red[8];
  const long long row = blockIdx.x;
  const T* xr = x + row * K;
  float m = -INFINITY;
  for (int i = threadIdx.x; i < K; i += blockDim.x) m = fmaxf(m, ld(xr, i));
  m = block_reduce(m, red, true);
  float s = 0.f;
  for (int i = threadIdx.x; i < K; i += blockDim.x) s += __expf(ld(xr, i) - m);
  s = block_reduce(s, red, false);
  const float inv = 1.f / s;
  for (int i = threadIdx.x; i < K; i += blockDim.x) st(y + row * K, i, __expf(ld(xr, i) - m) * inv);
}

template <typename T>
__global__ void __launch_bounds__(256) k_softmax_bwd(const T* __restrict__ gy, const T* __restrict__ y,
                                                     T* __restrict__ gx, int K) {
  __shared__ float red[8];
  const long long row = blockIdx.x;
  float s = 0.f;
  for (int i = threadIdx.x; i < K; i += blockDim.x) s += ld(gy + row * K, i) * ld(y + row * K, i);
  s = block_reduce(s, red, false);
  for (int i = threadIdx.x; i < K; i += blockDim.x)
    st(gx + row * K, i, ld(y + row * K, i) * (ld(gy + row * K, i) - s));
}

BIGDL_EXPORT int bigdl_softmax(const void* a, const void* b, void* out, long long rows, int K, int backward, int dtype,
                               hipStream_t s) {
  if (rows <= 0 || K <= 0 || rows > 0x7fffffffLL) return (int)hipErrorInvalidValue;
  if (!backward) {
    if (dtype == 1) hipLaunchKernelGGL(k_softmax_fwd<bf16_t>, dim3(rows), dim3(256), 0, s, (const bf16_t*)a, (bf16_t*)out, K);
    else hipLaunchKernelGGL(k_softmax_fwd<float>, dim3(rows), dim3(256), 0, s, (const float*)a, (float*)out, K);
  } else {
    if (dtype == 1)
      hipLaunchKernelGGL(k_softmax_bwd<bf16_t>, dim3(rows), dim3(256), 0, s, (const bf16_t*)a, (const bf16_t*)b,
                         (bf16_t*)out, K);
    else
      hipLaunchKernelGGL(k_softmax_bwd<float>, dim3(rows), dim3(256), 0, s, (const float*)a, (const float*)b,
                         (float*)out, K);
  }
  BIGDL_CHECK_LAUNCH();
}

// ------------------------------------------------------------------------------------------------
// ClassNLLCriterion on log-probabilities (ClassNLLCriterion.scala:89-230, K13 without the fused
// log-softmax): loss = −Σ w[t]·logp[i][t] / (sizeAverage ? Σ w : 1) over rows whose 1-based target
// is not paddingValue; gradient −w[t]/denominator at the target column, zero elsewhere.  One block
// reduces the B rows (out[0] = loss, out[1] = denominator); the gradient kernel writes every element
// once (no separate zero fill) and reads the denominator from device memory.
// ------------------------------------------------------------------------------------------------
template <typename T>
__global__ void __launch_bounds__(256) k_nll_fwd(const T* __restrict__ lp, const int* __restrict__ tgt,
                                                 const float* __restrict__ cw, long long B, int K, int padding,
                                                 int size_avg, float* __restrict__ out) {
  __shared__ float red[8];
  float l = 0.f, wsum = 0.f;
  for (long long i = threadIdx.x; i < B; i += blockDim.x) {
    const int t = tgt[i];
    if (t == padding) continue;
    const int c = min(max(t - 1, 0), K - 1);
    const float w = cw ? cw[c] : 1.f;
    l -= w * ld(lp, i * K + c);
    wsum += w;
  }
  l = block_reduce(l, red, false);
  wsum = block_reduce(wsum, red, false);
  if (threadIdx.x == 0) {
    const float den = size_avg ? (cw ? fmaxf(wsum, 1e-12f) : fmaxf(wsum, 1.f)) : 1.f;
    out[0] = l / den;
    out[1] = den;
  }
}

template <typename T>
__global__ void __launch_bounds__(256) k_nll_bwd(const int* __restrict__ tgt, const float* __restrict__ cw,
                                                 const float* __restrict__ out, long long B, int K, int padding,
                                                 T* __restrict__ gx) {
  const float den = out[1];
  const long long total = B * K;
  for (long long e = blockIdx.x * (long long)blockDim.x + threadIdx.x; e < total; e += (long long)gridDim.x * blockDim.x) {
    const long long i = e / K;
    const int k = (int)(e - i * K);
    const int t = tgt[i];
    float v = 0.f;
    if (t != padding && k == min(max(t - 1, 0), K - 1)) v = -(cw ? cw[k] : 1.f) / den;
    st(gx, e, v);
  }
}

BIGDL_EXPORT int bigdl_class_nll(const void* lp, const int* tgt, const float* cw, void* gx, long long B, int K,
                                 int padding, int size_avg, int dtype, float* out, hipStream_t s) {
  if (B <= 0 || K <= 0) return (int)hipErrorInvalidValue;
  if (dtype == 1)
    hipLaunchKernelGGL(k_nll_fwd<bf16_t>, dim3(1), dim3(256), 0, s, (const bf16_t*)lp, tgt, cw, B, K, padding, size_avg, out);
  else
    hipLaunchKernelGGL(k_nll_fwd<float>, dim3(1), dim3(256), 0, s, (const float*)lp, tgt, cw, B, K, padding, size_avg, out);
  if (gx) {
    const int grid = bigdl_grid(B * K, 256, 4096);
    if (dtype == 1)
      hipLaunchKernelGGL(k_nll_bwd<bf16_t>, dim3(grid), dim3(256), 0, s, tgt, cw, out, B, K, padding, (bf16_t*)gx);
    else
      hipLaunchKernelGGL(k_nll_bwd<float>, dim3(grid), dim3(256), 0, s, tgt, cw, out, B, K, padding, (float*)gx);
  }
  BIGDL_CHECK_LAUNCH();
}
