// CSR sparse × dense products (K27; reference SparseTensorBLAS.coomm / SparseLinear.scala).
//
// out[m][n] = alpha · Σ_j val[j] · B[col[j]][n] + beta · out[m][n]  for j in rowptr[m] .. rowptr[m+1]
//
// One wave owns one output row and walks its non-zeros in order (no atomics, so the result is
// deterministic); the 64 lanes sweep the row's N columns 4 at a time (16-B loads of B, 16-B
// stores of out).  B is fp32 or bf16; accumulation and output are fp32.  The transposed product
// (the sparse layer's weight gradient Xᵀ·G) runs through the same kernel on the CSR of Xᵀ, built
// on the host side, instead of scatter-adding with atomics.
#include "common.h"

template <typename TB>
__device__ __forceinline__ float4 ld4(const TB* p);
template <>
__device__ __forceinline__ float4 ld4<float>(const float* p) {
  return *reinterpret_cast<const float4*>(p);
}
template <>
__device__ __forceinline__ float4 ld4<bf16_t>(const bf16_t* p) {
  const uint2 u = *reinterpret_cast<const uint2*>(p);
  return make_float4(__uint_as_float(u.x << 16), __uint_as_float(u.x & 0xFFFF0000u), __uint_as_float(u.y << 16),
                     __uint_as_float(u.y & 0xFFFF0000u));
}

template <typename TB, typename TI>
__global__ void __launch_bounds__(256) k_spmm_csr(const TI* __restrict__ rowptr, const TI* __restrict__ col,
                                                  const float* __restrict__ val, const TB* __restrict__ B,
                                                  float* __restrict__ out, int M, int N, long long ldb,
                                                  long long ldo, float alpha, float beta) {
  const int m = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (m >= M) return;
  const int lane = threadIdx.x & 63;
  const long long j0 = rowptr[m], j1 = rowptr[m + 1];
  float* o = out + (long long)m * ldo;
  for (int n = lane * 4; n < N; n += 256) {
    float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
    for (long long j = j0; j < j1; ++j) {
      const float v = val[j];
      const float4 b = ld4<TB>(B + (long long)col[j] * ldb + n);
      acc.x = fmaf(v, b.x, acc.x);
      acc.y = fmaf(v, b.y, acc.y);
      acc.z = fmaf(v, b.z, acc.z);
      acc.w = fmaf(v, b.w, acc.w);
    }
    float4 r = make_float4(alpha * acc.x, alpha * acc.y, alpha * acc.z, alpha * acc.w);
    if (beta != 0.f) {
      const float4 p = *reinterpret_cast<const float4*>(o + n);
      r.x = fmaf(beta, p.x, r.x);
      r.y = fmaf(beta, p.y, r.y);
      r.z = fmaf(beta, p.z, r.z);
      r.w = fmaf(beta, p.w, r.w);
    }
    *reinterpret_cast<float4*>(o + n) = r;
  }
}

// itype: 0 = int32 indices, 1 = int64; btype: 0 = fp32 B, 1 = bf16 B.  Requirements (checked):
// N % 4 == 0, ldb/ldo multiples of 4 (16-B / 8-B aligned rows), B/out 16-B aligned.
BIGDL_EXPORT int bigdl_spmm_csr(const void* rowptr, const void* col, const float* val, int itype, const void* B,
                                int btype, float* out, int M, int N, long long ldb, long long ldo, float alpha,
                                float beta, hipStream_t s) {
  if (M <= 0 || N <= 0 || N % 4 || ldb % 4 || ldo % 4 || ldb < N || ldo < N) return (int)hipErrorInvalidValue;
  if (((uintptr_t)out & 15) || ((uintptr_t)B & (btype ? 7 : 15))) return (int)hipErrorInvalidValue;
  const dim3 g((unsigned)((M + 3) / 4));
  if (itype == 0 && btype == 0)
    hipLaunchKernelGGL((k_spmm_csr<float, int>), g, dim3(256), 0, s, (const int*)rowptr, (const int*)col, val,
                       (const float*)B, out, M, N, ldb, ldo, alpha, beta);
  else if (itype == 0)
    hipLaunchKernelGGL((k_spmm_csr<bf16_t, int>), g, dim3(256), 0, s, (const int*)rowptr, (const int*)col, val,
                       (const bf16_t*)B, out, M, N, ldb, ldo, alpha, beta);
  else if (btype == 0)
    hipLaunchKernelGGL((k_spmm_csr<float, long long>), g, dim3(256), 0, s, (const long long*)rowptr,
                       (const long long*)col, val, (const float*)B, out, M, N, ldb, ldo, alpha, beta);
  else
    hipLaunchKernelGGL((k_spmm_csr<bf16_t, long long>), g, dim3(256), 0, s, (const long long*)rowptr,
                       (const long long*)col, val, (const bf16_t*)B, out, M, N, ldb, ldo, alpha, beta);
  BIGDL_CHECK_LAUNCH();
}
