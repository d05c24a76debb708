// K17: dropout forward/backward without a stored mask (Dropout.updateOutput / updateGradInput,
// DL/nn/Dropout.scala:64-150: drop with probability p, scale kept values by 1/(1-p)).
//
// The keep decision of element i is a pure function of (seed, i): Philox-4x32-10 counter-based RNG,
// counter = (block index of i, salt), key = seed.  Forward writes y = x·keep·scale; backward
// regenerates the same decisions from the same seed, so no mask tensor is ever written or read —
// each pass is exactly one read + one write of the activation (16 B per lane, 8 bf16 or 2×4 fp32).
#include "common.h"

struct U4 { uint32_t x, y, z, w; };

__device__ __forceinline__ void mulhilo(uint32_t a, uint32_t b, uint32_t& hi, uint32_t& lo) {
  const uint64_t p = (uint64_t)a * b;
  hi = (uint32_t)(p >> 32);
  lo = (uint32_t)p;
}

__device__ __forceinline__ U4 philox(U4 c, uint32_t k0, uint32_t k1) {
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    uint32_t h0, l0, h1, l1;
    mulhilo(0xD2511F53u, c.x, h0, l0);
    mulhilo(0xCD9E8D57u, c.z, h1, l1);
    c = U4{h1 ^ c.y ^ k0, l1, h0 ^ c.w ^ k1, l0};
    k0 += 0x9E3779B9u;
    k1 += 0xBB67AE85u;
  }
  return c;
}

// 8 keep flags for elements [8j, 8j+8): two Philox blocks of 4 uniforms
__device__ __forceinline__ void keep8(unsigned long long seed, long long j, uint32_t thresh, bool* keep) {
  const uint32_t k0 = (uint32_t)seed, k1 = (uint32_t)(seed >> 32);
  U4 a = philox(U4{(uint32_t)(2 * j), (uint32_t)((2 * j) >> 32), 0x5bd1e995u, 0u}, k0, k1);
  U4 b = philox(U4{(uint32_t)(2 * j + 1), (uint32_t)((2 * j + 1) >> 32), 0x5bd1e995u, 0u}, k0, k1);
  const uint32_t r[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
#pragma unroll
  for (int e = 0; e < 8; ++e) keep[e] = r[e] >= thresh;  // P(drop) = thresh / 2^32 = p
}

template <typename T>
__device__ __forceinline__ void ld8(const T* p, float* o);
template <>
__device__ __forceinline__ void ld8<bf16_t>(const bf16_t* p, float* o) { load8(p, o); }
template <>
__device__ __forceinline__ void ld8<float>(const float* p, float* o) {
  const float4 a = reinterpret_cast<const float4*>(p)[0], b = reinterpret_cast<const float4*>(p)[1];
  o[0] = a.x; o[1] = a.y; o[2] = a.z; o[3] = a.w; o[4] = b.x; o[5] = b.y; o[6] = b.z; o[7] = b.w;
}
template <typename T>
__device__ __forceinline__ void st8(T* p, const float* o);
template <>
__device__ __forceinline__ void st8<bf16_t>(bf16_t* p, const float* o) { store8(p, o); }
template <>
__device__ __forceinline__ void st8<float>(float* p, const float* o) {
  reinterpret_cast<float4*>(p)[0] = make_float4(o[0], o[1], o[2], o[3]);
  reinterpret_cast<float4*>(p)[1] = make_float4(o[4], o[5], o[6], o[7]);
}
__device__ __forceinline__ float ldx(const bf16_t* p) { return bf2f(*p); }
__device__ __forceinline__ float ldx(const float* p) { return *p; }
__device__ __forceinline__ void stx(bf16_t* p, float v) { *p = f2bf(v); }
__device__ __forceinline__ void stx(float* p, float v) { *p = v; }

// y = x · keep · scale  (the same kernel is the backward: x ← gy)
template <typename T>
__global__ void __launch_bounds__(256) k_dropout(const T* __restrict__ x, T* __restrict__ y, long long n,
                                                 unsigned long long seed, uint32_t thresh, float scale,
                                                 const unsigned long long* __restrict__ seed_ptr) {
  // graph-captured launches read the seed from device memory (a counter advanced inside the graph),
  // so every replay draws a fresh mask
  if (seed_ptr) seed = *seed_ptr;
  const long long groups = n >> 3;
  for (long long j = blockIdx.x * (long long)blockDim.x + threadIdx.x; j < groups;
       j += (long long)gridDim.x * blockDim.x) {
    bool keep[8];
    keep8(seed, j, thresh, keep);
    float v[8];
    ld8<T>(x + 8 * j, v);
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] = keep[e] ? v[e] * scale : 0.f;
    st8<T>(y + 8 * j, v);
  }
  // tail (n % 8 elements): one thread
  if (blockIdx.x == 0 && threadIdx.x == 0 && (n & 7)) {
    bool keep[8];
    keep8(seed, groups, thresh, keep);
    for (long long i = groups * 8; i < n; ++i) stx(y + i, keep[i - groups * 8] ? ldx(x + i) * scale : 0.f);
  }
}

static int dropout_launch(const void* x, void* y, long long n, int dtype, float p, unsigned long long seed,
                          const unsigned long long* seed_ptr, hipStream_t s);

// dtype: 0 = bf16, 1 = fp32.  p ∈ [0, 1): drop probability.  Pointers 16-B aligned.
BIGDL_EXPORT int bigdl_dropout(const void* x, void* y, long long n, int dtype, float p, unsigned long long seed,
                               hipStream_t s) {
  return dropout_launch(x, y, n, dtype, p, seed, nullptr, s);
}

// Same, seed read on the device from `seed_ptr` (HIP-graph capture).
BIGDL_EXPORT int bigdl_dropout_devseed(const void* x, void* y, long long n, int dtype, float p,
                                       const unsigned long long* seed_ptr, hipStream_t s) {
  if (!seed_ptr) return (int)hipErrorInvalidValue;
  return dropout_launch(x, y, n, dtype, p, 0ull, seed_ptr, s);
}

static int dropout_launch(const void* x, void* y, long long n, int dtype, float p, unsigned long long seed,
                          const unsigned long long* seed_ptr, hipStream_t s) {
  if (n <= 0 || p < 0.f || p >= 1.f || ((uintptr_t)x & 15) || ((uintptr_t)y & 15) || dtype < 0 || dtype > 1)
    return (int)hipErrorInvalidValue;
  double t = (double)p * 4294967296.0;
  if (t > 4294967295.0) t = 4294967295.0;
  const uint32_t thresh = (uint32_t)t;
  const float scale = 1.f / (1.f - p);
  const int grid = bigdl_grid((n >> 3) + 1, 256, 16384);
  if (dtype == 0)
    hipLaunchKernelGGL(k_dropout<bf16_t>, dim3(grid), dim3(256), 0, s, (const bf16_t*)x, (bf16_t*)y, n, seed, thresh,
                       scale, seed_ptr);
  else
    hipLaunchKernelGGL(k_dropout<float>, dim3(grid), dim3(256), 0, s, (const float*)x, (float*)y, n, seed, thresh,
                       scale, seed_ptr);
  BIGDL_CHECK_LAUNCH();
}
