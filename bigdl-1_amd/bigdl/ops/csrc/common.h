// Common helpers for the bigdl HIP/CDNA4 kernels (gfx950 only).
//
// Conventions
//  * every exported launcher is `extern "C" int bigdl_<op>(..., hipStream_t)` returning hipError_t;
//  * activations are NHWC bf16 (`bf16_t`), accumulation / statistics / master weights fp32;
//  * memory-bound kernels move 16 B per lane (8 bf16 or 4 fp32) — CDNA4 has no auto-vectorised
//    bf16 loads (cdna_hip_programming.md Guideline 13);
//  * wave64: reductions use 64-lane shuffles, block sizes are multiples of 64.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef unsigned short bf16_t;

#define BIGDL_EXPORT extern "C" __attribute__((visibility("default")))

__device__ __forceinline__ float bf2f(bf16_t v) {
  return __uint_as_float(((uint32_t)v) << 16);
}

// round-to-nearest-even fp32 -> bf16 (hipcc lowers the __bf16 cast to v_cvt_pk_bf16_f32 on gfx950,
// which also keeps NaNs NaN — MI355X_MICROARCH.md 'Correctness boundaries')
__device__ __forceinline__ bf16_t f2bf(float f) {
  __bf16 b = (__bf16)f;
  return *reinterpret_cast<bf16_t*>(&b);
}

struct __attribute__((aligned(16))) bf16x8 { bf16_t v[8]; };

__device__ __forceinline__ void load8(const bf16_t* p, float* o) {
  uint4 u = *reinterpret_cast<const uint4*>(p);
  const uint32_t w[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    o[2 * i] = __uint_as_float(w[i] << 16);
    o[2 * i + 1] = __uint_as_float(w[i] & 0xFFFF0000u);
  }
}

// streaming (non-temporal) variant: for operands read once per pass whose next use is far away
// (BN apply / backward-apply inputs), so they do not displace reusable lines from L2 / MALL
typedef unsigned int bigdl_u32x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ void load8_nt(const bf16_t* p, float* o) {
  const bigdl_u32x4 u = __builtin_nontemporal_load(reinterpret_cast<const bigdl_u32x4*>(p));
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    o[2 * i] = __uint_as_float(u[i] << 16);
    o[2 * i + 1] = __uint_as_float(u[i] & 0xFFFF0000u);
  }
}

__device__ __forceinline__ void unpack8(uint4 u, float* o) {
  const uint32_t w[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    o[2 * i] = __uint_as_float(w[i] << 16);
    o[2 * i + 1] = __uint_as_float(w[i] & 0xFFFF0000u);
  }
}

__device__ __forceinline__ void store8(bf16_t* p, const float* o) {
  uint32_t w[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    w[i] = (uint32_t)f2bf(o[2 * i]) | ((uint32_t)f2bf(o[2 * i + 1]) << 16);
  }
  *reinterpret_cast<uint4*>(p) = make_uint4(w[0], w[1], w[2], w[3]);
}

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

static inline int bigdl_grid(long long work, int block, int cap = 2048) {
  long long g = (work + block - 1) / block;
  if (g < 1) g = 1;
  if (g > cap) g = cap;
  return (int)g;
}

#define BIGDL_CHECK_LAUNCH() return (int)hipGetLastError()

// Deterministic mode (bigdl.deterministic): kernels that reduce with float atomics
// from several blocks (split-K wgrad, column sums, embedding scatter-add) switch to a single
// writer per output element, so two runs on the same inputs are bit-identical.  Set from Python
// through bigdl_set_deterministic(); defined in registry.cpp.
extern int g_bigdl_deterministic;
