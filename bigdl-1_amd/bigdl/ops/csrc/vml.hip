// Vector math (N2 / K20 / K21): the reference's MKL VML calls behind TensorNumeric
// (tensor/TensorNumeric.scala:600-700: vsAdd/vsSub/vsMul/vsDiv, vsExp, vsLn, vsLog1p, vsSqrt,
// vsTanh, vsAbs, vsPowx) plus the elementwise-layer gradients and dimension reductions.
//
// Elementwise: contiguous fp32 or bf16 tensors, 16 B per lane per access (4 fp32 / 8 bf16), fp32
// math, a grid-stride loop over 16-B groups and a scalar tail.  The op code is a template
// parameter so each instantiation is a straight-line body.
//
// Reductions over the middle dimension of a [outer][n][inner] view, fp32 accumulation and output:
//  * inner == 1 (rows contiguous): each row is cut into S segments, one wave per segment (lanes
//    stride the segment, DPP/shuffle fold), then a second tiny launch folds the S partials of
//    each row in a fixed order — deterministic and parallel for one huge row as well as for many
//    short ones;
//  * inner > 1: one thread per (outer, inner) column walks n (consecutive threads read
//    consecutive addresses).
#include "common.h"

#include <utility>

enum : int {
  U_ABS = 0, U_EXP, U_LN, U_LOG1P, U_SQRT, U_TANH, U_SIGMOID, U_POWX, U_SQUARE, U_INV, U_NEG, U_AFFINE,
  U_COUNT
};
enum : int {
  B_ADD = 0, B_SUB, B_MUL, B_DIV, B_TANH_BWD, B_SIGMOID_BWD, B_SQRT_BWD, B_LOG_BWD, B_EXP_BWD, B_SQUARE_BWD,
  B_ABS_BWD, B_POW_BWD, B_COUNT
};

template <int OP>
__device__ __forceinline__ float unary(float x, float p, float q) {
  if constexpr (OP == U_ABS) return fabsf(x);
  else if constexpr (OP == U_EXP) return __expf(x);
  else if constexpr (OP == U_LN) return __logf(x);
  else if constexpr (OP == U_LOG1P) return log1pf(x);
  else if constexpr (OP == U_SQRT) return sqrtf(x);
  else if constexpr (OP == U_TANH) return tanhf(x);
  else if constexpr (OP == U_SIGMOID) return 1.f / (1.f + __expf(-x));
  else if constexpr (OP == U_POWX) return powf(x, p);
  else if constexpr (OP == U_SQUARE) return x * x;
  else if constexpr (OP == U_INV) return 1.f / x;
  else if constexpr (OP == U_NEG) return -x;
  else return fmaf(x, p, q);  // U_AFFINE
}

// z = f(a, b); for the *_BWD codes a is the upstream gradient and b the saved forward value
// (output for tanh / sigmoid / sqrt / exp, input for log / square / abs / pow)
template <int OP>
__device__ __forceinline__ float binary(float a, float b, float p) {
  if constexpr (OP == B_ADD) return fmaf(p, b, a);
  else if constexpr (OP == B_SUB) return fmaf(-p, b, a);
  else if constexpr (OP == B_MUL) return a * b;
  else if constexpr (OP == B_DIV) return a / b;
  else if constexpr (OP == B_TANH_BWD) return a * (1.f - b * b);
  else if constexpr (OP == B_SIGMOID_BWD) return a * b * (1.f - b);
  else if constexpr (OP == B_SQRT_BWD) return 0.5f * a / b;
  else if constexpr (OP == B_LOG_BWD) return a / b;
  else if constexpr (OP == B_EXP_BWD) return a * b;
  else if constexpr (OP == B_SQUARE_BWD) return 2.f * a * b;
  else if constexpr (OP == B_ABS_BWD) return b > 0.f ? a : (b < 0.f ? -a : 0.f);
  else return a * p * powf(b, p - 1.f);  // B_POW_BWD
}

template <typename T>
struct Vec;
template <>
struct Vec<float> {
  static constexpr int N = 4;
  __device__ static void ld(const float* p, float* o) {
    const float4 v = *reinterpret_cast<const float4*>(p);
    o[0] = v.x; o[1] = v.y; o[2] = v.z; o[3] = v.w;
  }
  __device__ static void st(float* p, const float* o) {
    *reinterpret_cast<float4*>(p) = make_float4(o[0], o[1], o[2], o[3]);
  }
  __device__ static float get(const float* p) { return *p; }
  __device__ static void put(float* p, float v) { *p = v; }
};
template <>
struct Vec<bf16_t> {
  static constexpr int N = 8;
  __device__ static void ld(const bf16_t* p, float* o) { load8(p, o); }
  __device__ static void st(bf16_t* p, const float* o) { store8(p, o); }
  __device__ static float get(const bf16_t* p) { return bf2f(*p); }
  __device__ static void put(bf16_t* p, float v) { *p = f2bf(v); }
};

template <typename T, int OP>
__global__ void __launch_bounds__(256) k_vml_unary(const T* __restrict__ x, T* __restrict__ y, long long n, float p,
                                                   float q) {
  constexpr int V = Vec<T>::N;
  const long long nv = n / V;
  const long long stride = (long long)gridDim.x * blockDim.x;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < nv; i += stride) {
    float v[V];
    Vec<T>::ld(x + i * V, v);
#pragma unroll
    for (int k = 0; k < V; ++k) v[k] = unary<OP>(v[k], p, q);
    Vec<T>::st(y + i * V, v);
  }
  for (long long i = nv * V + blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n; i += stride)
    Vec<T>::put(y + i, unary<OP>(Vec<T>::get(x + i), p, q));
}

template <typename T, int OP>
__global__ void __launch_bounds__(256) k_vml_binary(const T* __restrict__ a, const T* __restrict__ b, T* __restrict__ z,
                                                    long long n, float p) {
  constexpr int V = Vec<T>::N;
  const long long nv = n / V;
  const long long stride = (long long)gridDim.x * blockDim.x;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < nv; i += stride) {
    float va[V], vb[V];
    Vec<T>::ld(a + i * V, va);
    Vec<T>::ld(b + i * V, vb);
#pragma unroll
    for (int k = 0; k < V; ++k) va[k] = binary<OP>(va[k], vb[k], p);
    Vec<T>::st(z + i * V, va);
  }
  for (long long i = nv * V + blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n; i += stride)
    Vec<T>::put(z + i, binary<OP>(Vec<T>::get(a + i), Vec<T>::get(b + i), p));
}

template <typename T, int OP>
static void launch_unary(const void* x, void* y, long long n, float p, float q, hipStream_t s) {
  const int g = bigdl_grid((n + Vec<T>::N - 1) / Vec<T>::N, 256, 8192);
  hipLaunchKernelGGL((k_vml_unary<T, OP>), dim3(g), dim3(256), 0, s, (const T*)x, (T*)y, n, p, q);
}

template <typename T, int OP>
static void launch_binary(const void* a, const void* b, void* z, long long n, float p, hipStream_t s) {
  const int g = bigdl_grid((n + Vec<T>::N - 1) / Vec<T>::N, 256, 8192);
  hipLaunchKernelGGL((k_vml_binary<T, OP>), dim3(g), dim3(256), 0, s, (const T*)a, (const T*)b, (T*)z, n, p);
}

template <typename T, int... OPS>
static bool dispatch_unary(int op, const void* x, void* y, long long n, float p, float q, hipStream_t s,
                           std::integer_sequence<int, OPS...>) {
  bool done = false;
  ((op == OPS ? (launch_unary<T, OPS>(x, y, n, p, q, s), done = true) : false), ...);
  return done;
}

template <typename T, int... OPS>
static bool dispatch_binary(int op, const void* a, const void* b, void* z, long long n, float p, hipStream_t s,
                            std::integer_sequence<int, OPS...>) {
  bool done = false;
  ((op == OPS ? (launch_binary<T, OPS>(a, b, z, n, p, s), done = true) : false), ...);
  return done;
}

// dtype 0 = fp32, 1 = bf16; all operands contiguous with n elements, 16-B aligned
BIGDL_EXPORT int bigdl_vml_unary(int op, int dtype, const void* x, void* y, long long n, float p, float q,
                                 hipStream_t s) {
  if (n <= 0 || op < 0 || op >= U_COUNT || ((uintptr_t)x & 15) || ((uintptr_t)y & 15)) return (int)hipErrorInvalidValue;
  const bool ok = dtype == 0 ? dispatch_unary<float>(op, x, y, n, p, q, s, std::make_integer_sequence<int, U_COUNT>{})
                             : dispatch_unary<bf16_t>(op, x, y, n, p, q, s, std::make_integer_sequence<int, U_COUNT>{});
  if (!ok) return (int)hipErrorInvalidValue;
  BIGDL_CHECK_LAUNCH();
}

BIGDL_EXPORT int bigdl_vml_binary(int op, int dtype, const void* a, const void* b, void* z, long long n, float p,
                                  hipStream_t s) {
  if (n <= 0 || op < 0 || op >= B_COUNT || ((uintptr_t)a & 15) || ((uintptr_t)b & 15) || ((uintptr_t)z & 15))
    return (int)hipErrorInvalidValue;
  const bool ok = dtype == 0
                      ? dispatch_binary<float>(op, a, b, z, n, p, s, std::make_integer_sequence<int, B_COUNT>{})
                      : dispatch_binary<bf16_t>(op, a, b, z, n, p, s, std::make_integer_sequence<int, B_COUNT>{});
  if (!ok) return (int)hipErrorInvalidValue;
  BIGDL_CHECK_LAUNCH();
}

// ------------------------------------------------------------------------------------------------ reductions
enum : int { R_SUM = 0, R_MEAN, R_MAX, R_MIN };

template <int OP>
__device__ __forceinline__ float rinit() {
  if constexpr (OP == R_MAX) return -INFINITY;
  else if constexpr (OP == R_MIN) return INFINITY;
  else return 0.f;
}

template <int OP>
__device__ __forceinline__ float rcomb(float a, float b) {
  if constexpr (OP == R_MAX) return fmaxf(a, b);
  else if constexpr (OP == R_MIN) return fminf(a, b);
  else return a + b;
}

template <int OP>
__device__ __forceinline__ float wave_reduce(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = rcomb<OP>(v, __shfl_xor(v, o, 64));
  return v;
}

// rows contiguous: partial[row][seg] over elements [seg·L, min(n, (seg+1)·L)) of the row; 4 waves
// per block, one (row, seg) per wave
template <typename T, int OP>
__global__ void __launch_bounds__(256) k_reduce_rows(const T* __restrict__ x, long long rows, long long n, int S,
                                                     long long L, float* __restrict__ partial) {
  const long long task = blockIdx.x * 4ll + (threadIdx.x >> 6);
  if (task >= rows * S) return;
  const int lane = threadIdx.x & 63;
  const long long row = task / S;
  const int seg = (int)(task - row * S);
  const long long b = seg * L;
  long long e = b + L;
  if (e > n) e = n;
  const T* xr = x + row * n;
  float acc = rinit<OP>();
  for (long long i = b + lane; i < e; i += 64) acc = rcomb<OP>(acc, Vec<T>::get(xr + i));
  acc = wave_reduce<OP>(acc);
  if (lane == 0) partial[task] = acc;
}

template <int OP>
__global__ void __launch_bounds__(256) k_reduce_fold(const float* __restrict__ partial, long long rows, int S,
                                                     float scale, float* __restrict__ out) {
  const long long r = blockIdx.x * 256ll + threadIdx.x;
  if (r >= rows) return;
  float acc = rinit<OP>();
  for (int k = 0; k < S; ++k) acc = rcomb<OP>(acc, partial[r * S + k]);
  out[r] = OP == R_MEAN ? acc * scale : acc;
}

template <typename T, int OP>
__global__ void __launch_bounds__(256) k_reduce_cols(const T* __restrict__ x, long long outer, long long n,
                                                     long long inner, float scale, float* __restrict__ out) {
  const long long c = blockIdx.x * 256ll + threadIdx.x;
  if (c >= outer * inner) return;
  const long long o = c / inner, i = c - o * inner;
  const T* p = x + o * n * inner + i;
  float acc = rinit<OP>();
  for (long long k = 0; k < n; ++k) acc = rcomb<OP>(acc, Vec<T>::get(p + k * inner));
  out[c] = OP == R_MEAN ? acc * scale : acc;
}

template <typename T, int OP>
static int reduce_launch(const void* x, long long outer, long long n, long long inner, float* out, float* scratch,
                         long long scratch_len, hipStream_t s) {
  const float scale = 1.f / (float)n;
  if (inner == 1 && n > 64) {
    // segments per row: enough waves to fill the chip, ≥ 2048 elements each
    long long S = (n + 2047) / 2048;
    const long long want = (8192 + outer - 1) / outer;
    if (S > want) S = want;
    if (S < 1) S = 1;
    if (outer * S > scratch_len) S = scratch_len / outer;
    if (S < 1) return (int)hipErrorInvalidValue;
    const long long L = (n + S - 1) / S;
    const long long tasks = outer * S;
    hipLaunchKernelGGL((k_reduce_rows<T, OP>), dim3((unsigned)((tasks + 3) / 4)), dim3(256), 0, s, (const T*)x, outer,
                       n, (int)S, L, scratch);
    hipLaunchKernelGGL((k_reduce_fold<OP>), dim3((unsigned)((outer + 255) / 256)), dim3(256), 0, s, scratch, outer,
                       (int)S, scale, out);
  } else {
    const long long cols = outer * inner;
    hipLaunchKernelGGL((k_reduce_cols<T, OP>), dim3((unsigned)((cols + 255) / 256)), dim3(256), 0, s, (const T*)x,
                       outer, n, inner, scale, out);
  }
  BIGDL_CHECK_LAUNCH();
}

// out[outer][inner] (fp32) = reduce over n of x[outer][n][inner]; scratch: ≥ outer floats (more
// lets a long row split into more segments) — used only when inner == 1
BIGDL_EXPORT int bigdl_reduce(int op, int dtype, const void* x, long long outer, long long n, long long inner, float* out,
                              float* scratch, long long scratch_len, hipStream_t s) {
  if (outer <= 0 || n <= 0 || inner <= 0 || (outer * inner) >= (1ll << 40)) return (int)hipErrorInvalidValue;
  if ((outer * inner + 255) / 256 > 0x7fffffffll) return (int)hipErrorInvalidValue;
#define BIGDL_RED(T)                                                                                  \
  switch (op) {                                                                                       \
    case R_SUM: return reduce_launch<T, R_SUM>(x, outer, n, inner, out, scratch, scratch_len, s);     \
    case R_MEAN: return reduce_launch<T, R_MEAN>(x, outer, n, inner, out, scratch, scratch_len, s);   \
    case R_MAX: return reduce_launch<T, R_MAX>(x, outer, n, inner, out, scratch, scratch_len, s);     \
    case R_MIN: return reduce_launch<T, R_MIN>(x, outer, n, inner, out, scratch, scratch_len, s);     \
    default: return (int)hipErrorInvalidValue;                                                        \
  }
  if (dtype == 0) { BIGDL_RED(float) } else { BIGDL_RED(bf16_t) }
#undef BIGDL_RED
}
