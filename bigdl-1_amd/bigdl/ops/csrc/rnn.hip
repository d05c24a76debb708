// Fused LSTM pointwise step, forward and backward (K14 in SURVEY §2.15).
// Reference graph: DL/nn/LSTM.scala:124-187 — gates (i, g, f, o) in blocks of H along the last
// dim, i/f/o = sigmoid, g = tanh, c' = i*g + f*c, h' = o*tanh(c').
//
// One launch per time step replaces the reference's CAddTable + Reshape + 4 Select + 4
// activations + 3 CMulTable + CAddTable + Tanh modules.  The gate sum (input projection +
// recurrent projection) is formed in fp32 here, h is written straight into the (B, T, H)
// sequence output (row stride ldh), and the saved activations / tanh(c) / c are fp32 so the
// backward step needs no recomputation.  Backward fuses the add of the recurrent gradient
// (dL/dh from step t+1's dgrad GEMM) with the output gradient.
#include "common.h"

template <typename T> __device__ __forceinline__ float ld(const T* p);
template <> __device__ __forceinline__ float ld<float>(const float* p) { return *p; }
template <> __device__ __forceinline__ float ld<bf16_t>(const bf16_t* p) { return bf2f(*p); }
template <typename T> __device__ __forceinline__ void st(T* p, float v);
template <> __device__ __forceinline__ void st<float>(float* p, float v) { *p = v; }
template <> __device__ __forceinline__ void st<bf16_t>(bf16_t* p, float v) { *p = f2bf(v); }

__device__ __forceinline__ float sigm(float x) { return 1.f / (1.f + __expf(-x)); }

template <typename T>
__global__ void __launch_bounds__(256) k_lstm_fwd(const T* __restrict__ xg, long ldx, const T* __restrict__ hg,
                                                  long ldhg, const float* __restrict__ c_prev,
                                                  T* __restrict__ h_out, long ldh, float* __restrict__ c_out,
                                                  float* __restrict__ act, float* __restrict__ tc_out, int B,
                                                  int H) {
  const long idx = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= (long)B * H) return;
  const int b = (int)(idx / H), j = (int)(idx - (long)b * H);
  const T* x = xg + b * ldx;
  float gi = ld(x + j), gg = ld(x + H + j), gf = ld(x + 2 * H + j), go = ld(x + 3 * H + j);
  if (hg) {
    const T* r = hg + b * ldhg;
    gi += ld(r + j);
    gg += ld(r + H + j);
    gf += ld(r + 2 * H + j);
    go += ld(r + 3 * H + j);
  }
  const float i = sigm(gi), g = tanhf(gg), f = sigm(gf), o = sigm(go);
  const float c = i * g + f * c_prev[idx];
  const float tc = tanhf(c);
  st(h_out + b * ldh + j, o * tc);
  if (c_out) c_out[idx] = c;
  if (act) {
    float* a = act + (long)b * 4 * H;
    a[j] = i;
    a[H + j] = g;
    a[2 * H + j] = f;
    a[3 * H + j] = o;
  }
  if (tc_out) tc_out[idx] = tc;
}

template <typename T>
__global__ void __launch_bounds__(256) k_lstm_bwd(const T* __restrict__ gh, long ldgh, const T* __restrict__ gh2,
                                                  const float* __restrict__ gc_next, const float* __restrict__ act,
                                                  const float* __restrict__ tc, const float* __restrict__ c_prev,
                                                  T* __restrict__ dg, long lddg, float* __restrict__ dc_prev, int B,
                                                  int H) {
  const long idx = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= (long)B * H) return;
  const int b = (int)(idx / H), j = (int)(idx - (long)b * H);
  float d_h = ld(gh + b * ldgh + j);
  if (gh2) d_h += ld(gh2 + idx);
  const float* a = act + (long)b * 4 * H;
  const float i = a[j], g = a[H + j], f = a[2 * H + j], o = a[3 * H + j];
  const float t = tc[idx];
  float dc = d_h * o * (1.f - t * t);
  if (gc_next) dc += gc_next[idx];
  const float d_o = d_h * t;
  T* out = dg + b * lddg;
  st(out + j, dc * g * i * (1.f - i));
  st(out + H + j, dc * i * (1.f - g * g));
  st(out + 2 * H + j, dc * c_prev[idx] * f * (1.f - f));
  st(out + 3 * H + j, d_o * o * (1.f - o));
  dc_prev[idx] = dc * f;
}

// dtype: 0 = bf16 activations (xg, hg, h_out / gh, gh2, dg), 1 = fp32
BIGDL_EXPORT int bigdl_lstm_fwd(const void* xg, long ldx, const void* hg, long ldhg, const float* c_prev,
                                void* h_out, long ldh, float* c_out, float* act, float* tc, int B, int H, int dtype,
                                hipStream_t s) {
  if (B <= 0 || H <= 0) return (int)hipErrorInvalidValue;
  const long n = (long)B * H;
  dim3 grid((unsigned)((n + 255) / 256)), block(256);
  if (dtype == 0)
    hipLaunchKernelGGL(k_lstm_fwd<bf16_t>, grid, block, 0, s, (const bf16_t*)xg, ldx, (const bf16_t*)hg, ldhg,
                       c_prev, (bf16_t*)h_out, ldh, c_out, act, tc, B, H);
  else
    hipLaunchKernelGGL(k_lstm_fwd<float>, grid, block, 0, s, (const float*)xg, ldx, (const float*)hg, ldhg, c_prev,
                       (float*)h_out, ldh, c_out, act, tc, B, H);
  BIGDL_CHECK_LAUNCH();
}

BIGDL_EXPORT int bigdl_lstm_bwd(const void* gh, long ldgh, const void* gh2, const float* gc_next, const float* act,
                                const float* tc, const float* c_prev, void* dg, long lddg, float* dc_prev, int B,
                                int H, int dtype, hipStream_t s) {
  if (B <= 0 || H <= 0) return (int)hipErrorInvalidValue;
  const long n = (long)B * H;
  dim3 grid((unsigned)((n + 255) / 256)), block(256);
  if (dtype == 0)
    hipLaunchKernelGGL(k_lstm_bwd<bf16_t>, grid, block, 0, s, (const bf16_t*)gh, ldgh, (const bf16_t*)gh2, gc_next,
                       act, tc, c_prev, (bf16_t*)dg, lddg, dc_prev, B, H);
  else
    hipLaunchKernelGGL(k_lstm_bwd<float>, grid, block, 0, s, (const float*)gh, ldgh, (const float*)gh2, gc_next,
                       act, tc, c_prev, (float*)dg, lddg, dc_prev, B, H);
  BIGDL_CHECK_LAUNCH();
}
