// Fused recurrent time step: the h·Uᵀ recurrent GEMM on MFMA and the cell's pointwise math in ONE
// launch per step (K14 persistent-style LSTM step, K15 GRU).  Reference graphs: DL/nn/LSTM.scala:
// 124-187 (gates i, g, f, o), DL/nn/GRU.scala (r, z, ĥ = tanh(x_h + U_h(r∘h)), h' = (1−z)ĥ + z h),
// time loop / BPTT DL/nn/Recurrent.scala:283-400.
//
// Gate-grouped tiling: a block owns 16 hidden units j0..j0+15 and 32 batch rows, and computes the
// G gate groups of those units (LSTM: 4 tiles = rows g·H + j of U).  mfma_f32_16x16x32_bf16 with
// the weight row as the MFMA "A" side leaves, in each lane, the SAME (batch row, 4 consecutive
// units) for every gate tile — so the cell update runs in registers right after the MFMAs, with no
// LDS exchange between gates.  The reduction dim is split over the block's 4 waves (the per-step
// GEMMs are tiny and latency-bound: B·4H·H ≈ 20·800·200) and folded through LDS.  Fragments are
// read straight from global/L2 (each U row is used by one block only; h rows are L2-resident).
//
// Cells (template CELL):
//   0 LSTM forward   (G=4)  A = h_{t-1} [M][H],  U [4H][H]:  gates = xg + h Uᵀ → h, c (+ saves)
//   1 LSTM backward  (G=1)  A = dg_{t+1} [M][4H], Uᵀ [H][4H]: dh = gy + dg_{t+1} U → dg_t, dc_{t-1}
//   2 GRU forward 1  (G=2)  A = h_{t-1},  U_rz [2H][H]: r, z = σ(x_rz + h U_rzᵀ), rh = r∘h
//   3 GRU forward 2  (G=1)  A = rh,       U_h [H][H]:   n = tanh(x_h + rh U_hᵀ), h' = (1−z)n + z h
//   4 GRU backward 1 (G=1)  A = da_rz_{t+1}, U_rzᵀ [H][2H]: dh' = gy + carry + da_rz U_rz → da_z, da_n
//   5 GRU backward 2 (G=1)  A = da_n_t,   U_hᵀ [H][H]:  drh = da_n U_h → da_r, carry += drh∘r
#include "common.h"

typedef short v8s __attribute__((ext_vector_type(8)));
typedef float v4f __attribute__((ext_vector_type(4)));

struct RnnStep {
  const bf16_t* a;  // A operand rows [M][K] (row stride lda); null = zero (first / last step)
  long long lda;
  const bf16_t* u;  // B operand rows [G·Hs][K], contiguous
  int M, K, Hs;
  const void* xg;  // input projection rows (bf16, or fp32 when x_f32), row stride ldx
  long long ldx;
  int x_f32;
  const bf16_t* hprev;  // h_{t-1} rows (GRU), row stride ldhp
  long long ldhp;
  const float* c_prev;  // LSTM c_{t-1} [M][Hs] (null = 0)
  bf16_t* h_out;        // h_t rows, row stride ldho
  long long ldho;
  float* c_out;         // LSTM c_t [M][Hs]
  float* act;           // LSTM saved gate activations [M][4Hs]
  float* tc;            // LSTM saved tanh(c_t) [M][Hs]
  const bf16_t* gy;     // output gradient rows of this step, row stride ldgy
  long long ldgy;
  const float* gc_next; // LSTM dc from step t+1 (null = 0)
  bf16_t* dg;           // gate-gradient rows, row stride lddg
  long long lddg;
  float* dc_prev;       // LSTM dc_{t-1} [M][Hs]
  float* s0;            // GRU: fwd r save / bwd carry (in-out)
  float* s1;            // GRU: fwd z save / bwd z (cell 4) or r (cell 5)
  float* s2;            // GRU: fwd n save / bwd n (cell 4)
  bf16_t* rh;           // GRU r∘h_{t-1} rows, row stride ldrh
  long long ldrh;
};

__device__ __forceinline__ float sgm(float x) { return 1.f / (1.f + __expf(-x)); }

__device__ __forceinline__ void ld4(const void* base, int f32, long long off, float* o) {
  if (f32) {
    const float4 v = *reinterpret_cast<const float4*>(reinterpret_cast<const float*>(base) + off);
    o[0] = v.x; o[1] = v.y; o[2] = v.z; o[3] = v.w;
  } else {
    const uint2 v = *reinterpret_cast<const uint2*>(reinterpret_cast<const bf16_t*>(base) + off);
    o[0] = __uint_as_float(v.x << 16);
    o[1] = __uint_as_float(v.x & 0xFFFF0000u);
    o[2] = __uint_as_float(v.y << 16);
    o[3] = __uint_as_float(v.y & 0xFFFF0000u);
  }
}
__device__ __forceinline__ void ldf4(const float* p, float* o) {
  if (!p) { o[0] = o[1] = o[2] = o[3] = 0.f; return; }
  const float4 v = *reinterpret_cast<const float4*>(p);
  o[0] = v.x; o[1] = v.y; o[2] = v.z; o[3] = v.w;
}
__device__ __forceinline__ void stf4(float* p, const float* v) {
  *reinterpret_cast<float4*>(p) = make_float4(v[0], v[1], v[2], v[3]);
}
__device__ __forceinline__ void stb4(bf16_t* p, const float* v) {
  *reinterpret_cast<uint2*>(p) = make_uint2((uint32_t)f2bf(v[0]) | ((uint32_t)f2bf(v[1]) << 16),
                                            (uint32_t)f2bf(v[2]) | ((uint32_t)f2bf(v[3]) << 16));
}

template <int CELL, int G>
__global__ void __launch_bounds__(256) k_rnn_step(RnnStep p) {
  __shared__ v4f red[3][G * 2][64];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int fr = lane & 15, fq = lane >> 4;
  const int j0 = blockIdx.x * 16, m0 = blockIdx.y * 32;

  v4f acc[G][2];
#pragma unroll
  for (int g = 0; g < G; ++g) acc[g][0] = acc[g][1] = v4f{0.f, 0.f, 0.f, 0.f};

  if (p.a) {
    const bool ar0 = m0 + fr < p.M, ar1 = m0 + 16 + fr < p.M, bu = j0 + fr < p.Hs;
    const bf16_t* pa0 = p.a + (long long)(ar0 ? m0 + fr : 0) * p.lda;
    const bf16_t* pa1 = p.a + (long long)(ar1 ? m0 + 16 + fr : 0) * p.lda;
    const bf16_t* pu = p.u + (long long)(bu ? j0 + fr : 0) * p.K;
    const long long gstride = (long long)p.Hs * p.K;
    const int KS = (p.K + 31) / 32;
    const v8s zero = {0, 0, 0, 0, 0, 0, 0, 0};
    for (int ks = wid; ks < KS; ks += 4) {
      const int k = ks * 32 + fq * 8;
      const bool kin = k < p.K;
      const v8s x0 = (kin && ar0) ? *reinterpret_cast<const v8s*>(pa0 + k) : zero;
      const v8s x1 = (kin && ar1) ? *reinterpret_cast<const v8s*>(pa1 + k) : zero;
#pragma unroll
      for (int g = 0; g < G; ++g) {
        const v8s w = (kin && bu) ? *reinterpret_cast<const v8s*>(pu + g * gstride + k) : zero;
        acc[g][0] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w, x0, acc[g][0], 0, 0, 0);
        acc[g][1] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w, x1, acc[g][1], 0, 0, 0);
      }
    }
    if (wid > 0) {
#pragma unroll
      for (int g = 0; g < G; ++g) {
        red[wid - 1][g * 2][lane] = acc[g][0];
        red[wid - 1][g * 2 + 1][lane] = acc[g][1];
      }
    }
    __syncthreads();
    if (wid > 0) return;
#pragma unroll
    for (int w = 0; w < 3; ++w)
#pragma unroll
      for (int g = 0; g < G; ++g) {
        acc[g][0] += red[w][g * 2][lane];
        acc[g][1] += red[w][g * 2 + 1][lane];
      }
  } else if (wid > 0) {
    return;
  }

  const int H = p.Hs;
  const int j = j0 + fq * 4;
  if (j >= H) return;  // H % 4 == 0: a unit quad is all in or all out
#pragma unroll
  for (int t = 0; t < 2; ++t) {
    const int m = m0 + t * 16 + fr;
    if (m >= p.M) continue;
    const long long mh = (long long)m * H + j;
    if constexpr (CELL == 0) {
      float gi[4], gg[4], gf[4], go[4], cp[4];
      ld4(p.xg, p.x_f32, (long long)m * p.ldx + j, gi);
      ld4(p.xg, p.x_f32, (long long)m * p.ldx + H + j, gg);
      ld4(p.xg, p.x_f32, (long long)m * p.ldx + 2 * H + j, gf);
      ld4(p.xg, p.x_f32, (long long)m * p.ldx + 3 * H + j, go);
      ldf4(p.c_prev ? p.c_prev + mh : nullptr, cp);
      float h[4], c[4], tcv[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        gi[e] = sgm(gi[e] + acc[0][t][e]);
        gg[e] = tanhf(gg[e] + acc[1][t][e]);
        gf[e] = sgm(gf[e] + acc[2][t][e]);
        go[e] = sgm(go[e] + acc[3][t][e]);
        c[e] = gi[e] * gg[e] + gf[e] * cp[e];
        tcv[e] = tanhf(c[e]);
        h[e] = go[e] * tcv[e];
      }
      stb4(p.h_out + (long long)m * p.ldho + j, h);
      if (p.c_out) stf4(p.c_out + mh, c);
      if (p.act) {
        float* a = p.act + (long long)m * 4 * H + j;
        stf4(a, gi);
        stf4(a + H, gg);
        stf4(a + 2 * H, gf);
        stf4(a + 3 * H, go);
      }
      if (p.tc) stf4(p.tc + mh, tcv);
    } else if constexpr (CELL == 1) {
      float dh[4], i4[4], g4[4], f4[4], o4[4], tcv[4], cp[4], gcn[4];
      ld4(p.gy, 0, (long long)m * p.ldgy + j, dh);
      const float* a = p.act + (long long)m * 4 * H + j;
      ldf4(a, i4);
      ldf4(a + H, g4);
      ldf4(a + 2 * H, f4);
      ldf4(a + 3 * H, o4);
      ldf4(p.tc + mh, tcv);
      ldf4(p.c_prev ? p.c_prev + mh : nullptr, cp);
      ldf4(p.gc_next ? p.gc_next + mh : nullptr, gcn);
      float di[4], dgg[4], df[4], dout[4], dcp[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float d_h = dh[e] + acc[0][t][e];
        const float dc = d_h * o4[e] * (1.f - tcv[e] * tcv[e]) + gcn[e];
        di[e] = dc * g4[e] * i4[e] * (1.f - i4[e]);
        dgg[e] = dc * i4[e] * (1.f - g4[e] * g4[e]);
        df[e] = dc * cp[e] * f4[e] * (1.f - f4[e]);
        dout[e] = d_h * tcv[e] * o4[e] * (1.f - o4[e]);
        dcp[e] = dc * f4[e];
      }
      bf16_t* o = p.dg + (long long)m * p.lddg + j;
      stb4(o, di);
      stb4(o + H, dgg);
      stb4(o + 2 * H, df);
      stb4(o + 3 * H, dout);
      stf4(p.dc_prev + mh, dcp);
    } else if constexpr (CELL == 2) {
      float xr[4], xz[4], hp[4], r[4], z[4], rh[4];
      ld4(p.xg, p.x_f32, (long long)m * p.ldx + j, xr);
      ld4(p.xg, p.x_f32, (long long)m * p.ldx + H + j, xz);
      ld4(p.hprev, 0, (long long)m * p.ldhp + j, hp);
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        r[e] = sgm(xr[e] + acc[0][t][e]);
        z[e] = sgm(xz[e] + acc[1][t][e]);
        rh[e] = r[e] * hp[e];
      }
      stb4(p.rh + (long long)m * p.ldrh + j, rh);
      stf4(p.s0 + mh, r);
      stf4(p.s1 + mh, z);
    } else if constexpr (CELL == 3) {
      float xn[4], hp[4], z[4], n[4], h[4];
      ld4(p.xg, p.x_f32, (long long)m * p.ldx + 2 * H + j, xn);
      ld4(p.hprev, 0, (long long)m * p.ldhp + j, hp);
      ldf4(p.s1 + mh, z);
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        n[e] = tanhf(xn[e] + acc[0][t][e]);
        h[e] = (1.f - z[e]) * n[e] + z[e] * hp[e];
      }
      stb4(p.h_out + (long long)m * p.ldho + j, h);
      if (p.s2) stf4(p.s2 + mh, n);
    } else if constexpr (CELL == 4) {
      float gy[4], carry[4], z[4], n[4], hp[4], daz[4], dan[4], nc[4];
      ld4(p.gy, 0, (long long)m * p.ldgy + j, gy);
      ldf4(p.s0 + mh, carry);
      ldf4(p.s1 + mh, z);
      ldf4(p.s2 + mh, n);
      ld4(p.hprev, 0, (long long)m * p.ldhp + j, hp);
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float dh = gy[e] + carry[e] + acc[0][t][e];
        dan[e] = dh * (1.f - z[e]) * (1.f - n[e] * n[e]);
        daz[e] = dh * (hp[e] - n[e]) * z[e] * (1.f - z[e]);
        nc[e] = dh * z[e];
      }
      bf16_t* o = p.dg + (long long)m * p.lddg + j;
      stb4(o + H, daz);
      stb4(o + 2 * H, dan);
      stf4(p.s0 + mh, nc);
    } else {  // CELL == 5
      float carry[4], r[4], hp[4], dar[4];
      ldf4(p.s0 + mh, carry);
      ldf4(p.s1 + mh, r);
      ld4(p.hprev, 0, (long long)m * p.ldhp + j, hp);
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float drh = acc[0][t][e];
        dar[e] = drh * hp[e] * r[e] * (1.f - r[e]);
        carry[e] += drh * r[e];
      }
      stb4(p.dg + (long long)m * p.lddg + j, dar);
      stf4(p.s0 + mh, carry);
    }
  }
}

static bool a16(const void* q) { return ((uintptr_t)q & 15) == 0; }
static bool a8(const void* q) { return ((uintptr_t)q & 7) == 0; }

// Host launcher: validates everything the kernel's vector accesses assume (H % 8, K % 8, 16-B
// aligned operand rows, 8-B aligned bf16 / 16-B aligned fp32 quads) before any launch.
BIGDL_EXPORT int bigdl_rnn_step(int cell, const void* a, long long lda, const void* u, int M, int K, int Hs,
                                const void* xg, long long ldx, int x_f32, const void* hprev, long long ldhp,
                                const float* c_prev, void* h_out, long long ldho, float* c_out, float* act, float* tc,
                                const void* gy, long long ldgy, const float* gc_next, void* dg, long long lddg,
                                float* dc_prev, float* s0, float* s1, float* s2, void* rh, long long ldrh,
                                hipStream_t s) {
  if (M <= 0 || K <= 0 || Hs <= 0 || Hs % 8 || K % 8 || cell < 0 || cell > 5) return (int)hipErrorInvalidValue;
  if (a && (lda < K || lda % 8 || !a16(a))) return (int)hipErrorInvalidValue;
  if (!u || !a16(u)) return (int)hipErrorInvalidValue;
  static const int G[6] = {4, 1, 2, 1, 1, 1};
  static const int KWANT[6] = {1, 4, 1, 1, 2, 1};  // K in units of Hs
  if (K != KWANT[cell] * Hs) return (int)hipErrorInvalidValue;
  const void* f32s[] = {c_prev, c_out, act, tc, gc_next, dc_prev, s0, s1, s2};
  for (const void* q : f32s)
    if (q && !a16(q)) return (int)hipErrorInvalidValue;
  if (xg && (ldx % 4 || (x_f32 ? !a16(xg) : !a8(xg)))) return (int)hipErrorInvalidValue;
  const void* b8s[] = {hprev, h_out, gy, dg, rh};
  const long long lds_[] = {ldhp, ldho, ldgy, lddg, ldrh};
  for (int i = 0; i < 5; ++i)
    if (b8s[i] && (!a8(b8s[i]) || lds_[i] % 4)) return (int)hipErrorInvalidValue;
  // per-cell required tensors
  bool ok = true;
  switch (cell) {
    case 0: ok = xg && h_out; break;
    case 1: ok = gy && act && tc && dg && dc_prev; break;
    case 2: ok = xg && hprev && rh && s0 && s1; break;
    case 3: ok = xg && hprev && s1 && h_out; break;
    case 4: ok = gy && s0 && s1 && s2 && hprev && dg; break;
    case 5: ok = a && s0 && s1 && hprev && dg; break;
  }
  if (!ok) return (int)hipErrorInvalidValue;
  RnnStep p;
  p.a = (const bf16_t*)a; p.lda = lda; p.u = (const bf16_t*)u; p.M = M; p.K = K; p.Hs = Hs;
  p.xg = xg; p.ldx = ldx; p.x_f32 = x_f32; p.hprev = (const bf16_t*)hprev; p.ldhp = ldhp; p.c_prev = c_prev;
  p.h_out = (bf16_t*)h_out; p.ldho = ldho; p.c_out = c_out; p.act = act; p.tc = tc; p.gy = (const bf16_t*)gy;
  p.ldgy = ldgy; p.gc_next = gc_next; p.dg = (bf16_t*)dg; p.lddg = lddg; p.dc_prev = dc_prev; p.s0 = s0; p.s1 = s1;
  p.s2 = s2; p.rh = (bf16_t*)rh; p.ldrh = ldrh;
  dim3 grid((unsigned)((Hs + 15) / 16), (unsigned)((M + 31) / 32)), block(256);
  (void)G;
  switch (cell) {
    case 0: hipLaunchKernelGGL((k_rnn_step<0, 4>), grid, block, 0, s, p); break;
    case 1: hipLaunchKernelGGL((k_rnn_step<1, 1>), grid, block, 0, s, p); break;
    case 2: hipLaunchKernelGGL((k_rnn_step<2, 2>), grid, block, 0, s, p); break;
    case 3: hipLaunchKernelGGL((k_rnn_step<3, 1>), grid, block, 0, s, p); break;
    case 4: hipLaunchKernelGGL((k_rnn_step<4, 1>), grid, block, 0, s, p); break;
    default: hipLaunchKernelGGL((k_rnn_step<5, 1>), grid, block, 0, s, p); break;
  }
  BIGDL_CHECK_LAUNCH();
}
