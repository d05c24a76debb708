// Fused recurrent time step: the h·Uᵀ recurrent GEMM on MFMA and the cell's pointwise math in ONE
// launch per step (K14 persistent-style LSTM step, K15 GRU).  Reference graphs: DL/nn/LSTM.scala:
// 124-187 (gates i, g, f, o), DL/nn/GRU.scala (r, z, ĥ = tanh(x_h + U_h(r∘h)), h' = (1−z)ĥ + z h),
// time loop / BPTT DL/nn/Recurrent.scala:283-400.
//
// Gate-grouped tiling: a block owns 16 hidden units j0..j0+15 and 32 batch rows, and computes the
// G gate groups of those units (LSTM: 4 tiles = rows g·H + j of U).  mfma_f32_16x16x32_bf16 with
// the weight row as the MFMA "A" side leaves, in each lane, the SAME (batch row, 4 consecutive
// units) for every gate tile — so the cell update runs in registers right after the MFMAs, with no
// LDS exchange between gates.  The reduction dim is split over the block's 8 waves (the per-step
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
  // optional second reduction segment (stacked layers, k_rnn_step_pair): acc += a2 · u2ᵀ over K2 more
  // indices — layer l+1's input product h_l·W folded into its recurrent step (forward), layer l's
  // dh contribution dg_{l+1}·W folded into its step (backward).  a2 null = zero rows; K2 = 0 = none.
  const bf16_t* a2;
  long long lda2;
  const bf16_t* u2;     // [G·Hs][K2]
  int K2;
  // fp32 recurrence (k_rnn_step<…, F32 = true>): every pointer typed bf16_t above (a, a2, u, u2,
  // hprev, h_out, gy, dg, rh) holds fp32 instead, and the products run as bf16x3 on the matrix
  // cores (hi·hi + lo·hi + hi·lo, hi = rne(v), lo = rne(v − hi)) — fp32-accurate recurrent GEMMs
  int f32;
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
// a quad of the activation element type (bf16, or fp32 when F32) at element offset `off`
template <bool F32>
__device__ __forceinline__ void st4(bf16_t* base, long long off, const float* v) {
  if constexpr (F32) stf4(reinterpret_cast<float*>(base) + off, v);
  else stb4(base + off, v);
}

// number of fp32 quads of per-(row, unit) epilogue operands each cell reads
template <int CELL> struct NPre;
template <> struct NPre<0> { static constexpr int v = 5; };  // xg i,g,f,o, c_prev
template <> struct NPre<1> { static constexpr int v = 8; };  // gy, act i,g,f,o, tanh(c), c_prev, dc_next
template <> struct NPre<2> { static constexpr int v = 3; };  // x_r, x_z, h_prev
template <> struct NPre<3> { static constexpr int v = 3; };  // x_h, h_prev, z
template <> struct NPre<4> { static constexpr int v = 5; };  // gy, carry, z, n, h_prev
template <> struct NPre<5> { static constexpr int v = 3; };  // carry, r, h_prev

// The epilogue's operands are fetched by wave 0 BEFORE the reduction loop so their memory latency
// overlaps the MFMA chain instead of following it (the step kernels are latency-bound).
template <int CELL, bool F32>
__device__ __forceinline__ void pre_load(const RnnStep& p, int m, int j, float (&v)[NPre<CELL>::v][4]) {
  const int H = p.Hs;
  const long long mh = (long long)m * H + j;
  if constexpr (CELL == 0) {
#pragma unroll
    for (int g = 0; g < 4; ++g) ld4(p.xg, p.x_f32, (long long)m * p.ldx + g * H + j, v[g]);
    ldf4(p.c_prev ? p.c_prev + mh : nullptr, v[4]);
  } else if constexpr (CELL == 1) {
    if (p.gy) ld4(p.gy, F32, (long long)m * p.ldgy + j, v[0]);
    else v[0][0] = v[0][1] = v[0][2] = v[0][3] = 0.f;
    const float* a = p.act + (long long)m * 4 * H + j;
#pragma unroll
    for (int g = 0; g < 4; ++g) ldf4(a + g * H, v[1 + g]);
    ldf4(p.tc + mh, v[5]);
    ldf4(p.c_prev ? p.c_prev + mh : nullptr, v[6]);
    ldf4(p.gc_next ? p.gc_next + mh : nullptr, v[7]);
  } else if constexpr (CELL == 2) {
    ld4(p.xg, p.x_f32, (long long)m * p.ldx + j, v[0]);
    ld4(p.xg, p.x_f32, (long long)m * p.ldx + H + j, v[1]);
    ld4(p.hprev, F32, (long long)m * p.ldhp + j, v[2]);
  } else if constexpr (CELL == 3) {
    ld4(p.xg, p.x_f32, (long long)m * p.ldx + 2 * H + j, v[0]);
    ld4(p.hprev, F32, (long long)m * p.ldhp + j, v[1]);
    ldf4(p.s1 + mh, v[2]);
  } else if constexpr (CELL == 4) {
    ld4(p.gy, F32, (long long)m * p.ldgy + j, v[0]);
    ldf4(p.s0 + mh, v[1]);
    ldf4(p.s1 + mh, v[2]);
    ldf4(p.s2 + mh, v[3]);
    ld4(p.hprev, F32, (long long)m * p.ldhp + j, v[4]);
  } else {
    ldf4(p.s0 + mh, v[0]);
    ldf4(p.s1 + mh, v[1]);
    ld4(p.hprev, F32, (long long)m * p.ldhp + j, v[2]);
  }
}

template <int CELL, int G, bool F32>
__device__ __forceinline__ void epilogue(const RnnStep& p, int m, int j, const float (&v)[NPre<CELL>::v][4],
                                         const v4f (&acc)[G]) {
  const int H = p.Hs;
  const long long mh = (long long)m * H + j;
  if constexpr (CELL == 0) {
    float gi[4], gg[4], gf[4], go[4], h[4], c[4], tcv[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      gi[e] = sgm(v[0][e] + acc[0][e]);
      gg[e] = tanhf(v[1][e] + acc[1][e]);
      gf[e] = sgm(v[2][e] + acc[2][e]);
      go[e] = sgm(v[3][e] + acc[3][e]);
      c[e] = gi[e] * gg[e] + gf[e] * v[4][e];
      tcv[e] = tanhf(c[e]);
      h[e] = go[e] * tcv[e];
    }
    st4<F32>(p.h_out, (long long)m * p.ldho + j, h);
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
    float di[4], dgg[4], df[4], dout[4], dcp[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const float i = v[1][e], g = v[2][e], f = v[3][e], o = v[4][e], tcv = v[5][e];
      const float d_h = v[0][e] + acc[0][e];
      const float dc = d_h * o * (1.f - tcv * tcv) + v[7][e];
      di[e] = dc * g * i * (1.f - i);
      dgg[e] = dc * i * (1.f - g * g);
      df[e] = dc * v[6][e] * f * (1.f - f);
      dout[e] = d_h * tcv * o * (1.f - o);
      dcp[e] = dc * f;
    }
    const long long o = (long long)m * p.lddg + j;
    st4<F32>(p.dg, o, di);
    st4<F32>(p.dg, o + H, dgg);
    st4<F32>(p.dg, o + 2 * H, df);
    st4<F32>(p.dg, o + 3 * H, dout);
    stf4(p.dc_prev + mh, dcp);
  } else if constexpr (CELL == 2) {
    float r[4], z[4], rh[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      r[e] = sgm(v[0][e] + acc[0][e]);
      z[e] = sgm(v[1][e] + acc[1][e]);
      rh[e] = r[e] * v[2][e];
    }
    st4<F32>(p.rh, (long long)m * p.ldrh + j, rh);
    stf4(p.s0 + mh, r);
    stf4(p.s1 + mh, z);
  } else if constexpr (CELL == 3) {
    float n[4], h[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      n[e] = tanhf(v[0][e] + acc[0][e]);
      h[e] = (1.f - v[2][e]) * n[e] + v[2][e] * v[1][e];
    }
    st4<F32>(p.h_out, (long long)m * p.ldho + j, h);
    if (p.s2) stf4(p.s2 + mh, n);
  } else if constexpr (CELL == 4) {
    float daz[4], dan[4], nc[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const float z = v[2][e], n = v[3][e];
      const float dh = v[0][e] + v[1][e] + acc[0][e];
      dan[e] = dh * (1.f - z) * (1.f - n * n);
      daz[e] = dh * (v[4][e] - n) * z * (1.f - z);
      nc[e] = dh * z;
    }
    const long long o = (long long)m * p.lddg + j;
    st4<F32>(p.dg, o + H, daz);
    st4<F32>(p.dg, o + 2 * H, dan);
    stf4(p.s0 + mh, nc);
  } else {
    float dar[4], carry[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const float drh = acc[0][e], r = v[1][e];
      dar[e] = drh * v[2][e] * r * (1.f - r);
      carry[e] = v[0][e] + drh * r;
    }
    st4<F32>(p.dg, (long long)m * p.lddg + j, dar);
    stf4(p.s0 + mh, carry);
  }
}

// 8 waves per block split the reduction dim 8 ways: every wave has at most ⌈K/256⌉ fragment loads
// in flight for the whole step (one L2 round trip instead of up to 7 dependent ones at K = 4H = 800)
constexpr int kStepWaves = 8;

// 8 consecutive fp32 values → (rne bf16 hi, rne bf16 of the residual) as two MFMA fragments
__device__ __forceinline__ void split_x3(const float* q, bool live, v8s& hi, v8s& lo) {
  float v[8];
  if (live) {
    const float4 a = *reinterpret_cast<const float4*>(q), b = *reinterpret_cast<const float4*>(q + 4);
    v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w; v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
  } else {
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] = 0.f;
  }
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    const bf16_t h = f2bf(v[e]);
    hi[e] = (short)h;
    lo[e] = (short)f2bf(v[e] - bf2f(h));
  }
}

template <int CELL, int G, bool F32 = false>
__device__ __forceinline__ void rnn_step_body(const RnnStep& p) {
  constexpr int NW = kStepWaves;
  __shared__ v4f red[NW - 1][G * 2][64];
  constexpr int NP = NPre<CELL>::v;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int fr = lane & 15, fq = lane >> 4;
  const int j0 = blockIdx.x * 16, m0 = blockIdx.y * 32;
  const int j = j0 + fq * 4;
  const bool jin = j < p.Hs;  // Hs % 4 == 0: a unit quad is all in or all out
  const bool min0 = m0 + fr < p.M, min1 = m0 + 16 + fr < p.M;

  float pre0[NP][4], pre1[NP][4];
  if (wid == 0 && jin) {
    if (min0) pre_load<CELL, F32>(p, m0 + fr, j, pre0);
    if (min1) pre_load<CELL, F32>(p, m0 + 16 + fr, j, pre1);
  }

  v4f acc0[G], acc1[G];
#pragma unroll
  for (int g = 0; g < G; ++g) acc0[g] = acc1[g] = v4f{0.f, 0.f, 0.f, 0.f};

  if constexpr (F32) {
    if (p.a || p.a2) {
      const bool bu = j0 + fr < p.Hs;
      const long long r0 = min0 ? m0 + fr : 0, r1 = min1 ? m0 + 16 + fr : 0;
      const float* A = reinterpret_cast<const float*>(p.a);
      const float* A2 = reinterpret_cast<const float*>(p.a2);
      const float* pa0 = A ? A + r0 * p.lda : nullptr;
      const float* pa1 = A ? A + r1 * p.lda : nullptr;
      const float* pb0 = A2 ? A2 + r0 * p.lda2 : nullptr;
      const float* pb1 = A2 ? A2 + r1 * p.lda2 : nullptr;
      const float* pu = reinterpret_cast<const float*>(p.u) + (long long)(bu ? j0 + fr : 0) * p.K;
      const float* pu2 = p.K2 ? reinterpret_cast<const float*>(p.u2) + (long long)(bu ? j0 + fr : 0) * p.K2 : nullptr;
      const long long gstride = (long long)p.Hs * p.K, gstride2 = (long long)p.Hs * p.K2;
      const int KT = p.K + p.K2;
      const int KS = (KT + 31) / 32;
      for (int ks = wid; ks < KS; ks += NW) {
        const int k = ks * 32 + fq * 8;
        const bool kin = k < KT, seg2 = k >= p.K;
        const int kk = seg2 ? k - p.K : k;
        const float* s0 = seg2 ? pb0 : pa0;
        const float* s1 = seg2 ? pb1 : pa1;
        v8s xh0, xl0, xh1, xl1;
        split_x3(s0 ? s0 + kk : nullptr, kin && min0 && s0, xh0, xl0);
        split_x3(s1 ? s1 + kk : nullptr, kin && min1 && s1, xh1, xl1);
        const float* wu = seg2 ? pu2 : pu;
        const long long gs = seg2 ? gstride2 : gstride;
#pragma unroll
        for (int g = 0; g < G; ++g) {
          v8s wh, wl;
          split_x3(wu ? wu + g * gs + kk : nullptr, kin && bu && wu, wh, wl);
          acc0[g] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wh, xh0, acc0[g], 0, 0, 0);
          acc1[g] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wh, xh1, acc1[g], 0, 0, 0);
          acc0[g] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wl, xh0, acc0[g], 0, 0, 0);
          acc1[g] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wl, xh1, acc1[g], 0, 0, 0);
          acc0[g] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wh, xl0, acc0[g], 0, 0, 0);
          acc1[g] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wh, xl1, acc1[g], 0, 0, 0);
        }
      }
      if (wid > 0) {
#pragma unroll
        for (int g = 0; g < G; ++g) {
          red[wid - 1][g * 2][lane] = acc0[g];
          red[wid - 1][g * 2 + 1][lane] = acc1[g];
        }
      }
      __syncthreads();
      if (wid > 0) return;
#pragma unroll
      for (int w = 0; w < NW - 1; ++w)
#pragma unroll
        for (int g = 0; g < G; ++g) {
          acc0[g] += red[w][g * 2][lane];
          acc1[g] += red[w][g * 2 + 1][lane];
        }
    } else if (wid > 0) {
      return;
    }
  } else if (p.a || p.a2) {
    const bool bu = j0 + fr < p.Hs;
    const long long r0 = min0 ? m0 + fr : 0, r1 = min1 ? m0 + 16 + fr : 0;
    const bf16_t* pa0 = p.a ? p.a + r0 * p.lda : nullptr;
    const bf16_t* pa1 = p.a ? p.a + r1 * p.lda : nullptr;
    const bf16_t* pb0 = p.a2 ? p.a2 + r0 * p.lda2 : nullptr;
    const bf16_t* pb1 = p.a2 ? p.a2 + r1 * p.lda2 : nullptr;
    const bf16_t* pu = p.u + (long long)(bu ? j0 + fr : 0) * p.K;
    const bf16_t* pu2 = p.K2 ? p.u2 + (long long)(bu ? j0 + fr : 0) * p.K2 : nullptr;
    const long long gstride = (long long)p.Hs * p.K, gstride2 = (long long)p.Hs * p.K2;
    const int KT = p.K + p.K2;  // K % 8 == 0: a lane's 8-index chunk never straddles the segments
    const int KS = (KT + 31) / 32;
    const v8s zero = {0, 0, 0, 0, 0, 0, 0, 0};
#pragma unroll 4
    for (int ks = wid; ks < KS; ks += NW) {
      const int k = ks * 32 + fq * 8;
      const bool kin = k < KT, seg2 = k >= p.K;
      const int kk = seg2 ? k - p.K : k;
      const bf16_t* s0 = seg2 ? pb0 : pa0;
      const bf16_t* s1 = seg2 ? pb1 : pa1;
      const v8s x0 = (kin && min0 && s0) ? *reinterpret_cast<const v8s*>(s0 + kk) : zero;
      const v8s x1 = (kin && min1 && s1) ? *reinterpret_cast<const v8s*>(s1 + kk) : zero;
      const bf16_t* wu = seg2 ? pu2 : pu;
      const long long gs = seg2 ? gstride2 : gstride;
      v8s w[G];
#pragma unroll
      for (int g = 0; g < G; ++g) w[g] = (kin && bu) ? *reinterpret_cast<const v8s*>(wu + g * gs + kk) : zero;
#pragma unroll
      for (int g = 0; g < G; ++g) {
        acc0[g] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w[g], x0, acc0[g], 0, 0, 0);
        acc1[g] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w[g], x1, acc1[g], 0, 0, 0);
      }
    }
    if (wid > 0) {
#pragma unroll
      for (int g = 0; g < G; ++g) {
        red[wid - 1][g * 2][lane] = acc0[g];
        red[wid - 1][g * 2 + 1][lane] = acc1[g];
      }
    }
    __syncthreads();
    if (wid > 0) return;
#pragma unroll
    for (int w = 0; w < NW - 1; ++w)
#pragma unroll
      for (int g = 0; g < G; ++g) {
        acc0[g] += red[w][g * 2][lane];
        acc1[g] += red[w][g * 2 + 1][lane];
      }
  } else if (wid > 0) {
    return;
  }
  if (!jin) return;
  if (min0) epilogue<CELL, G, F32>(p, m0 + fr, j, pre0, acc0);
  if (min1) epilogue<CELL, G, F32>(p, m0 + 16 + fr, j, pre1, acc1);
}

template <int CELL, int G, bool F32 = false>
__global__ void __launch_bounds__(64 * kStepWaves) k_rnn_step(RnnStep p) {
  rnn_step_body<CELL, G, F32>(p);
}

// Two stacked layers in ONE launch (blockIdx.z = layer; bit z of `live` = that layer has a step in
// this wave): the layer wavefront — layer 1 runs step t−1 while layer 0 runs step t (forward), layer 0
// runs step t+1 while layer 1 runs step t (backward, reversed), so a 2-layer sequence takes T + 1
// dependent launches instead of 2T.
template <int CELL, int G>
__global__ void __launch_bounds__(64 * kStepWaves) k_rnn_step_pair(RnnStep p0, RnnStep p1, int live) {
  const int z = blockIdx.z;
  if (!((live >> z) & 1)) return;
  const RnnStep& p = z ? p1 : p0;
  if ((int)blockIdx.x * 16 >= p.Hs || (int)blockIdx.y * 32 >= p.M) return;
  rnn_step_body<CELL, G>(p);
}

static bool a16(const void* q) { return ((uintptr_t)q & 15) == 0; }
static bool a8(const void* q) { return ((uintptr_t)q & 7) == 0; }

// Host-side validation of everything the kernel's vector accesses assume (H % 8, K % 8, 16-B aligned
// operand rows, 8-B aligned bf16 / 16-B aligned fp32 quads), before any launch.
static int rnn_step_check(int cell, const RnnStep& p) {
  const int M = p.M, K = p.K, Hs = p.Hs;
  if (M <= 0 || K <= 0 || Hs <= 0 || Hs % 8 || K % 8 || cell < 0 || cell > 5) return (int)hipErrorInvalidValue;
  if (p.a && (p.lda < K || p.lda % 8 || !a16(p.a))) return (int)hipErrorInvalidValue;
  if (!p.u || !a16(p.u)) return (int)hipErrorInvalidValue;
  static const int KWANT[6] = {1, 4, 1, 1, 2, 1};  // K in units of Hs
  if (K != KWANT[cell] * Hs) return (int)hipErrorInvalidValue;
  if (p.K2 < 0 || p.K2 % 8 || (p.K2 && (!p.u2 || !a16(p.u2))) || (!p.K2 && p.a2)) return (int)hipErrorInvalidValue;
  if (p.a2 && (p.lda2 < p.K2 || p.lda2 % 8 || !a16(p.a2))) return (int)hipErrorInvalidValue;
  const void* f32s[] = {p.c_prev, p.c_out, p.act, p.tc, p.gc_next, p.dc_prev, p.s0, p.s1, p.s2};
  for (const void* q : f32s)
    if (q && !a16(q)) return (int)hipErrorInvalidValue;
  if (p.xg && (p.ldx % 4 || (p.x_f32 ? !a16(p.xg) : !a8(p.xg)))) return (int)hipErrorInvalidValue;
  const void* b8s[] = {p.hprev, p.h_out, p.gy, p.dg, p.rh};
  const long long lds_[] = {p.ldhp, p.ldho, p.ldgy, p.lddg, p.ldrh};
  for (int i = 0; i < 5; ++i)
    if (b8s[i] && (!(p.f32 ? a16(b8s[i]) : a8(b8s[i])) || lds_[i] % 4)) return (int)hipErrorInvalidValue;
  // per-cell required tensors (cell 1: gy may be null when the second segment carries it)
  bool ok = true;
  switch (cell) {
    case 0: ok = p.xg && p.h_out; break;
    case 1: ok = (p.gy || p.K2) && p.act && p.tc && p.dg && p.dc_prev; break;
    case 2: ok = p.xg && p.hprev && p.rh && p.s0 && p.s1; break;
    case 3: ok = p.xg && p.hprev && p.s1 && p.h_out; break;
    case 4: ok = p.gy && p.s0 && p.s1 && p.s2 && p.hprev && p.dg; break;
    case 5: ok = p.a && p.s0 && p.s1 && p.hprev && p.dg; break;
  }
  return ok ? 0 : (int)hipErrorInvalidValue;
}

static dim3 rnn_step_grid(int Hs, int M, int z = 1) {
  return dim3((unsigned)((Hs + 15) / 16), (unsigned)((M + 31) / 32), (unsigned)z);
}

static int rnn_step_run(int cell, const void* a, long long lda, const void* u, int M, int K, int Hs, const void* xg,
                        long long ldx, int x_f32, const void* hprev, long long ldhp, const float* c_prev, void* h_out,
                        long long ldho, float* c_out, float* act, float* tc, const void* gy, long long ldgy,
                        const float* gc_next, void* dg, long long lddg, float* dc_prev, float* s0, float* s1, float* s2,
                        void* rh, long long ldrh, int f32, hipStream_t s) {
  RnnStep p{};  // value-initialised: the second segment stays off
  p.f32 = f32;
  p.a = (const bf16_t*)a; p.lda = lda; p.u = (const bf16_t*)u; p.M = M; p.K = K; p.Hs = Hs;
  p.xg = xg; p.ldx = ldx; p.x_f32 = x_f32; p.hprev = (const bf16_t*)hprev; p.ldhp = ldhp; p.c_prev = c_prev;
  p.h_out = (bf16_t*)h_out; p.ldho = ldho; p.c_out = c_out; p.act = act; p.tc = tc; p.gy = (const bf16_t*)gy;
  p.ldgy = ldgy; p.gc_next = gc_next; p.dg = (bf16_t*)dg; p.lddg = lddg; p.dc_prev = dc_prev; p.s0 = s0; p.s1 = s1;
  p.s2 = s2; p.rh = (bf16_t*)rh; p.ldrh = ldrh;
  const int rc = rnn_step_check(cell, p);
  if (rc) return rc;
  const dim3 grid = rnn_step_grid(Hs, M), block(64 * kStepWaves);
  if (f32) {
    switch (cell) {
      case 0: hipLaunchKernelGGL((k_rnn_step<0, 4, true>), grid, block, 0, s, p); break;
      case 1: hipLaunchKernelGGL((k_rnn_step<1, 1, true>), grid, block, 0, s, p); break;
      case 2: hipLaunchKernelGGL((k_rnn_step<2, 2, true>), grid, block, 0, s, p); break;
      case 3: hipLaunchKernelGGL((k_rnn_step<3, 1, true>), grid, block, 0, s, p); break;
      case 4: hipLaunchKernelGGL((k_rnn_step<4, 1, true>), grid, block, 0, s, p); break;
      default: hipLaunchKernelGGL((k_rnn_step<5, 1, true>), grid, block, 0, s, p); break;
    }
  } else {
    switch (cell) {
      case 0: hipLaunchKernelGGL((k_rnn_step<0, 4>), grid, block, 0, s, p); break;
      case 1: hipLaunchKernelGGL((k_rnn_step<1, 1>), grid, block, 0, s, p); break;
      case 2: hipLaunchKernelGGL((k_rnn_step<2, 2>), grid, block, 0, s, p); break;
      case 3: hipLaunchKernelGGL((k_rnn_step<3, 1>), grid, block, 0, s, p); break;
      case 4: hipLaunchKernelGGL((k_rnn_step<4, 1>), grid, block, 0, s, p); break;
      default: hipLaunchKernelGGL((k_rnn_step<5, 1>), grid, block, 0, s, p); break;
    }
  }
  BIGDL_CHECK_LAUNCH();
}

BIGDL_EXPORT int bigdl_rnn_step(int cell, const void* a, long long lda, const void* u, int M, int K, int Hs,
                                const void* xg, long long ldx, int x_f32, const void* hprev, long long ldhp,
                                const float* c_prev, void* h_out, long long ldho, float* c_out, float* act, float* tc,
                                const void* gy, long long ldgy, const float* gc_next, void* dg, long long lddg,
                                float* dc_prev, float* s0, float* s1, float* s2, void* rh, long long ldrh,
                                hipStream_t s) {
  return rnn_step_run(cell, a, lda, u, M, K, Hs, xg, ldx, x_f32, hprev, ldhp, c_prev, h_out, ldho, c_out, act, tc, gy,
                      ldgy, gc_next, dg, lddg, dc_prev, s0, s1, s2, rh, ldrh, 0, s);
}

// ------------------------------------------------------------------------------------------------
// Persistent whole-sequence LSTM (small batch, H ≤ 256): ONE workgroup of 16 waves runs every time
// step of a layer-direction, so a PTB-shape layer (B 20, H 200, T 20) is one launch instead of T.
// The recurrent state never leaves the CU between steps: h_{t-1} (forward) / dg_{t+1} (backward)
// sits in an LDS double buffer (the step writes the other buffer; one barrier per step), c / dc
// live in the registers of the lane that owns the (row, unit quad), and only the U fragments are
// re-read from L2 each step (U is L2-resident: 4H·H bf16).  Wave w owns unit tile w (16 units ×
// 4 gates as MFMA rows, the batch rows as MFMA columns — the tiling of k_rnn_step, whose epilogue
// math this reuses) and all ⌈B/16⌉ batch tiles, so a U fragment feeds NBT MFMAs.  No inter-
// workgroup communication: nothing to spin on, nothing placement-dependent.
// ------------------------------------------------------------------------------------------------
struct LstmSeqP {
  const void* x2;  // [B][T][4H] input projection (bf16, or fp32 when x_f32)
  int x_f32;
  const bf16_t* h0;  // [B][H]
  const float* c0;   // [B][H] or null
  const bf16_t* u;   // forward: U [4H][H]; backward: Uᵀ [H][4H]
  bf16_t* out;       // [B][T][H]
  float* cs;         // [T][B][H] (training saves; null = inference)
  float* acts;       // [T][B][4H]
  float* tcs;        // [T][B][H]
  float* cbuf;       // inference: c ping-pong [2][B][H]
  const bf16_t* gy;  // backward: [B][T][H]
  bf16_t* dg;        // backward: [B][T][4H]
  float* gc;         // backward: dc of step 0 → [B][H]
  int B, T, H;
  unsigned long long* xg;  // multi-workgroup granule protocol: [2][B][K/2] {tag, 2 bf16} exchange slots
  // multi-workgroup kernels: the grid holds `spread` × tiles workgroups and only every spread-th one
  // works (tile = blockIdx.x / spread).  Workgroups are dealt to the 8 XCDs round-robin, so with
  // spread 8 all working tiles share one XCD's L2 and the step-to-step hand-off stays inside it
  // (placement is a speed matter only: the exchange protocol is agent-scope either way).
  int spread;
};

constexpr int kPersistMaxH = 256;

template <int NBT>
__global__ void __launch_bounds__(1024) k_lstm_seq_fwd_p(LstmSeqP p) {
  constexpr int LDH = kPersistMaxH + 8;  // padded LDS row (elements)
  __shared__ __attribute__((aligned(16))) bf16_t hs[2][NBT * 16 * LDH];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, fr = lane & 15, fq = lane >> 4;
  const int H = p.H, B = p.B, T = p.T, G = 4 * H;
  const int j = w * 16 + fq * 4;                 // this lane's unit quad
  const bool jin = j < H;
  const bool urow = w * 16 + fr < H;             // this lane's U row (A operand) exists
  const int KC = (H + 31) / 32;
  for (int i = tid; i < 2 * NBT * 16 * LDH; i += 1024) (&hs[0][0])[i] = 0;
  __syncthreads();
  for (int i = tid; i < B * H; i += 1024) hs[0][(i / H) * LDH + i % H] = p.h0[i];
  float c[NBT][4];
#pragma unroll
  for (int bt = 0; bt < NBT; ++bt) {
    const int m = bt * 16 + fr;
#pragma unroll
    for (int e = 0; e < 4; ++e) c[bt][e] = (p.c0 && m < B && jin) ? p.c0[(long long)m * H + j + e] : 0.f;
  }
  __syncthreads();
  const bf16_t* ub = p.u + (long long)(urow ? w * 16 + fr : 0) * H;
  const long long gstride = (long long)H * H;
  const v8s zero = {0, 0, 0, 0, 0, 0, 0, 0};
  for (int t = 0; t < T; ++t) {
    const bf16_t* hc = hs[t & 1];
    bf16_t* hn = hs[(t + 1) & 1];
    if (w * 16 < H) {
      // epilogue operands first (bf16 x2: raw 8-B quads, 2 VGPRs each), so their latency hides under
      // the MFMA chain; an fp32 x2 is read in the epilogue
      uint2 xr[NBT][4];
#pragma unroll
      for (int bt = 0; bt < NBT; ++bt) {
        const int m = bt * 16 + fr;
#pragma unroll
        for (int g = 0; g < 4; ++g)
          xr[bt][g] = (!p.x_f32 && m < B && jin)
                          ? *reinterpret_cast<const uint2*>((const bf16_t*)p.x2 + ((long long)m * T + t) * G + g * H + j)
                          : make_uint2(0u, 0u);
      }
      v4f acc[NBT][4];
#pragma unroll
      for (int bt = 0; bt < NBT; ++bt)
#pragma unroll
        for (int g = 0; g < 4; ++g) acc[bt][g] = v4f{0.f, 0.f, 0.f, 0.f};
#pragma unroll 2
      for (int kc = 0; kc < KC; ++kc) {
        const int k = kc * 32 + fq * 8;
        const bool kin = k < H;
        v8s wf[4];
#pragma unroll
        for (int g = 0; g < 4; ++g) wf[g] = (kin && urow) ? *reinterpret_cast<const v8s*>(ub + g * gstride + k) : zero;
#pragma unroll
        for (int bt = 0; bt < NBT; ++bt) {
          const v8s hf = kin ? *reinterpret_cast<const v8s*>(&hc[(bt * 16 + fr) * LDH + k]) : zero;
#pragma unroll
          for (int g = 0; g < 4; ++g) acc[bt][g] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[g], hf, acc[bt][g], 0, 0, 0);
        }
      }
#pragma unroll
      for (int bt = 0; bt < NBT; ++bt) {
        const int m = bt * 16 + fr;
        if (m >= B || !jin) continue;
        float xg[4][4];
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          if (p.x_f32) {
            ld4(p.x2, 1, ((long long)m * T + t) * G + g * H + j, xg[g]);
          } else {
            xg[g][0] = __uint_as_float(xr[bt][g].x << 16);
            xg[g][1] = __uint_as_float(xr[bt][g].x & 0xFFFF0000u);
            xg[g][2] = __uint_as_float(xr[bt][g].y << 16);
            xg[g][3] = __uint_as_float(xr[bt][g].y & 0xFFFF0000u);
          }
        }
        float gi[4], gg[4], gf[4], go[4], h[4], tcv[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          gi[e] = sgm(xg[0][e] + acc[bt][0][e]);
          gg[e] = tanhf(xg[1][e] + acc[bt][1][e]);
          gf[e] = sgm(xg[2][e] + acc[bt][2][e]);
          go[e] = sgm(xg[3][e] + acc[bt][3][e]);
          c[bt][e] = gi[e] * gg[e] + gf[e] * c[bt][e];
          tcv[e] = tanhf(c[bt][e]);
          h[e] = go[e] * tcv[e];
        }
        stb4(p.out + ((long long)m * T + t) * H + j, h);
        stb4(&hn[m * LDH + j], h);
        const long long mh = ((long long)t * B + m) * H + j;
        if (p.cs) {
          stf4(p.cs + mh, c[bt]);
          stf4(p.tcs + mh, tcv);
          float* a = p.acts + ((long long)t * B + m) * G + j;
          stf4(a, gi);
          stf4(a + H, gg);
          stf4(a + 2 * H, gf);
          stf4(a + 3 * H, go);
        } else if (p.cbuf) {
          stf4(p.cbuf + (long long)(t & 1) * B * H + (long long)m * H + j, c[bt]);
        }
      }
    }
    __syncthreads();  // h_t complete in LDS; every read of h_{t-1} retired
  }
}

template <int NBT>
__global__ void __launch_bounds__(1024) k_lstm_seq_bwd_p(LstmSeqP p) {
  constexpr int LDG = 4 * kPersistMaxH + 8;
  __shared__ __attribute__((aligned(16))) bf16_t gs[2][NBT * 16 * LDG];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, fr = lane & 15, fq = lane >> 4;
  const int H = p.H, B = p.B, T = p.T, G = 4 * H;
  const int j = w * 16 + fq * 4;
  const bool jin = j < H;
  const bool urow = w * 16 + fr < H;
  const int KC = (G + 31) / 32;
  for (int i = tid; i < 2 * NBT * 16 * LDG; i += 1024) (&gs[0][0])[i] = 0;
  __syncthreads();
  float dc[NBT][4];
#pragma unroll
  for (int bt = 0; bt < NBT; ++bt)
#pragma unroll
    for (int e = 0; e < 4; ++e) dc[bt][e] = 0.f;
  const bf16_t* ub = p.u + (long long)(urow ? w * 16 + fr : 0) * G;  // Uᵀ row j: Σ_k dg[k]·U[k][j]
  const v8s zero = {0, 0, 0, 0, 0, 0, 0, 0};
  for (int t = T - 1; t >= 0; --t) {
    const bf16_t* gc_ = gs[t & 1];  // dg_{t+1} (zero at the last step)
    bf16_t* gn = gs[(t + 1) & 1];
    if (w * 16 < H) {
      float pre[NBT][7][4];  // gy, act i, g, f, o, tanh(c), c_prev
#pragma unroll
      for (int bt = 0; bt < NBT; ++bt) {
        const int m = bt * 16 + fr;
        if (m < B && jin) {
          ld4(p.gy, 0, ((long long)m * T + t) * H + j, pre[bt][0]);
          const float* a = p.acts + ((long long)t * B + m) * G + j;
#pragma unroll
          for (int g = 0; g < 4; ++g) ldf4(a + g * H, pre[bt][1 + g]);
          ldf4(p.tcs + ((long long)t * B + m) * H + j, pre[bt][5]);
          ldf4(t > 0 ? p.cs + ((long long)(t - 1) * B + m) * H + j : (p.c0 ? p.c0 + (long long)m * H + j : nullptr),
               pre[bt][6]);
        } else {
#pragma unroll
          for (int q = 0; q < 7; ++q) pre[bt][q][0] = pre[bt][q][1] = pre[bt][q][2] = pre[bt][q][3] = 0.f;
        }
      }
      v4f acc[NBT];
#pragma unroll
      for (int bt = 0; bt < NBT; ++bt) acc[bt] = v4f{0.f, 0.f, 0.f, 0.f};
      if (t + 1 < T) {
#pragma unroll 4
        for (int kc = 0; kc < KC; ++kc) {
          const int k = kc * 32 + fq * 8;
          const bool kin = k < G;
          const v8s wf = (kin && urow) ? *reinterpret_cast<const v8s*>(ub + k) : zero;
#pragma unroll
          for (int bt = 0; bt < NBT; ++bt) {
            const v8s gf = kin ? *reinterpret_cast<const v8s*>(&gc_[(bt * 16 + fr) * LDG + k]) : zero;
            acc[bt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf, gf, acc[bt], 0, 0, 0);
          }
        }
      }
#pragma unroll
      for (int bt = 0; bt < NBT; ++bt) {
        const int m = bt * 16 + fr;
        if (m >= B || !jin) continue;
        float di[4], dgg[4], df[4], dout[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const float i = pre[bt][1][e], g = pre[bt][2][e], f = pre[bt][3][e], o = pre[bt][4][e], tcv = pre[bt][5][e];
          const float d_h = pre[bt][0][e] + acc[bt][e];
          const float d_c = d_h * o * (1.f - tcv * tcv) + dc[bt][e];
          di[e] = d_c * g * i * (1.f - i);
          dgg[e] = d_c * i * (1.f - g * g);
          df[e] = d_c * pre[bt][6][e] * f * (1.f - f);
          dout[e] = d_h * tcv * o * (1.f - o);
          dc[bt][e] = d_c * f;
        }
        bf16_t* o = p.dg + ((long long)m * T + t) * G + j;
        stb4(o, di);
        stb4(o + H, dgg);
        stb4(o + 2 * H, df);
        stb4(o + 3 * H, dout);
        bf16_t* l = &gn[m * LDG + j];
        stb4(l, di);
        stb4(l + H, dgg);
        stb4(l + 2 * H, df);
        stb4(l + 3 * H, dout);
      }
    }
    __syncthreads();
  }
  if (w * 16 < H) {
#pragma unroll
    for (int bt = 0; bt < NBT; ++bt) {
      const int m = bt * 16 + fr;
      if (m < B && jin) stf4(p.gc + (long long)m * H + j, dc[bt]);
    }
  }
}

// ------------------------------------------------------------------------------------------------
// Multi-workgroup persistent LSTM (K14 resident-weight variant): ⌈H/16⌉ single-wave workgroups, one
// per 16-unit tile, run every time step of a layer-direction.  A workgroup's slice of the recurrent
// weight (forward: the 4 gate rows of its 16 units, 4·16×H; backward: the 16 Uᵀ rows, 16×4H) is
// loaded into REGISTERS once and stays there for the whole sequence — the step only reads the
// B×H (forward) / B×4H (backward) recurrent state written by all tiles in the previous step.
// Steps are separated by a grid barrier: a monotone arrival counter in global memory (agent-scope
// release add by each tile after its stores, agent-scope acquire spin before the next step's
// reads).  The tiles are few (≤ 16 workgroups of one wave) so they are always co-resident; the spin
// is bounded (a tile that waits ~1 s gives up and raises the error word instead of hanging).
// ------------------------------------------------------------------------------------------------
constexpr int kMpMaxKC = 8;    // forward: H ≤ 256 → ≤ 8 k-chunks of 32
constexpr int kMpMaxKCb = 32;  // backward: 4H ≤ 1024 → ≤ 32 k-chunks

// Two exchange protocols (template SC), selected by BIGDL_RNN_MP_SYNC (default 1):
//   SC = 0: plain stores / loads of the exchanged state; an agent-scope release fence (L2 write-back)
//           before the arrival and an agent-scope acquire fence (L2 invalidate) after the wait.
//   SC = 1: the exchanged state itself is written and read with agent-scope (device-coherent) 8-byte
//           accesses, so the barrier needs only the store acknowledgements (workgroup-scope release)
//           before the arrival — no whole-L2 write-back / invalidate per step.
// Either way the spin polls with relaxed agent-scope loads.
template <int SC>
__device__ __forceinline__ void mp_arrive(int* cnt) {
  if constexpr (SC == 1) __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
  else __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");  // this wave's stores → visible device-wide
  if ((threadIdx.x & 63) == 0) __hip_atomic_fetch_add(cnt, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

template <int SC>
__device__ __forceinline__ bool mp_wait(int* cnt, int target, int* err) {
  int spins = 0;
  while (__hip_atomic_load(cnt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target) {
    __builtin_amdgcn_s_sleep(1);
    if (++spins > (1 << 22)) {  // seconds: a tile never arrived (not co-resident?) — fail, do not hang
      if ((threadIdx.x & 63) == 0) __hip_atomic_store(err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      return false;
    }
  }
  if constexpr (SC == 1) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
  else __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
  return true;
}

// exchanged-state accessors: 4 bf16 (8 B) store, 8 bf16 (16 B) fragment load
template <int SC>
__device__ __forceinline__ void xst4(bf16_t* p, const float* v) {
  if constexpr (SC == 1) {
    const unsigned long long w = (unsigned long long)((uint32_t)f2bf(v[0]) | ((uint32_t)f2bf(v[1]) << 16)) |
                                 ((unsigned long long)((uint32_t)f2bf(v[2]) | ((uint32_t)f2bf(v[3]) << 16)) << 32);
    __hip_atomic_store(reinterpret_cast<unsigned long long*>(p), w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  } else {
    stb4(p, v);
  }
}
template <int SC>
__device__ __forceinline__ v8s xld8(const bf16_t* p) {
  if constexpr (SC == 1) {
    const unsigned long long* q = reinterpret_cast<const unsigned long long*>(p);
    const unsigned long long a = __hip_atomic_load(q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const unsigned long long b = __hip_atomic_load(q + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    typedef unsigned long long u2 __attribute__((ext_vector_type(2)));
    return __builtin_bit_cast(v8s, u2{a, b});
  } else {
    return *reinterpret_cast<const v8s*>(p);
  }
}

// SC = 2: no barrier at all — the exchanged state IS the flag (cdna_hip_programming.md §6 Guideline
// 16, R2).  Every 2 bf16 of h_t (forward) / dg_t (backward) travel as one naturally aligned 8-byte
// granule {tag = epoch, value} written by ONE agent-scope (sc1, write-through) store into a
// double-buffered slot; a consumer re-reads the granules of a 32-wide k-chunk with agent-scope (sc1,
// L1-bypassing) loads until every tag carries the step's epoch, then feeds them to the MFMA.  No
// counter, fence or acquire: a step's hand-off costs one store→load round trip through L2/fabric
// instead of store-ack → counter add → poll → fence → load.  Slot reuse (step t+2 overwrites step t)
// is safe: a tile writes step t+2 only after reading all of step t+1, which every tile wrote only
// after reading all of step t.  Epochs count from 1 within the launch; the launcher zeroes the
// slots first (a memset node under graph replay).
typedef __attribute__((address_space(1))) unsigned long long gu64_t;
__device__ __forceinline__ void gput(unsigned long long* g, unsigned epoch, const float* v) {
  const unsigned lo = (uint32_t)f2bf(v[0]) | ((uint32_t)f2bf(v[1]) << 16);
  const unsigned hi = (uint32_t)f2bf(v[2]) | ((uint32_t)f2bf(v[3]) << 16);
  __hip_atomic_store((gu64_t*)g, ((unsigned long long)epoch << 32) | lo, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __hip_atomic_store((gu64_t*)(g + 1), ((unsigned long long)epoch << 32) | hi, __ATOMIC_RELAXED,
                     __HIP_MEMORY_SCOPE_AGENT);
}
// 8 bf16 (4 granules) at g; returns whether every tag is `epoch`
__device__ __forceinline__ bool gget8(const unsigned long long* g, unsigned epoch, v8s& out) {
  unsigned v[4];
  bool ok = true;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const unsigned long long x = __hip_atomic_load((const gu64_t*)(g + q), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    v[q] = (unsigned)x;
    ok &= (unsigned)(x >> 32) == epoch;
  }
  typedef unsigned u4 __attribute__((ext_vector_type(4)));
  out = __builtin_bit_cast(v8s, u4{v[0], v[1], v[2], v[3]});
  return ok;
}
constexpr unsigned kGranSpin = 1u << 22;  // bounded spin: a tile that never publishes fails, no hang

// the same 4 granules as two 16-B agent-coherent (sc1, aux = 16) buffer loads: half the load
// instructions of gget8 (each 8-B half of a 16-B sc1 load is untorn on gfx950, MI355X_MICROARCH.md
// §visibility R2); `boff` is the byte offset of the first granule in the exchange buffer
__device__ __forceinline__ bool gget8b(__amdgpu_buffer_rsrc_t r, uint32_t boff, unsigned epoch, v8s& out) {
  typedef unsigned u4 __attribute__((ext_vector_type(4)));
  const u4 a = __builtin_bit_cast(u4, __builtin_amdgcn_raw_buffer_load_b128(r, (int)boff, 0, 16));
  const u4 b = __builtin_bit_cast(u4, __builtin_amdgcn_raw_buffer_load_b128(r, (int)boff + 16, 0, 16));
  out = __builtin_bit_cast(v8s, u4{a.x, a.z, b.x, b.z});
  return a.y == epoch && a.w == epoch && b.y == epoch && b.w == epoch;
}

template <int NBT, int SC>
__global__ void __launch_bounds__(64) k_lstm_seq_fwd_mp(LstmSeqP p, int* sync) {
  const int spread = p.spread > 0 ? p.spread : 1;
  if (blockIdx.x % spread) return;  // an idle slot of the XCD-confined grid
  const int tile = blockIdx.x / spread, ntiles = gridDim.x / spread;
  const int lane = threadIdx.x & 63, fr = lane & 15, fq = lane >> 4;
  const int H = p.H, B = p.B, T = p.T, G = 4 * H;
  const int u0 = tile * 16;
  const int j = u0 + fq * 4;  // this lane's unit quad
  const bool jin = j < H;
  const bool urow = u0 + fr < H;
  const int KC = (H + 31) / 32;
  const v8s zero = {0, 0, 0, 0, 0, 0, 0, 0};
  // resident weight fragments: gate g, k-chunk kc (lane = U row u0 + fr, k = 32 kc + 8 fq .. +7)
  v8s wf[4][kMpMaxKC];
  const bf16_t* ub = p.u + (long long)(urow ? u0 + fr : 0) * H;
#pragma unroll
  for (int g = 0; g < 4; ++g)
#pragma unroll
    for (int kc = 0; kc < kMpMaxKC; ++kc) {
      const int k = kc * 32 + fq * 8;
      wf[g][kc] = (kc < KC && k < H && urow) ? *reinterpret_cast<const v8s*>(ub + (long long)g * H * H + k) : zero;
    }
  float c[NBT][4];
#pragma unroll
  for (int bt = 0; bt < NBT; ++bt) {
    const int m = bt * 16 + fr;
#pragma unroll
    for (int e = 0; e < 4; ++e) c[bt][e] = (p.c0 && m < B && jin) ? p.c0[(long long)m * H + j + e] : 0.f;
  }
  int* cnt = sync;
  int* err = sync + 1;
  for (int t = 0; t < T; ++t) {
    // epilogue operands first: they do not depend on the other tiles
    uint2 xr[NBT][4];
#pragma unroll
    for (int bt = 0; bt < NBT; ++bt) {
      const int m = bt * 16 + fr;
#pragma unroll
      for (int g = 0; g < 4; ++g)
        xr[bt][g] = (!p.x_f32 && m < B && jin)
                        ? *reinterpret_cast<const uint2*>((const bf16_t*)p.x2 + ((long long)m * T + t) * G + g * H + j)
                        : make_uint2(0u, 0u);
    }
    if constexpr (SC < 2) {
      if (t > 0 && !mp_wait<SC>(cnt, t * ntiles, err)) return;
    }
    // h_{t-1}: the initial state or the previous step's output column of every tile
    const bf16_t* hb = t == 0 ? p.h0 : p.out + (long long)(t - 1) * H;
    const long long ldh = t == 0 ? H : (long long)T * H;
    // granule protocol: h_{t-1} sits in slot (t-1)&1 with epoch t
    const unsigned long long* gsl = p.xg + (size_t)((t - 1) & 1) * B * (H / 2);
    v4f acc[NBT][4];
#pragma unroll
    for (int bt = 0; bt < NBT; ++bt)
#pragma unroll
      for (int g = 0; g < 4; ++g) acc[bt][g] = v4f{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int kc = 0; kc < kMpMaxKC; ++kc) {
      const int k = kc * 32 + fq * 8;
      const bool kin = kc < KC && k < H;
      v8s hf[NBT];
      if (SC == 2 && t > 0) {
        for (unsigned spins = 0;; ++spins) {
          bool ok = true;
#pragma unroll
          for (int bt = 0; bt < NBT; ++bt) {
            const int m = bt * 16 + fr;
            hf[bt] = zero;
            if (kin && m < B) ok &= gget8(gsl + (size_t)m * (H / 2) + k / 2, (unsigned)t, hf[bt]);
          }
          if (__all(ok)) break;
          if (spins > kGranSpin) {
            if (lane == 0) __hip_atomic_store(err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            return;
          }
          __builtin_amdgcn_s_sleep(1);
        }
      } else {
#pragma unroll
        for (int bt = 0; bt < NBT; ++bt) {
          const int m = bt * 16 + fr;
          hf[bt] = (kin && m < B) ? (t == 0 ? *reinterpret_cast<const v8s*>(hb + m * ldh + k) : xld8<SC>(hb + m * ldh + k))
                                  : zero;
        }
      }
#pragma unroll
      for (int bt = 0; bt < NBT; ++bt)
#pragma unroll
        for (int g = 0; g < 4; ++g) acc[bt][g] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[g][kc], hf[bt], acc[bt][g], 0, 0, 0);
    }
#pragma unroll
    for (int bt = 0; bt < NBT; ++bt) {
      const int m = bt * 16 + fr;
      if (m >= B || !jin) continue;
      float xg[4][4];
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        if (p.x_f32) {
          ld4(p.x2, 1, ((long long)m * T + t) * G + g * H + j, xg[g]);
        } else {
          xg[g][0] = __uint_as_float(xr[bt][g].x << 16);
          xg[g][1] = __uint_as_float(xr[bt][g].x & 0xFFFF0000u);
          xg[g][2] = __uint_as_float(xr[bt][g].y << 16);
          xg[g][3] = __uint_as_float(xr[bt][g].y & 0xFFFF0000u);
        }
      }
      float gi[4], gg[4], gf[4], go[4], h[4], tcv[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        gi[e] = sgm(xg[0][e] + acc[bt][0][e]);
        gg[e] = tanhf(xg[1][e] + acc[bt][1][e]);
        gf[e] = sgm(xg[2][e] + acc[bt][2][e]);
        go[e] = sgm(xg[3][e] + acc[bt][3][e]);
        c[bt][e] = gi[e] * gg[e] + gf[e] * c[bt][e];
        tcv[e] = tanhf(c[bt][e]);
        h[e] = go[e] * tcv[e];
      }
      xst4<SC>(p.out + ((long long)m * T + t) * H + j, h);
      if (SC == 2 && t + 1 < T) gput(p.xg + (size_t)(t & 1) * B * (H / 2) + (size_t)m * (H / 2) + j / 2, (unsigned)(t + 1), h);
      const long long mh = ((long long)t * B + m) * H + j;
      if (p.cs) {
        stf4(p.cs + mh, c[bt]);
        stf4(p.tcs + mh, tcv);
        float* a = p.acts + ((long long)t * B + m) * G + j;
        stf4(a, gi);
        stf4(a + H, gg);
        stf4(a + 2 * H, gf);
        stf4(a + 3 * H, go);
      }
    }
    if constexpr (SC < 2) {
      if (t + 1 < T) mp_arrive<SC>(cnt);
    }
  }
  if (p.cbuf) {  // inference: the final c, where the step path leaves it (slot (T-1)&1)
#pragma unroll
    for (int bt = 0; bt < NBT; ++bt) {
      const int m = bt * 16 + fr;
      if (m < B && jin) stf4(p.cbuf + (long long)((T - 1) & 1) * B * H + (long long)m * H + j, c[bt]);
    }
  }
}

template <int NBT, int SC>
__global__ void __launch_bounds__(64) k_lstm_seq_bwd_mp(LstmSeqP p, int* sync) {
  const int spread = p.spread > 0 ? p.spread : 1;
  if (blockIdx.x % spread) return;
  const int tile = blockIdx.x / spread, ntiles = gridDim.x / spread;
  const int lane = threadIdx.x & 63, fr = lane & 15, fq = lane >> 4;
  const int H = p.H, B = p.B, T = p.T, G = 4 * H;
  const int u0 = tile * 16;
  const int j = u0 + fq * 4;
  const bool jin = j < H;
  const bool urow = u0 + fr < H;
  const int KC = (G + 31) / 32;
  const v8s zero = {0, 0, 0, 0, 0, 0, 0, 0};
  v8s wf[kMpMaxKCb];  // Uᵀ row u0 + fr: Σ_k dg[k]·U[k][j]
  const bf16_t* ub = p.u + (long long)(urow ? u0 + fr : 0) * G;
#pragma unroll
  for (int kc = 0; kc < kMpMaxKCb; ++kc) {
    const int k = kc * 32 + fq * 8;
    wf[kc] = (kc < KC && k < G && urow) ? *reinterpret_cast<const v8s*>(ub + k) : zero;
  }
  float dc[NBT][4];
#pragma unroll
  for (int bt = 0; bt < NBT; ++bt)
#pragma unroll
    for (int e = 0; e < 4; ++e) dc[bt][e] = 0.f;
  int* cnt = sync;
  int* err = sync + 1;
  for (int t = T - 1; t >= 0; --t) {
    float pre[NBT][7][4];  // gy, act i, g, f, o, tanh(c), c_prev
#pragma unroll
    for (int bt = 0; bt < NBT; ++bt) {
      const int m = bt * 16 + fr;
      if (m < B && jin) {
        ld4(p.gy, 0, ((long long)m * T + t) * H + j, pre[bt][0]);
        const float* a = p.acts + ((long long)t * B + m) * G + j;
#pragma unroll
        for (int g = 0; g < 4; ++g) ldf4(a + g * H, pre[bt][1 + g]);
        ldf4(p.tcs + ((long long)t * B + m) * H + j, pre[bt][5]);
        ldf4(t > 0 ? p.cs + ((long long)(t - 1) * B + m) * H + j : (p.c0 ? p.c0 + (long long)m * H + j : nullptr),
             pre[bt][6]);
      } else {
#pragma unroll
        for (int q = 0; q < 7; ++q) pre[bt][q][0] = pre[bt][q][1] = pre[bt][q][2] = pre[bt][q][3] = 0.f;
      }
    }
    v4f acc[NBT];
#pragma unroll
    for (int bt = 0; bt < NBT; ++bt) acc[bt] = v4f{0.f, 0.f, 0.f, 0.f};
    if (t + 1 < T) {
      if constexpr (SC < 2) {
        if (!mp_wait<SC>(cnt, (T - 1 - t) * ntiles, err)) return;
      }
      const bf16_t* gb = p.dg + (long long)(t + 1) * G;  // dg_{t+1} rows, stride T·G
      // granule protocol: dg_{t+1} sits in slot (t+1)&1 with epoch T-1-t
      const unsigned long long* gsl = p.xg + (size_t)((t + 1) & 1) * B * (G / 2);
      const unsigned ep = (unsigned)(T - 1 - t);
#pragma unroll
      for (int kc = 0; kc < kMpMaxKCb; ++kc) {  // chunks past 4H hold zero fragments (no branch: keeps wf in VGPRs)
        const int k = kc * 32 + fq * 8;
        const bool kin = kc < KC && k < G;
        v8s gf[NBT];
        if constexpr (SC == 2) {
          for (unsigned spins = 0;; ++spins) {
            bool ok = true;
#pragma unroll
            for (int bt = 0; bt < NBT; ++bt) {
              const int m = bt * 16 + fr;
              gf[bt] = zero;
              if (kin && m < B) ok &= gget8(gsl + (size_t)m * (G / 2) + k / 2, ep, gf[bt]);
            }
            if (__all(ok)) break;
            if (spins > kGranSpin) {
              if (lane == 0) __hip_atomic_store(err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
              return;
            }
            __builtin_amdgcn_s_sleep(1);
          }
        } else {
#pragma unroll
          for (int bt = 0; bt < NBT; ++bt) {
            const int m = bt * 16 + fr;
            gf[bt] = (kin && m < B) ? xld8<SC>(gb + (long long)m * T * G + k) : zero;
          }
        }
#pragma unroll
        for (int bt = 0; bt < NBT; ++bt) acc[bt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[kc], gf[bt], acc[bt], 0, 0, 0);
      }
    }
#pragma unroll
    for (int bt = 0; bt < NBT; ++bt) {
      const int m = bt * 16 + fr;
      if (m >= B || !jin) continue;
      float di[4], dgg[4], df[4], dout[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float i = pre[bt][1][e], g = pre[bt][2][e], f = pre[bt][3][e], o = pre[bt][4][e], tcv = pre[bt][5][e];
        const float d_h = pre[bt][0][e] + acc[bt][e];
        const float d_c = d_h * o * (1.f - tcv * tcv) + dc[bt][e];
        di[e] = d_c * g * i * (1.f - i);
        dgg[e] = d_c * i * (1.f - g * g);
        df[e] = d_c * pre[bt][6][e] * f * (1.f - f);
        dout[e] = d_h * tcv * o * (1.f - o);
        dc[bt][e] = d_c * f;
      }
      bf16_t* o = p.dg + ((long long)m * T + t) * G + j;
      xst4<SC>(o, di);
      xst4<SC>(o + H, dgg);
      xst4<SC>(o + 2 * H, df);
      xst4<SC>(o + 3 * H, dout);
      if (SC == 2 && t > 0) {
        unsigned long long* gq = p.xg + (size_t)(t & 1) * B * (G / 2) + (size_t)m * (G / 2) + j / 2;
        const unsigned ep = (unsigned)(T - t);
        gput(gq, ep, di);
        gput(gq + H / 2, ep, dgg);
        gput(gq + H, ep, df);
        gput(gq + 3 * H / 2, ep, dout);
      }
    }
    if constexpr (SC < 2) {
      if (t > 0) mp_arrive<SC>(cnt);
    }
  }
#pragma unroll
  for (int bt = 0; bt < NBT; ++bt) {
    const int m = bt * 16 + fr;
    if (m < B && jin) stf4(p.gc + (long long)m * H + j, dc[bt]);
  }
}

// ------------------------------------------------------------------------------------------------
// Granule hand-off with FOUR waves per 16-unit tile (BIGDL_RNN_PERSIST=6 / 7): the k-chunks of the
// recurrent product are dealt round-robin to the waves (wave w: kc ≡ w mod 4), so each wave holds a
// quarter of the tile's weight slice and sweeps a quarter of the exchanged granules — the per-step
// poll + load + MFMA chain, which is the step's latency, is ~4× shorter.  The partial accumulators
// meet in LDS; wave 0 runs the cell and publishes the tile's granules.  A wave whose bounded spin
// expires raises the block's abort word (LDS) and the error word, and the whole block leaves at the
// next barrier (no wave is left waiting at a barrier).
constexpr int kGw = 4;  // waves per tile

template <int NBT>
__global__ void __launch_bounds__(64 * kGw) k_lstm_seq_fwd_gw(LstmSeqP p, int* sync) {
  const int spread = p.spread > 0 ? p.spread : 1;
  if (blockIdx.x % spread) return;
  const int tile = blockIdx.x / spread;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, fr = lane & 15, fq = lane >> 4;
  const int H = p.H, B = p.B, T = p.T, G = 4 * H;
  const int u0 = tile * 16;
  const int j = u0 + fq * 4;
  const bool jin = j < H;
  const bool urow = u0 + fr < H;
  const int KC = (H + 31) / 32;
  constexpr int QC = kMpMaxKC / kGw;  // chunks per wave
  const v8s zero = {0, 0, 0, 0, 0, 0, 0, 0};
  __shared__ v4f red[kGw][NBT][4][64];
  __shared__ int abort_flag;
  if (threadIdx.x == 0) abort_flag = 0;
  v8s wf[4][QC];
  const bf16_t* ub = p.u + (long long)(urow ? u0 + fr : 0) * H;
#pragma unroll
  for (int g = 0; g < 4; ++g)
#pragma unroll
    for (int q = 0; q < QC; ++q) {
      const int kc = q * kGw + w, k = kc * 32 + fq * 8;
      wf[g][q] = (kc < KC && k < H && urow) ? *reinterpret_cast<const v8s*>(ub + (long long)g * H * H + k) : zero;
    }
  float c[NBT][4];
#pragma unroll
  for (int bt = 0; bt < NBT; ++bt) {
    const int m = bt * 16 + fr;
#pragma unroll
    for (int e = 0; e < 4; ++e) c[bt][e] = (w == 0 && p.c0 && m < B && jin) ? p.c0[(long long)m * H + j + e] : 0.f;
  }
  int* err = sync + 1;
  const __amdgpu_buffer_rsrc_t xgr =
      __builtin_amdgcn_make_buffer_rsrc((void*)p.xg, 0, (int)((size_t)2 * B * (H / 2) * 8), 0x00020000);
  __syncthreads();
  for (int t = 0; t < T; ++t) {
    uint2 xr[NBT][4];
#pragma unroll
    for (int bt = 0; bt < NBT; ++bt) {
      const int m = bt * 16 + fr;
#pragma unroll
      for (int g = 0; g < 4; ++g)
        xr[bt][g] = (w == 0 && !p.x_f32 && m < B && jin)
                        ? *reinterpret_cast<const uint2*>((const bf16_t*)p.x2 + ((long long)m * T + t) * G + g * H + j)
                        : make_uint2(0u, 0u);
    }
    const unsigned long long* gsl = p.xg + (size_t)((t - 1) & 1) * B * (H / 2);
    v4f acc[NBT][4];
#pragma unroll
    for (int bt = 0; bt < NBT; ++bt)
#pragma unroll
      for (int g = 0; g < 4; ++g) acc[bt][g] = v4f{0.f, 0.f, 0.f, 0.f};
    bool failed = false;
#pragma unroll
    for (int q = 0; q < QC; ++q) {
      const int kc = q * kGw + w, k = kc * 32 + fq * 8;
      if (kc >= KC) continue;  // wave-uniform; lanes past H (k ≥ H) feed zero fragments
      const bool kin = k < H;
      v8s hf[NBT];
      if (t > 0) {
        for (unsigned spins = 0;; ++spins) {
          bool ok = true;
#pragma unroll
          for (int bt = 0; bt < NBT; ++bt) {
            const int m = bt * 16 + fr;
            hf[bt] = zero;
            if (kin && m < B)
              ok &= gget8b(xgr, (uint32_t)((((t - 1) & 1) * B * (H / 2) + m * (H / 2) + k / 2) * 8), (unsigned)t, hf[bt]);
          }
          if (__all(ok)) break;
          if (spins > kGranSpin) { failed = true; break; }
          __builtin_amdgcn_s_sleep(1);
        }
      } else {
#pragma unroll
        for (int bt = 0; bt < NBT; ++bt) {
          const int m = bt * 16 + fr;
          hf[bt] = (kin && m < B) ? *reinterpret_cast<const v8s*>(p.h0 + (long long)m * H + k) : zero;
        }
      }
      if (failed) break;
#pragma unroll
      for (int bt = 0; bt < NBT; ++bt)
#pragma unroll
        for (int g = 0; g < 4; ++g) acc[bt][g] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[g][q], hf[bt], acc[bt][g], 0, 0, 0);
    }
    if (failed && lane == 0) {
      abort_flag = 1;
      __hip_atomic_store(err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    if (w > 0) {
#pragma unroll
      for (int bt = 0; bt < NBT; ++bt)
#pragma unroll
        for (int g = 0; g < 4; ++g) red[w][bt][g][lane] = acc[bt][g];
    }
    __syncthreads();
    if (abort_flag) return;  // block-uniform after the barrier
    if (w == 0) {
#pragma unroll
      for (int v = 1; v < kGw; ++v)
#pragma unroll
        for (int bt = 0; bt < NBT; ++bt)
#pragma unroll
          for (int g = 0; g < 4; ++g) acc[bt][g] += red[v][bt][g][lane];
#pragma unroll
      for (int bt = 0; bt < NBT; ++bt) {
        const int m = bt * 16 + fr;
        if (m >= B || !jin) continue;
        float xg[4][4];
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          if (p.x_f32) {
            ld4(p.x2, 1, ((long long)m * T + t) * G + g * H + j, xg[g]);
          } else {
            xg[g][0] = __uint_as_float(xr[bt][g].x << 16);
            xg[g][1] = __uint_as_float(xr[bt][g].x & 0xFFFF0000u);
            xg[g][2] = __uint_as_float(xr[bt][g].y << 16);
            xg[g][3] = __uint_as_float(xr[bt][g].y & 0xFFFF0000u);
          }
        }
        float gi[4], gg[4], gf[4], go[4], h[4], tcv[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          gi[e] = sgm(xg[0][e] + acc[bt][0][e]);
          gg[e] = tanhf(xg[1][e] + acc[bt][1][e]);
          gf[e] = sgm(xg[2][e] + acc[bt][2][e]);
          go[e] = sgm(xg[3][e] + acc[bt][3][e]);
          c[bt][e] = gi[e] * gg[e] + gf[e] * c[bt][e];
          tcv[e] = tanhf(c[bt][e]);
          h[e] = go[e] * tcv[e];
        }
        if (t + 1 < T) gput(p.xg + (size_t)(t & 1) * B * (H / 2) + (size_t)m * (H / 2) + j / 2, (unsigned)(t + 1), h);
        stb4(p.out + ((long long)m * T + t) * H + j, h);
        const long long mh = ((long long)t * B + m) * H + j;
        if (p.cs) {
          stf4(p.cs + mh, c[bt]);
          stf4(p.tcs + mh, tcv);
          float* a = p.acts + ((long long)t * B + m) * G + j;
          stf4(a, gi);
          stf4(a + H, gg);
          stf4(a + 2 * H, gf);
          stf4(a + 3 * H, go);
        }
      }
    }
    __syncthreads();  // wave 0 is done with `red` before the next step's partials land
  }
  if (p.cbuf && w == 0) {
#pragma unroll
    for (int bt = 0; bt < NBT; ++bt) {
      const int m = bt * 16 + fr;
      if (m < B && jin) stf4(p.cbuf + (long long)((T - 1) & 1) * B * H + (long long)m * H + j, c[bt]);
    }
  }
}

template <int NBT>
__global__ void __launch_bounds__(64 * kGw) k_lstm_seq_bwd_gw(LstmSeqP p, int* sync) {
  const int spread = p.spread > 0 ? p.spread : 1;
  if (blockIdx.x % spread) return;
  const int tile = blockIdx.x / spread;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, fr = lane & 15, fq = lane >> 4;
  const int H = p.H, B = p.B, T = p.T, G = 4 * H;
  const int u0 = tile * 16;
  const int j = u0 + fq * 4;
  const bool jin = j < H;
  const bool urow = u0 + fr < H;
  const int KC = (G + 31) / 32;
  constexpr int QC = kMpMaxKCb / kGw;
  const v8s zero = {0, 0, 0, 0, 0, 0, 0, 0};
  __shared__ v4f red[kGw][NBT][64];
  __shared__ int abort_flag;
  if (threadIdx.x == 0) abort_flag = 0;
  v8s wf[QC];
  const bf16_t* ub = p.u + (long long)(urow ? u0 + fr : 0) * G;
#pragma unroll
  for (int q = 0; q < QC; ++q) {
    const int kc = q * kGw + w, k = kc * 32 + fq * 8;
    wf[q] = (kc < KC && k < G && urow) ? *reinterpret_cast<const v8s*>(ub + k) : zero;
  }
  float dc[NBT][4];
#pragma unroll
  for (int bt = 0; bt < NBT; ++bt)
#pragma unroll
    for (int e = 0; e < 4; ++e) dc[bt][e] = 0.f;
  int* err = sync + 1;
  const __amdgpu_buffer_rsrc_t xgr =
      __builtin_amdgcn_make_buffer_rsrc((void*)p.xg, 0, (int)((size_t)2 * B * (G / 2) * 8), 0x00020000);
  __syncthreads();
  for (int t = T - 1; t >= 0; --t) {
    float pre[NBT][7][4];  // gy, act i, g, f, o, tanh(c), c_prev (wave 0)
#pragma unroll
    for (int bt = 0; bt < NBT; ++bt) {
      const int m = bt * 16 + fr;
      if (w == 0 && m < B && jin) {
        ld4(p.gy, 0, ((long long)m * T + t) * H + j, pre[bt][0]);
        const float* a = p.acts + ((long long)t * B + m) * G + j;
#pragma unroll
        for (int g = 0; g < 4; ++g) ldf4(a + g * H, pre[bt][1 + g]);
        ldf4(p.tcs + ((long long)t * B + m) * H + j, pre[bt][5]);
        ldf4(t > 0 ? p.cs + ((long long)(t - 1) * B + m) * H + j : (p.c0 ? p.c0 + (long long)m * H + j : nullptr),
             pre[bt][6]);
      } else {
#pragma unroll
        for (int q = 0; q < 7; ++q) pre[bt][q][0] = pre[bt][q][1] = pre[bt][q][2] = pre[bt][q][3] = 0.f;
      }
    }
    v4f acc[NBT];
#pragma unroll
    for (int bt = 0; bt < NBT; ++bt) acc[bt] = v4f{0.f, 0.f, 0.f, 0.f};
    bool failed = false;
    if (t + 1 < T) {
      const unsigned long long* gsl = p.xg + (size_t)((t + 1) & 1) * B * (G / 2);
      const unsigned ep = (unsigned)(T - 1 - t);
#pragma unroll
      for (int q = 0; q < QC; ++q) {
        const int kc = q * kGw + w, k = kc * 32 + fq * 8;
        if (kc >= KC) continue;  // wave-uniform; lanes past 4H feed zero fragments
        const bool kin = k < G;
        v8s gf[NBT];
        for (unsigned spins = 0;; ++spins) {
          bool ok = true;
#pragma unroll
          for (int bt = 0; bt < NBT; ++bt) {
            const int m = bt * 16 + fr;
            gf[bt] = zero;
            if (kin && m < B)
              ok &= gget8b(xgr, (uint32_t)((((t + 1) & 1) * B * (G / 2) + m * (G / 2) + k / 2) * 8), ep, gf[bt]);
          }
          if (__all(ok)) break;
          if (spins > kGranSpin) { failed = true; break; }
          __builtin_amdgcn_s_sleep(1);
        }
        if (failed) break;
#pragma unroll
        for (int bt = 0; bt < NBT; ++bt) acc[bt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[q], gf[bt], acc[bt], 0, 0, 0);
      }
    }
    if (failed && lane == 0) {
      abort_flag = 1;
      __hip_atomic_store(err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    if (w > 0) {
#pragma unroll
      for (int bt = 0; bt < NBT; ++bt) red[w][bt][lane] = acc[bt];
    }
    __syncthreads();
    if (abort_flag) return;
    if (w == 0) {
#pragma unroll
      for (int v = 1; v < kGw; ++v)
#pragma unroll
        for (int bt = 0; bt < NBT; ++bt) acc[bt] += red[v][bt][lane];
#pragma unroll
      for (int bt = 0; bt < NBT; ++bt) {
        const int m = bt * 16 + fr;
        if (m >= B || !jin) continue;
        float di[4], dgg[4], df[4], dout[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const float i = pre[bt][1][e], g = pre[bt][2][e], f = pre[bt][3][e], o = pre[bt][4][e], tcv = pre[bt][5][e];
          const float d_h = pre[bt][0][e] + acc[bt][e];
          const float d_c = d_h * o * (1.f - tcv * tcv) + dc[bt][e];
          di[e] = d_c * g * i * (1.f - i);
          dgg[e] = d_c * i * (1.f - g * g);
          df[e] = d_c * pre[bt][6][e] * f * (1.f - f);
          dout[e] = d_h * tcv * o * (1.f - o);
          dc[bt][e] = d_c * f;
        }
        if (t > 0) {
          unsigned long long* gq = p.xg + (size_t)(t & 1) * B * (G / 2) + (size_t)m * (G / 2) + j / 2;
          const unsigned ep = (unsigned)(T - t);
          gput(gq, ep, di);
          gput(gq + H / 2, ep, dgg);
          gput(gq + H, ep, df);
          gput(gq + 3 * H / 2, ep, dout);
        }
        bf16_t* o = p.dg + ((long long)m * T + t) * G + j;
        stb4(o, di);
        stb4(o + H, dgg);
        stb4(o + 2 * H, df);
        stb4(o + 3 * H, dout);
      }
    }
    __syncthreads();
  }
  if (w == 0) {
#pragma unroll
    for (int bt = 0; bt < NBT; ++bt) {
      const int m = bt * 16 + fr;
      if (m < B && jin) stf4(p.gc + (long long)m * H + j, dc[bt]);
    }
  }
}

// Resident-weight multi-workgroup path: B ≤ 32, 8 ≤ H ≤ 256, H % 8 == 0, a sync word pair given.
// OPT-IN (BIGDL_RNN_PERSIST=2).  Measured at the PTB shape (B 20, H 200, T 20, 2 layers) it is
// SLOWER than one k_rnn_step launch per step — 1.34 (fence protocol) / 1.40 (scoped accesses) vs
// 1.05–1.12 ms per training step, profiles/r3_ptb_persist_ab.txt: the step-to-step hand-off crosses
// XCDs (each has its own L2), so every step pays device-coherent store → counter → poll → load round
// trips at memory-side latency, which costs more than the back-to-back launch of the next step
// whose h reads hit L2.
static bool lstm_mp_sc() {
  const char* e = getenv("BIGDL_RNN_MP_SYNC");
  return !(e && e[0] == '0');
}

static int lstm_persist_mode() {  // read per whole-sequence call (tests switch it in-process)
  const char* e = getenv("BIGDL_RNN_PERSIST");
  return e ? atoi(e) : 0;
}

// BIGDL_RNN_PERSIST=2: the multi-workgroup kernels on ⌈H/16⌉ workgroups wherever they land, counter
// barrier (protocol BIGDL_RNN_MP_SYNC 0/1); =3: the same tiles confined to one XCD (8 × tiles
// workgroups, every 8th one works); =4 / =5: the granule protocol (SC = 2, no barrier), spread 1 / 8;
// =6 / =7: the granule protocol with four waves per tile (k_lstm_seq_{fwd,bwd}_gw), spread 1 / 8
static bool lstm_mp_ok(int B, int H, const int* sync, const void* xg) {
  const int m = lstm_persist_mode();
  if (m < 2 || m > 7 || (m >= 4 && !xg)) return false;
  return sync && B >= 1 && B <= 32 && H >= 8 && H <= kPersistMaxH && H % 8 == 0;
}

static int lstm_mp_spread() {
  const int m = lstm_persist_mode();
  return (m == 3 || m == 5 || m == 7) ? 8 : 1;
}

static int lstm_mp_proto() {
  const int m = lstm_persist_mode();
  return m >= 6 ? 3 : (m == 4 || m == 5) ? 2 : (lstm_mp_sc() ? 1 : 0);
}

template <int NBT>
static void launch_fwd_mp(int proto, dim3 grid, hipStream_t s, const LstmSeqP& p, int* sync) {
  if (proto == 3) hipLaunchKernelGGL((k_lstm_seq_fwd_gw<NBT>), grid, dim3(64 * kGw), 0, s, p, sync);
  else if (proto == 2) hipLaunchKernelGGL((k_lstm_seq_fwd_mp<NBT, 2>), grid, dim3(64), 0, s, p, sync);
  else if (proto == 1) hipLaunchKernelGGL((k_lstm_seq_fwd_mp<NBT, 1>), grid, dim3(64), 0, s, p, sync);
  else hipLaunchKernelGGL((k_lstm_seq_fwd_mp<NBT, 0>), grid, dim3(64), 0, s, p, sync);
}

template <int NBT>
static void launch_bwd_mp(int proto, dim3 grid, hipStream_t s, const LstmSeqP& p, int* sync) {
  if (proto == 3) hipLaunchKernelGGL((k_lstm_seq_bwd_gw<NBT>), grid, dim3(64 * kGw), 0, s, p, sync);
  else if (proto == 2) hipLaunchKernelGGL((k_lstm_seq_bwd_mp<NBT, 2>), grid, dim3(64), 0, s, p, sync);
  else if (proto == 1) hipLaunchKernelGGL((k_lstm_seq_bwd_mp<NBT, 1>), grid, dim3(64), 0, s, p, sync);
  else hipLaunchKernelGGL((k_lstm_seq_bwd_mp<NBT, 0>), grid, dim3(64), 0, s, p, sync);
}

// The persistent path covers B ≤ 32 and 8 ≤ H ≤ 256 (H % 8 == 0).  It is OPT-IN
// (BIGDL_RNN_PERSIST=1): one CU re-streams all of U from L2 every step, and a single CU's L2 read
// rate (tens of GB/s) makes that ~3× slower than the 13-workgroup step launches at the PTB shape
// (B 20, H 200: 1.50 vs 1.13 ms per training step, profiles/r3_ptb_persist_ab.txt).
static bool lstm_persist_ok(int B, int H) {
  if (lstm_persist_mode() != 1) return false;
  return B >= 1 && B <= 32 && H >= 8 && H <= kPersistMaxH && H % 8 == 0;
}

// ------------------------------------------------------------------------------------------------
// Whole-sequence launchers: the time loop runs on the host in C++, one validated rnn_step launch
// per step — the Python side makes ONE call per layer per direction (the eager PTB step was bound
// by per-step Python/ctypes dispatch, not by the GPU).  Layouts (elements, bf16 unless noted):
//   x2 [B][T][G·H] input projection, out [B][T][H] hidden sequence, per-step fp32 saves [T][B][·],
//   DG [B][T][G·H] gate gradients.  Graph-capturable (launches only, no host sync).
// ------------------------------------------------------------------------------------------------
static const bf16_t* bo(const void* p, long long off) { return p ? (const bf16_t*)p + off : nullptr; }

// element pointer `off` elements past p in the activation type (bf16 or fp32)
static const void* eo(const void* p, long long off, int f32) { return p ? (const char*)p + off * (f32 ? 4 : 2) : nullptr; }
static void* eo(void* p, long long off, int f32) { return p ? (char*)p + off * (f32 ? 4 : 2) : nullptr; }

// The per-step loop of a single-layer LSTM forward (one rnn_step launch per step).
static int lstm_fwd_steps(const void* x2, int x_f32, const void* h0, const float* c0, const void* U, void* out,
                          float* cs, float* acts, float* tcs, float* cbuf, int B, int T, int H, int f32, hipStream_t s) {
  const bool train = cs && acts && tcs;
  const long long G = 4LL * H, BH = (long long)B * H;
  const int esz = x_f32 ? 4 : 2;
  for (int t = 0; t < T; ++t) {
    const void* a = t == 0 ? h0 : eo((const void*)out, (long long)(t - 1) * H, f32);
    const long long lda = t == 0 ? H : (long long)T * H;
    const void* xg = (const char*)x2 + (long long)t * G * esz;
    const float* cp = t == 0 ? c0 : (train ? cs + (t - 1) * BH : cbuf + ((t - 1) & 1) * BH);
    float* co = train ? cs + t * BH : cbuf + (t & 1) * BH;
    int rc = rnn_step_run(0, a, lda, U, B, H, H, xg, (long long)T * G, x_f32, nullptr, 0, cp,
                          eo(out, (long long)t * H, f32), (long long)T * H, co, train ? acts + t * B * G : nullptr,
                          train ? tcs + t * BH : nullptr, nullptr, 0, nullptr, nullptr, 0, nullptr, nullptr, nullptr,
                          nullptr, nullptr, 0, f32, s);
    if (rc) return rc;
  }
  return 0;
}

// The per-step loop of a single-layer LSTM backward.
static int lstm_bwd_steps(const void* gy, const void* Ut, const float* acts, const float* tcs, const float* cs,
                          const float* c0, void* DG, float* gc, int B, int T, int H, int f32, hipStream_t s) {
  const long long G = 4LL * H, BH = (long long)B * H;
  for (int t = T - 1; t >= 0; --t) {
    const bool last = t + 1 == T;
    int rc = rnn_step_run(1, last ? nullptr : eo((const void*)DG, (t + 1) * G, f32), (long long)T * G, Ut, B, (int)G,
                          H, nullptr, 0, 0, nullptr, 0, t > 0 ? cs + (t - 1) * BH : c0, nullptr, 0, nullptr,
                          (float*)acts + t * B * G, (float*)tcs + t * BH, eo(gy, (long long)t * H, f32), (long long)T * H,
                          last ? nullptr : gc, eo(DG, t * G, f32), (long long)T * G, gc, nullptr, nullptr, nullptr,
                          nullptr, 0, f32, s);
    if (rc) return rc;
  }
  return 0;
}

BIGDL_EXPORT int bigdl_lstm_seq_fwd(const void* x2, int x_f32, const void* h0, const float* c0, const void* U, void* out,
                                    float* cs, float* acts, float* tcs, float* cbuf, int B, int T, int H, int* sync,
                                    void* xg, hipStream_t s) {
  if (B <= 0 || T <= 0 || H <= 0 || !x2 || !h0 || !U || !out) return (int)hipErrorInvalidValue;
  const bool train = cs && acts && tcs;
  if (!train && !cbuf) return (int)hipErrorInvalidValue;
  const long long G = 4LL * H, BH = (long long)B * H;
  const int esz = x_f32 ? 4 : 2;
  if (lstm_mp_ok(B, H, sync, xg)) {
    if (!a16(U) || !a16(h0) || !a16(out) || (x_f32 ? !a16(x2) : !a8(x2)) || ((uintptr_t)sync & 7) || !a16(xg))
      return (int)hipErrorInvalidValue;
    const void* f32s[] = {c0, cs, acts, tcs, cbuf};
    for (const void* q : f32s)
      if (q && !a16(q)) return (int)hipErrorInvalidValue;
    LstmSeqP p{};
    p.x2 = x2; p.x_f32 = x_f32; p.h0 = (const bf16_t*)h0; p.c0 = c0; p.u = (const bf16_t*)U; p.out = (bf16_t*)out;
    p.cs = train ? cs : nullptr; p.acts = acts; p.tcs = tcs; p.cbuf = train ? nullptr : cbuf;
    p.B = B; p.T = T; p.H = H; p.spread = lstm_mp_spread();
    p.xg = (unsigned long long*)xg;
    const int proto = lstm_mp_proto();
    hipError_t e = hipMemsetAsync(sync, 0, 2 * sizeof(int), s);
    if (e == hipSuccess && proto >= 2) e = hipMemsetAsync(xg, 0, (size_t)2 * B * (H / 2) * 8, s);
    if (e != hipSuccess) return (int)e;
    const dim3 grid((unsigned)((H + 15) / 16 * p.spread));
    if (B <= 16) launch_fwd_mp<1>(proto, grid, s, p, sync);
    else launch_fwd_mp<2>(proto, grid, s, p, sync);
    BIGDL_CHECK_LAUNCH();
  }
  if (lstm_persist_ok(B, H)) {
    if (!a16(U) || !a8(h0) || !a8(out) || (x_f32 ? !a16(x2) : !a8(x2))) return (int)hipErrorInvalidValue;
    const void* f32s[] = {c0, cs, acts, tcs, cbuf};
    for (const void* q : f32s)
      if (q && !a16(q)) return (int)hipErrorInvalidValue;
    LstmSeqP p{};
    p.x2 = x2; p.x_f32 = x_f32; p.h0 = (const bf16_t*)h0; p.c0 = c0; p.u = (const bf16_t*)U; p.out = (bf16_t*)out;
    p.cs = train ? cs : nullptr; p.acts = acts; p.tcs = tcs; p.cbuf = train ? nullptr : cbuf;
    p.B = B; p.T = T; p.H = H;
    if (B <= 16) hipLaunchKernelGGL(k_lstm_seq_fwd_p<1>, dim3(1), dim3(1024), 0, s, p);
    else hipLaunchKernelGGL(k_lstm_seq_fwd_p<2>, dim3(1), dim3(1024), 0, s, p);
    BIGDL_CHECK_LAUNCH();
  }
  return lstm_fwd_steps(x2, x_f32, h0, c0, U, out, cs, acts, tcs, cbuf, B, T, H, 0, s);
}

// All-fp32 LSTM (bf16x3 recurrent products, k_rnn_step<…, true>): x2, h0, U, out fp32.
BIGDL_EXPORT int bigdl_lstm_seq_fwd32(const float* x2, const float* h0, const float* c0, const float* U, float* out,
                                      float* cs, float* acts, float* tcs, float* cbuf, int B, int T, int H,
                                      hipStream_t s) {
  if (B <= 0 || T <= 0 || H <= 0 || !x2 || !h0 || !U || !out) return (int)hipErrorInvalidValue;
  if (!(cs && acts && tcs) && !cbuf) return (int)hipErrorInvalidValue;
  return lstm_fwd_steps(x2, 1, h0, c0, U, out, cs, acts, tcs, cbuf, B, T, H, 1, s);
}

BIGDL_EXPORT int bigdl_lstm_seq_bwd(const void* gy, const void* Ut, const float* acts, const float* tcs, const float* cs,
                                    const float* c0, void* DG, float* gc, int B, int T, int H, int* sync,
                                    void* xg, hipStream_t s) {
  if (B <= 0 || T <= 0 || H <= 0 || !gy || !Ut || !DG || !gc) return (int)hipErrorInvalidValue;
  const long long G = 4LL * H, BH = (long long)B * H;
  if (lstm_mp_ok(B, H, sync, xg)) {
    if (!acts || !tcs || !cs || !a16(Ut) || !a8(gy) || !a16(DG) || !a16(acts) || !a16(tcs) || !a16(cs) || !a16(gc) ||
        (c0 && !a16(c0)) || ((uintptr_t)sync & 7) || !a16(xg))
      return (int)hipErrorInvalidValue;
    LstmSeqP p{};
    p.u = (const bf16_t*)Ut; p.acts = (float*)acts; p.tcs = (float*)tcs; p.cs = (float*)cs; p.c0 = c0;
    p.gy = (const bf16_t*)gy; p.dg = (bf16_t*)DG; p.gc = gc; p.B = B; p.T = T; p.H = H; p.spread = lstm_mp_spread();
    p.xg = (unsigned long long*)xg;
    const int proto = lstm_mp_proto();
    hipError_t e = hipMemsetAsync(sync, 0, 2 * sizeof(int), s);
    if (e == hipSuccess && proto >= 2) e = hipMemsetAsync(xg, 0, (size_t)2 * B * (2 * H) * 8, s);
    if (e != hipSuccess) return (int)e;
    const dim3 grid((unsigned)((H + 15) / 16 * p.spread));
    if (B <= 16) launch_bwd_mp<1>(proto, grid, s, p, sync);
    else launch_bwd_mp<2>(proto, grid, s, p, sync);
    BIGDL_CHECK_LAUNCH();
  }
  if (lstm_persist_ok(B, H)) {
    if (!acts || !tcs || !cs || !a16(Ut) || !a8(gy) || !a8(DG) || !a16(acts) || !a16(tcs) || !a16(cs) || !a16(gc) ||
        (c0 && !a16(c0)))
      return (int)hipErrorInvalidValue;
    LstmSeqP p{};
    p.u = (const bf16_t*)Ut; p.acts = (float*)acts; p.tcs = (float*)tcs; p.cs = (float*)cs; p.c0 = c0;
    p.gy = (const bf16_t*)gy; p.dg = (bf16_t*)DG; p.gc = gc; p.B = B; p.T = T; p.H = H;
    if (B <= 16) hipLaunchKernelGGL(k_lstm_seq_bwd_p<1>, dim3(1), dim3(1024), 0, s, p);
    else hipLaunchKernelGGL(k_lstm_seq_bwd_p<2>, dim3(1), dim3(1024), 0, s, p);
    BIGDL_CHECK_LAUNCH();
  }
  return lstm_bwd_steps(gy, Ut, acts, tcs, cs, c0, DG, gc, B, T, H, 0, s);
}

BIGDL_EXPORT int bigdl_lstm_seq_bwd32(const float* gy, const float* Ut, const float* acts, const float* tcs,
                                      const float* cs, const float* c0, float* DG, float* gc, int B, int T, int H,
                                      hipStream_t s) {
  if (B <= 0 || T <= 0 || H <= 0 || !gy || !Ut || !DG || !gc || !acts || !tcs || !cs) return (int)hipErrorInvalidValue;
  return lstm_bwd_steps(gy, Ut, acts, tcs, cs, c0, DG, gc, B, T, H, 1, s);
}

// ------------------------------------------------------------------------------------------------
// Two stacked LSTM layers on the layer wavefront (k_rnn_step_pair): layer 1's gates are
// b1 + h0_t·W1ᵀ + h1_{t-1}·U1ᵀ, the input product folded into the recurrent step as a second
// reduction segment, so layer 1 runs step t−1 in the same launch as layer 0's step t and the whole
// two-layer sequence is T + 1 dependent launches (2T + an input-projection GEMM layer by layer).
// Backward mirrors it: layer 0's dh_t = dg0_{t+1}·U0 + dg1_t·W1 in one step.  Layouts as the
// single-layer launchers; b1 fp32 [4H1]; W1 [4H1][H0] (forward) / W1ᵀ [H0][4H1] (backward).
// ------------------------------------------------------------------------------------------------
static dim3 pair_grid(int H0, int H1, int B) {
  const int hs = H0 > H1 ? H0 : H1;
  return rnn_step_grid(hs, B, 2);
}

BIGDL_EXPORT int bigdl_lstm2_seq_fwd(const void* x2, int x_f32, const void* h00, const float* c00, const void* U0,
                                     void* out0, float* cs0, float* acts0, float* tcs0, float* cbuf0, const float* b1,
                                     const void* W1, const void* h01, const float* c01, const void* U1, void* out1,
                                     float* cs1, float* acts1, float* tcs1, float* cbuf1, int B, int T, int H0,
                                     int H1, hipStream_t s) {
  if (B <= 0 || T <= 0 || H0 <= 0 || H1 <= 0 || !x2 || !h00 || !U0 || !out0 || !b1 || !W1 || !h01 || !U1 || !out1)
    return (int)hipErrorInvalidValue;
  const bool train = cs0 && acts0 && tcs0 && cs1 && acts1 && tcs1;
  if (!train && (!cbuf0 || !cbuf1)) return (int)hipErrorInvalidValue;
  const long long G0 = 4LL * H0, G1 = 4LL * H1, BH0 = (long long)B * H0, BH1 = (long long)B * H1;
  const int esz = x_f32 ? 4 : 2;
  const dim3 grid = pair_grid(H0, H1, B), block(64 * kStepWaves);
  for (int w = 0; w <= T; ++w) {
    RnnStep q0{}, q1{};
    int live = 0;
    if (w < T) {  // layer 0, step t = w (the single-layer step)
      const int t = w;
      q0.a = t == 0 ? (const bf16_t*)h00 : (const bf16_t*)out0 + (long long)(t - 1) * H0;
      q0.lda = t == 0 ? H0 : (long long)T * H0;
      q0.u = (const bf16_t*)U0; q0.M = B; q0.K = H0; q0.Hs = H0;
      q0.xg = (const char*)x2 + (long long)t * G0 * esz; q0.ldx = (long long)T * G0; q0.x_f32 = x_f32;
      q0.c_prev = t == 0 ? c00 : (train ? cs0 + (t - 1) * BH0 : cbuf0 + ((t - 1) & 1) * BH0);
      q0.h_out = (bf16_t*)out0 + (long long)t * H0; q0.ldho = (long long)T * H0;
      q0.c_out = train ? cs0 + t * BH0 : cbuf0 + (t & 1) * BH0;
      q0.act = train ? acts0 + t * B * G0 : nullptr;
      q0.tc = train ? tcs0 + t * BH0 : nullptr;
      const int rc = rnn_step_check(0, q0);
      if (rc) return rc;
      live |= 1;
    }
    if (w >= 1) {  // layer 1, step t = w − 1: recurrent segment h1_{t-1}·U1ᵀ + input segment h0_t·W1ᵀ + b1
      const int t = w - 1;
      q1.a = t == 0 ? (const bf16_t*)h01 : (const bf16_t*)out1 + (long long)(t - 1) * H1;
      q1.lda = t == 0 ? H1 : (long long)T * H1;
      q1.u = (const bf16_t*)U1; q1.M = B; q1.K = H1; q1.Hs = H1;
      q1.a2 = (const bf16_t*)out0 + (long long)t * H0; q1.lda2 = (long long)T * H0;
      q1.u2 = (const bf16_t*)W1; q1.K2 = H0;
      q1.xg = b1; q1.ldx = 0; q1.x_f32 = 1;  // the bias row, broadcast over the batch
      q1.c_prev = t == 0 ? c01 : (train ? cs1 + (t - 1) * BH1 : cbuf1 + ((t - 1) & 1) * BH1);
      q1.h_out = (bf16_t*)out1 + (long long)t * H1; q1.ldho = (long long)T * H1;
      q1.c_out = train ? cs1 + t * BH1 : cbuf1 + (t & 1) * BH1;
      q1.act = train ? acts1 + t * B * G1 : nullptr;
      q1.tc = train ? tcs1 + t * BH1 : nullptr;
      const int rc = rnn_step_check(0, q1);
      if (rc) return rc;
      live |= 2;
    }
    hipLaunchKernelGGL((k_rnn_step_pair<0, 4>), grid, block, 0, s, q0, q1, live);
  }
  BIGDL_CHECK_LAUNCH();
}

BIGDL_EXPORT int bigdl_lstm2_seq_bwd(const void* gy1, const void* U1t, const float* acts1, const float* tcs1,
                                     const float* cs1, const float* c01, void* DG1, float* gc1, const void* U0t,
                                     const void* W1t, const float* acts0, const float* tcs0, const float* cs0,
                                     const float* c00, void* DG0, float* gc0, int B, int T, int H0, int H1,
                                     hipStream_t s) {
  if (B <= 0 || T <= 0 || H0 <= 0 || H1 <= 0 || !gy1 || !U1t || !DG1 || !gc1 || !U0t || !W1t || !DG0 || !gc0 ||
      !acts1 || !tcs1 || !cs1 || !acts0 || !tcs0 || !cs0)
    return (int)hipErrorInvalidValue;
  const long long G0 = 4LL * H0, G1 = 4LL * H1, BH0 = (long long)B * H0, BH1 = (long long)B * H1;
  const dim3 grid = pair_grid(H0, H1, B), block(64 * kStepWaves);
  for (int w = 0; w <= T; ++w) {
    RnnStep q0{}, q1{};
    int live = 0;
    const int t1 = T - 1 - w, t0 = T - w;
    if (t1 >= 0) {  // layer 1, step t1 (the single-layer backward step)
      const bool last = t1 + 1 == T;
      q1.a = last ? nullptr : (const bf16_t*)DG1 + (t1 + 1) * G1; q1.lda = (long long)T * G1;
      q1.u = (const bf16_t*)U1t; q1.M = B; q1.K = (int)G1; q1.Hs = H1;
      q1.c_prev = t1 > 0 ? cs1 + (t1 - 1) * BH1 : c01;
      q1.act = (float*)acts1 + t1 * B * G1; q1.tc = (float*)tcs1 + t1 * BH1;
      q1.gy = (const bf16_t*)gy1 + (long long)t1 * H1; q1.ldgy = (long long)T * H1;
      q1.gc_next = last ? nullptr : gc1;
      q1.dg = (bf16_t*)DG1 + t1 * G1; q1.lddg = (long long)T * G1; q1.dc_prev = gc1;
      const int rc = rnn_step_check(1, q1);
      if (rc) return rc;
      live |= 2;
    }
    if (t0 >= 0 && t0 < T) {  // layer 0, step t0: dh = dg0_{t0+1}·U0 + dg1_{t0}·W1 (no separate gy)
      const bool last = t0 + 1 == T;
      q0.a = last ? nullptr : (const bf16_t*)DG0 + (t0 + 1) * G0; q0.lda = (long long)T * G0;
      q0.u = (const bf16_t*)U0t; q0.M = B; q0.K = (int)G0; q0.Hs = H0;
      q0.a2 = (const bf16_t*)DG1 + t0 * G1; q0.lda2 = (long long)T * G1;
      q0.u2 = (const bf16_t*)W1t; q0.K2 = (int)G1;
      q0.c_prev = t0 > 0 ? cs0 + (t0 - 1) * BH0 : c00;
      q0.act = (float*)acts0 + t0 * B * G0; q0.tc = (float*)tcs0 + t0 * BH0;
      q0.gc_next = last ? nullptr : gc0;
      q0.dg = (bf16_t*)DG0 + t0 * G0; q0.lddg = (long long)T * G0; q0.dc_prev = gc0;
      const int rc = rnn_step_check(1, q0);
      if (rc) return rc;
      live |= 1;
    }
    hipLaunchKernelGGL((k_rnn_step_pair<1, 1>), grid, block, 0, s, q0, q1, live);
  }
  BIGDL_CHECK_LAUNCH();
}

// GRU: R, Z, Nn fp32 [S][B][H] and RH bf16 [B][S][H] with S = T (training) or 1 (inference: slot 0
// reused every step; Nn may be null)
static int gru_fwd_steps(const void* x2, int x_f32, const void* h0, const void* Urz, const void* Uh, void* out, float* R,
                         float* Z, float* Nn, void* RH, int train, int B, int T, int H, int f32, hipStream_t s) {
  const long long G = 3LL * H, BH = (long long)B * H;
  const int S = train ? T : 1;
  const int esz = x_f32 ? 4 : 2;
  for (int t = 0; t < T; ++t) {
    const int k = train ? t : 0;
    const void* hp = t == 0 ? h0 : eo((const void*)out, (long long)(t - 1) * H, f32);
    const long long ldhp = t == 0 ? H : (long long)T * H;
    const void* xg = (const char*)x2 + (long long)t * G * esz;
    void* rh = eo(RH, (long long)k * H, f32);
    int rc = rnn_step_run(2, hp, ldhp, Urz, B, H, H, xg, (long long)T * G, x_f32, hp, ldhp, nullptr, nullptr, 0, nullptr,
                          nullptr, nullptr, nullptr, 0, nullptr, nullptr, 0, nullptr, R + k * BH, Z + k * BH, nullptr,
                          rh, (long long)S * H, f32, s);
    if (rc) return rc;
    rc = rnn_step_run(3, rh, (long long)S * H, Uh, B, H, H, xg, (long long)T * G, x_f32, hp, ldhp, nullptr,
                      eo(out, (long long)t * H, f32), (long long)T * H, nullptr, nullptr, nullptr, nullptr, 0, nullptr,
                      nullptr, 0, nullptr, nullptr, Z + k * BH, (train && Nn) ? Nn + k * BH : nullptr, nullptr, 0, f32, s);
    if (rc) return rc;
  }
  return 0;
}

BIGDL_EXPORT int bigdl_gru_seq_fwd(const void* x2, int x_f32, const void* h0, const void* Urz, const void* Uh, void* out,
                                   float* R, float* Z, float* Nn, void* RH, int train, int B, int T, int H,
                                   hipStream_t s) {
  if (B <= 0 || T <= 0 || H <= 0 || !x2 || !h0 || !Urz || !Uh || !out || !R || !Z || !RH) return (int)hipErrorInvalidValue;
  return gru_fwd_steps(x2, x_f32, h0, Urz, Uh, out, R, Z, Nn, RH, train, B, T, H, 0, s);
}

// All-fp32 GRU (bf16x3 recurrent products): x2, h0, Urz, Uh, out, RH fp32.
BIGDL_EXPORT int bigdl_gru_seq_fwd32(const float* x2, const float* h0, const float* Urz, const float* Uh, float* out,
                                     float* R, float* Z, float* Nn, float* RH, int train, int B, int T, int H,
                                     hipStream_t s) {
  if (B <= 0 || T <= 0 || H <= 0 || !x2 || !h0 || !Urz || !Uh || !out || !R || !Z || !RH) return (int)hipErrorInvalidValue;
  return gru_fwd_steps(x2, 1, h0, Urz, Uh, out, R, Z, Nn, RH, train, B, T, H, 1, s);
}

static int gru_bwd_steps(const void* gy, const void* Urz_t, const void* Uh_t, const float* R, const float* Z,
                         const float* Nn, const void* out, const void* h0, void* DG, float* carry, int B, int T, int H,
                         int f32, hipStream_t s) {
  const long long G = 3LL * H, BH = (long long)B * H;
  for (int t = T - 1; t >= 0; --t) {
    const bool last = t + 1 == T;
    const void* hp = t == 0 ? h0 : eo(out, (long long)(t - 1) * H, f32);
    const long long ldhp = t == 0 ? H : (long long)T * H;
    void* dg = eo(DG, t * G, f32);
    int rc = rnn_step_run(4, last ? nullptr : eo((const void*)DG, (t + 1) * G, f32), (long long)T * G, Urz_t, B, 2 * H, H,
                          nullptr, 0, 0, hp, ldhp, nullptr, nullptr, 0, nullptr, nullptr, nullptr,
                          eo(gy, (long long)t * H, f32), (long long)T * H, nullptr, dg, (long long)T * G, nullptr, carry,
                          (float*)Z + t * BH, (float*)Nn + t * BH, nullptr, 0, f32, s);
    if (rc) return rc;
    rc = rnn_step_run(5, eo((const void*)dg, 2 * H, f32), (long long)T * G, Uh_t, B, H, H, nullptr, 0, 0, hp, ldhp,
                      nullptr, nullptr, 0, nullptr, nullptr, nullptr, nullptr, 0, nullptr, dg, (long long)T * G, nullptr,
                      carry, (float*)R + t * BH, nullptr, nullptr, 0, f32, s);
    if (rc) return rc;
  }
  return 0;
}

BIGDL_EXPORT int bigdl_gru_seq_bwd(const void* gy, const void* Urz_t, const void* Uh_t, const float* R, const float* Z,
                                   const float* Nn, const void* out, const void* h0, void* DG, float* carry, int B, int T,
                                   int H, hipStream_t s) {
  if (B <= 0 || T <= 0 || H <= 0 || !gy || !Urz_t || !Uh_t || !R || !Z || !Nn || !out || !h0 || !DG || !carry)
    return (int)hipErrorInvalidValue;
  return gru_bwd_steps(gy, Urz_t, Uh_t, R, Z, Nn, out, h0, DG, carry, B, T, H, 0, s);
}

BIGDL_EXPORT int bigdl_gru_seq_bwd32(const float* gy, const float* Urz_t, const float* Uh_t, const float* R,
                                     const float* Z, const float* Nn, const float* out, const float* h0, float* DG,
                                     float* carry, int B, int T, int H, hipStream_t s) {
  if (B <= 0 || T <= 0 || H <= 0 || !gy || !Urz_t || !Uh_t || !R || !Z || !Nn || !out || !h0 || !DG || !carry)
    return (int)hipErrorInvalidValue;
  return gru_bwd_steps(gy, Urz_t, Uh_t, R, Z, Nn, out, h0, DG, carry, B, T, H, 1, s);
}
