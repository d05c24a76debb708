// Cached incremental-decoding attention (Attention.updateOutputCache, DL/nn/Attention.scala:118-140,
// driven by SequenceBeamSearch / Transformer.symbols): a few new queries per sequence attend over a
// KV cache that grows by one position per decoding step.
//
// The cache lives in preallocated [rows][Lmax][ld] bf16 buffers (head h = columns h·D … h·D+D−1)
// that the caller appends to in place, so a step reads the first L positions and never copies
// the history (the reference concatenates [new; cache] every step).  That concatenation puts the
// NEWEST key first; a bias over keys is indexed in that order, so with ``bias_rev`` the kernel
// reads key position p's bias at logical index L−1−p.
//
// One workgroup per (row, head, query): 4 waves split the L keys into contiguous chunks.  A wave
// takes 64 keys at a time, one key per lane — the score q·k is a per-lane dot product over D (q is
// broadcast from LDS), so the online-softmax max / sum are wave reductions — and then accumulates
// o[d] += p_j·v_j[d] with lane = d (p_j broadcast through LDS, each v row read coalesced).  The
// four waves' (m, l, o) are merged through LDS at the end.  Decode is latency / bandwidth bound:
// no MFMA (a 1 × L × D product per head), every load is 16 B per lane where the layout allows.
#include "common.h"

constexpr int kDecWaves = 4;
constexpr int kDecMaxD = 256;

struct DecParams {
  const bf16_t* q;   // [rows·Lq][ldq]
  const bf16_t* k;   // [rows][Lmax][ldk]   (row stride sk = Lmax·ldk)
  const bf16_t* v;
  bf16_t* out;       // [rows·Lq][ldo]
  const float* bias; // optional, element (row, h, qi, j) at row·sbb + h·sbh + qi·sbq + j·sbk
  long long ldq, ldk, ldv, ldo, skr, svr;
  long long sbb, sbh, sbq, sbk;
  int rows, Hh, Lq, L, D, bias_rev;
  float scale;
};

template <int DPL>  // output dims per lane (D ≤ 64·DPL)
__global__ void __launch_bounds__(64 * kDecWaves) k_attn_decode(DecParams p) {
  __shared__ float qs[kDecMaxD];
  __shared__ float ps[kDecWaves][64];
  __shared__ float ws_m[kDecWaves], ws_l[kDecWaves];
  __shared__ float ws_o[kDecWaves][kDecMaxD];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int h = blockIdx.y, qi = blockIdx.z;
  const int row = blockIdx.x;
  const int D = p.D;
  const bf16_t* qrow = p.q + ((long long)row * p.Lq + qi) * p.ldq + (long long)h * D;
  for (int d = threadIdx.x; d < D; d += 64 * kDecWaves) qs[d] = bf2f(qrow[d]) * p.scale;
  __syncthreads();
  const bf16_t* kb = p.k + (long long)row * p.skr + (long long)h * D;
  const bf16_t* vb = p.v + (long long)row * p.svr + (long long)h * D;
  const float* brow = p.bias ? p.bias + row * p.sbb + h * p.sbh + qi * p.sbq : nullptr;
  const int chunk = (p.L + kDecWaves - 1) / kDecWaves;
  const int j0 = wv * chunk, j1 = min(p.L, j0 + chunk);
  float m = -INFINITY, l = 0.f;
  float o[DPL];
#pragma unroll
  for (int e = 0; e < DPL; ++e) o[e] = 0.f;
  for (int base = j0; base < j1; base += 64) {
    const int j = base + lane;
    float s = -INFINITY;
    if (j < j1) {
      const bf16_t* kr = kb + (long long)j * p.ldk;
      float acc = 0.f;
      for (int d = 0; d < D; d += 8) {
        float kv[8];
        load8(kr + d, kv);
#pragma unroll
        for (int e = 0; e < 8; ++e) acc = fmaf(qs[d + e], kv[e], acc);
      }
      if (brow) acc += brow[(long long)(p.bias_rev ? p.L - 1 - j : j) * p.sbk];
      s = acc;
    }
    const float mt = wave_max(s);
    const float mn = fmaxf(m, mt);
    // every key of this tile masked to −∞ (and nothing before): keep the state as is
    const float alpha = (mn == -INFINITY) ? 1.f : __expf(m - mn);
    const float pj = (s == -INFINITY) ? 0.f : __expf(s - mn);
    l = l * alpha + wave_sum(pj);
#pragma unroll
    for (int e = 0; e < DPL; ++e) o[e] *= alpha;
    m = mn;
    ps[wv][lane] = pj;
    __builtin_amdgcn_wave_barrier();
    const int nj = min(64, j1 - base);
    for (int t = 0; t < nj; ++t) {
      const float w = ps[wv][t];
      const bf16_t* vr = vb + (long long)(base + t) * p.ldv;
#pragma unroll
      for (int e = 0; e < DPL; ++e) {
        const int d = lane + 64 * e;
        if (d < D) o[e] = fmaf(w, bf2f(vr[d]), o[e]);
      }
    }
    __builtin_amdgcn_wave_barrier();
  }
  if (lane == 0) {
    ws_m[wv] = m;
    ws_l[wv] = l;
  }
#pragma unroll
  for (int e = 0; e < DPL; ++e) {
    const int d = lane + 64 * e;
    if (d < D) ws_o[wv][d] = o[e];
  }
  __syncthreads();
  if (wv != 0) return;
  float M = -INFINITY;
#pragma unroll
  for (int w = 0; w < kDecWaves; ++w) M = fmaxf(M, ws_m[w]);
  float Lsum = 0.f, f[kDecWaves];
#pragma unroll
  for (int w = 0; w < kDecWaves; ++w) {
    f[w] = (ws_m[w] == -INFINITY) ? 0.f : __expf(ws_m[w] - M);
    Lsum += ws_l[w] * f[w];
  }
  const float inv = Lsum > 0.f ? 1.f / Lsum : 0.f;
  bf16_t* orow = p.out + ((long long)row * p.Lq + qi) * p.ldo + (long long)h * D;
#pragma unroll
  for (int e = 0; e < DPL; ++e) {
    const int d = lane + 64 * e;
    if (d < D) {
      float acc = 0.f;
#pragma unroll
      for (int w = 0; w < kDecWaves; ++w) acc = fmaf(ws_o[w][d], f[w], acc);
      orow[d] = f2bf(acc * inv);
    }
  }
}

// o[row, qi, h·D + d] = softmax_j(scale·q·k_j + bias) · v_j over the first L cached positions.
// q/out: [rows·Lq][ld] bf16; k/v: [rows][*][ld] bf16 with per-row stride skr/svr elements; D % 8 == 0,
// D ≤ 256; q, k, v 16-B aligned with ldq/ldk % 8 == 0 (16-B key-row loads).
BIGDL_EXPORT int bigdl_attn_decode(const void* q, long long ldq, const void* k, long long ldk, long long skr,
                                   const void* v, long long ldv, long long svr, void* out, long long ldo,
                                   const float* bias, long long sbb, long long sbh, long long sbq, long long sbk,
                                   int bias_rev, int rows, int Hh, int Lq, int L, int D, float scale, hipStream_t s) {
  if (!q || !k || !v || !out || rows <= 0 || Hh <= 0 || Lq <= 0 || L <= 0 || D <= 0 || D % 8 || D > kDecMaxD)
    return (int)hipErrorInvalidValue;
  if (((uintptr_t)q & 15) || ((uintptr_t)k & 15) || ldq % 8 || ldk % 8 || skr % 8)
    return (int)hipErrorInvalidValue;
  const long long hd = (long long)Hh * D;
  if (ldq < hd || ldk < hd || ldv < hd || ldo < hd || skr < (long long)L * ldk || svr < (long long)L * ldv)
    return (int)hipErrorInvalidValue;
  if (rows > 0x7fffffff || Hh > 65535 || Lq > 65535) return (int)hipErrorInvalidValue;
  DecParams p{};
  p.q = (const bf16_t*)q; p.k = (const bf16_t*)k; p.v = (const bf16_t*)v; p.out = (bf16_t*)out;
  p.bias = bias; p.ldq = ldq; p.ldk = ldk; p.ldv = ldv; p.ldo = ldo; p.skr = skr; p.svr = svr;
  p.sbb = sbb; p.sbh = sbh; p.sbq = sbq; p.sbk = sbk;
  p.rows = rows; p.Hh = Hh; p.Lq = Lq; p.L = L; p.D = D; p.bias_rev = bias_rev; p.scale = scale;
  const dim3 grid((unsigned)rows, (unsigned)Hh, (unsigned)Lq);
  if (D <= 64) hipLaunchKernelGGL(k_attn_decode<1>, grid, dim3(64 * kDecWaves), 0, s, p);
  else if (D <= 128) hipLaunchKernelGGL(k_attn_decode<2>, grid, dim3(64 * kDecWaves), 0, s, p);
  else hipLaunchKernelGGL(k_attn_decode<4>, grid, dim3(64 * kDecWaves), 0, s, p);
  BIGDL_CHECK_LAUNCH();
}
