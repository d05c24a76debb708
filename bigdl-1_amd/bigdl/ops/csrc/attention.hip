// Fused multi-head attention on MFMA (flash-style: the Lq × Lk score matrix never reaches HBM).
// Reference: Attention.scala:30-111 (q·depth^-0.5, QKᵀ + bias → softmax → dropout → ·V, split /
// combine heads) — here one kernel reads Q/K/V straight out of the projection GEMM's [B·L][ld]
// rows (head h = columns h·D … h·D+D−1, so split_heads / combine_heads are addressing, not copies)
// and writes O in the same layout for the output projection.
//
// Forward, per workgroup (4 waves) 64 queries of one (batch, head); per wave 16 queries:
//   Sᵀ = K·Qᵀ with mfma_f32_16x16x32_bf16, the KEY on the MFMA row and the QUERY on the lane
//   (A = K rows from LDS, B = Q fragments held in registers for the whole pass), so a lane owns
//   one query's scores: the online-softmax max needs two lane swaps (the 4 lane groups of a
//   query), the row sum none until the end.  The Sᵀ accumulators ARE the B operand of
//   Oᵀ += Vᵀ·Pᵀ (an accumulator summed over its row index needs no lane movement,
//   cdna_hip_programming.md §3); the matching permuted-k A operand Vᵀ comes from the row-major V
//   tile through ds_read_b64_tr_b16 (T10).  K/V tiles: 64 keys, global → registers issued before
//   the tile's MFMAs, written to LDS after the next barrier (T14).
// Scores are kept in the log2 domain (x = S·scale·log2e + bias·log2e, p = exp2(x − m)), the
// forward stores LSE₂ = m + log2 Σp per query for the backward.
//
// Backward (recompute P from Q, K and LSE₂; δ = rowsum(dO ∘ O)):
//   k_attn_bwd_dq   query on the lane (the forward's structure): Sᵀ = K·Qᵀ, dPᵀ = V·dOᵀ,
//                   dSᵀ = Pᵀ∘(dPᵀ·m − δ), dQᵀ += Kᵀ·dSᵀ; it also writes δ.
//   k_attn_bwd_dkdv key on the lane: S = Q·Kᵀ, dP = dO·Vᵀ (K, V fragments in registers, Q / dO
//                   tiles in LDS), dVᵀ += dOᵀ·(P∘m), dKᵀ += Qᵀ·dS — dK and dV summed inside one
//                   workgroup, so the backward needs no atomics and is bitwise reproducible.
//
// Masks: an optional additive fp32 bias with broadcast strides (padding / arbitrary masks), an
// in-kernel causal mask (key > query → −∞; key tiles past the diagonal are skipped), keys ≥ Lk.
// Attention dropout: keep bit = hash(seed, batch·heads + head, query, key) < keep·2³², the same
// function in the backward (and in ops/reference.py::attention_dropout_mask for tests); kept
// probabilities are scaled by 1/keep, the softmax normaliser is taken before dropout (the
// reference's softmax → Dropout order).
#include "common.h"

typedef short v8s __attribute__((ext_vector_type(8)));
typedef short v4s __attribute__((ext_vector_type(4)));
typedef float v4f __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) v4s lds_v4s;

struct AttnParams {
  const bf16_t* q;
  const bf16_t* k;
  const bf16_t* v;
  const bf16_t* o;     // backward: forward output
  const bf16_t* dout;  // backward: output gradient
  bf16_t* out;         // forward: O; backward: dQ
  bf16_t* dk;
  bf16_t* dv;
  float* lse;          // [B][Hh][Lq] log2-domain log-sum-exp
  float* delta;        // [B][Hh][Lq] rowsum(dO ∘ O)
  const float* bias;   // optional additive bias, element (b, h, q, k) at b·sbb + h·sbh + q·sbq + k·sbk
  long long sbb, sbh, sbq, sbk;
  long long ldq, ldk, ldv, ldo, ldd, ldg, ldgk, ldgv;  // row strides (elements)
  int B, Hh, Lq, Lk;
  float scale;       // softmax scale (depth^-0.5)
  float scale_log2;  // scale · log2(e)
  int causal;
  int dropout;
  uint32_t keep_thr;
  float inv_keep;
  uint32_t seed;
  const uint32_t* seed_dev;  // optional device seed (HIP-graph capture: low word of an int64 counter)
  int bias_vec;  // bias rows contiguous along keys, 16-B aligned: float4 loads
};

constexpr float kLog2e = 1.4426950408889634f;

__device__ __forceinline__ uint32_t amix(uint32_t x) {
  x ^= x >> 16;
  x *= 0x7feb352du;
  x ^= x >> 15;
  x *= 0x846ca68bu;
  x ^= x >> 16;
  return x;
}

__device__ __forceinline__ uint32_t bh_seed(const AttnParams& p, int b, int h) {
  const uint32_t s = p.seed_dev ? p.seed_dev[0] : p.seed;
  return amix(s + (uint32_t)(b * p.Hh + h) * 0x85EBCA77u);
}

// dropout keep bit of (query, key) under a (batch, head) seed
__device__ __forceinline__ bool akeep(uint32_t s, int q, int k, uint32_t thr) {
  return amix(s ^ amix((uint32_t)q * 0x9E3779B1u + (uint32_t)k)) < thr;
}

__device__ __forceinline__ void bias4(const AttnParams& p, long long row, int key, float (&o)[4]) {
  if (p.bias_vec && key + 3 < p.Lk) {
    const float4 f = *reinterpret_cast<const float4*>(p.bias + row + key);
    o[0] = f.x; o[1] = f.y; o[2] = f.z; o[3] = f.w;
    return;
  }
#pragma unroll
  for (int e = 0; e < 4; ++e) o[e] = key + e < p.Lk ? p.bias[row + (long long)(key + e) * p.sbk] : 0.f;
}

__device__ __forceinline__ short bfs(float f) { return (short)f2bf(f); }

// 64 rows × D of a [rows][ld] bf16 matrix → registers (rows ≥ nvalid read as zero)
template <int D>
__device__ __forceinline__ void ld_rows(const bf16_t* base, long long ld, int row0, int nvalid,
                                        uint4 (&r)[D / 32]) {
  constexpr int CPR = D / 8;
#pragma unroll
  for (int i = 0; i < D / 32; ++i) {
    const int c = threadIdx.x + 256 * i;
    const int row = c / CPR, col = (c % CPR) * 8;
    r[i] = row0 + row < nvalid ? *reinterpret_cast<const uint4*>(base + (long long)(row0 + row) * ld + col)
                               : make_uint4(0u, 0u, 0u, 0u);
  }
}

// registers → LDS tile [64][D + 8] (the 16-B row pad puts the 16 rows of a fragment read on 16
// distinct bank slots)
template <int D>
__device__ __forceinline__ void st_rows(bf16_t* lds, const uint4 (&r)[D / 32]) {
  constexpr int CPR = D / 8;
#pragma unroll
  for (int i = 0; i < D / 32; ++i) {
    const int c = threadIdx.x + 256 * i;
    const int row = c / CPR, col = (c % CPR) * 8;
    *reinterpret_cast<uint4*>(&lds[row * (D + 8) + col]) = r[i];
  }
}

// A fragment of Xᵀ (X = an LDS tile [rows][cols], ld LD) for an MFMA whose k index runs over X's
// rows in the accumulator-operand order: element j < 4 ↔ row rA + j, j ≥ 4 ↔ row rB + j − 4 (per
// 16-lane group), MFMA row ↔ column c0 + (lane & 15).  Two ds_read_b64_tr_b16: lane 4q + p of a
// group addresses row r0 + q, columns c0 + 4p … c0 + 4p + 3 and receives column c0 + lane of the
// four rows.
template <int LD>
__device__ __forceinline__ v8s tr_frag(const bf16_t* img, int rA, int rB, int c0) {
  const int i = threadIdx.x & 15;
  const int off = (i >> 2) * LD + c0 + 4 * (i & 3);
  const v4s lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4s*)(img + rA * LD + off));
  const v4s hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4s*)(img + rB * LD + off));
  return v8s{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
}

__device__ __forceinline__ v8s pack8(const v4f& a, const v4f& b) {
  return v8s{bfs(a[0]), bfs(a[1]), bfs(a[2]), bfs(a[3]), bfs(b[0]), bfs(b[1]), bfs(b[2]), bfs(b[3])};
}

__device__ __forceinline__ void store4(bf16_t* dst, const v4f& v, float s) {
  const uint32_t lo = (uint32_t)f2bf(v[0] * s) | ((uint32_t)f2bf(v[1] * s) << 16);
  const uint32_t hi = (uint32_t)f2bf(v[2] * s) | ((uint32_t)f2bf(v[3] * s) << 16);
  *reinterpret_cast<uint2*>(dst) = make_uint2(lo, hi);
}

// ------------------------------------------------------------------------------------------ forward
template <int D>
__global__ void __launch_bounds__(256) k_attn_fwd(AttnParams p) {
  constexpr int LD = D + 8, KS = D / 32, DT = D / 16;
  __shared__ __attribute__((aligned(16))) bf16_t ks[64 * LD];
  __shared__ __attribute__((aligned(16))) bf16_t vs[64 * LD];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, fr = lane & 15, g = lane >> 4;
  const int b = blockIdx.z, h = blockIdx.y, q0 = blockIdx.x * 64;
  const int qi = q0 + 16 * w + fr;
  const bool qok = qi < p.Lq;
  const bf16_t* kb = p.k + (long long)b * p.Lk * p.ldk + h * D;
  const bf16_t* vb = p.v + (long long)b * p.Lk * p.ldv + h * D;
  v8s qf[KS];
  {
    const bf16_t* qr = p.q + ((long long)b * p.Lq + (qok ? qi : 0)) * p.ldq + h * D + 8 * g;
#pragma unroll
    for (int s = 0; s < KS; ++s) qf[s] = qok ? *reinterpret_cast<const v8s*>(qr + 32 * s) : v8s{0, 0, 0, 0, 0, 0, 0, 0};
  }
  const uint32_t sd = bh_seed(p, b, h);
  const long long brow = (long long)b * p.sbb + (long long)h * p.sbh + (long long)(qok ? qi : 0) * p.sbq;
  int nkt = (p.Lk + 63) / 64;
  if (p.causal) nkt = min(nkt, q0 / 64 + 1);
  float m = -INFINITY, l = 0.f;
  v4f acc[DT];
#pragma unroll
  for (int i = 0; i < DT; ++i) acc[i] = v4f{0.f, 0.f, 0.f, 0.f};
  uint4 kr[D / 32], vr[D / 32];
  ld_rows<D>(kb, p.ldk, 0, p.Lk, kr);
  ld_rows<D>(vb, p.ldv, 0, p.Lk, vr);
  for (int kt = 0; kt < nkt; ++kt) {
    __syncthreads();  // every wave is done reading the previous tile
    st_rows<D>(ks, kr);
    st_rows<D>(vs, vr);
    __syncthreads();
    if (kt + 1 < nkt) {  // next tile's loads fly under this tile's MFMAs
      ld_rows<D>(kb, p.ldk, (kt + 1) * 64, p.Lk, kr);
      ld_rows<D>(vb, p.ldv, (kt + 1) * 64, p.Lk, vr);
    }
    v4f s[4];
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      s[t] = v4f{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int ss = 0; ss < KS; ++ss) {
        const v8s a = *reinterpret_cast<const v8s*>(&ks[(16 * t + fr) * LD + 32 * ss + 8 * g]);
        s[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, qf[ss], s[t], 0, 0, 0);
      }
    }
    // lane: scores of query qi against keys kt·64 + 16t + 4g + r
    float tmax = -INFINITY;
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      const int key0 = kt * 64 + 16 * t + 4 * g;
      float bv[4] = {0.f, 0.f, 0.f, 0.f};
      if (p.bias) bias4(p, brow, key0, bv);
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int key = key0 + r;
        float x = fmaf(s[t][r], p.scale_log2, bv[r] * kLog2e);
        if (key >= p.Lk || (p.causal && key > qi)) x = -INFINITY;
        s[t][r] = x;
        tmax = fmaxf(tmax, x);
      }
    }
    tmax = fmaxf(tmax, __shfl_xor(tmax, 16, 64));
    tmax = fmaxf(tmax, __shfl_xor(tmax, 32, 64));
    const float mn = fmaxf(m, tmax);
    const float mu = mn == -INFINITY ? 0.f : mn;
    const float alpha = exp2f(m - mu);
    m = mn;
    l *= alpha;
#pragma unroll
    for (int i = 0; i < DT; ++i) acc[i] *= alpha;
#pragma unroll
    for (int t = 0; t < 4; ++t) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        float e = exp2f(s[t][r] - mu);
        l += e;
        if (p.dropout) e = akeep(sd, qi, kt * 64 + 16 * t + 4 * g + r, p.keep_thr) ? e * p.inv_keep : 0.f;
        s[t][r] = e;
      }
    }
#pragma unroll
    for (int k2 = 0; k2 < 2; ++k2) {
      const v8s pf = pack8(s[2 * k2], s[2 * k2 + 1]);
#pragma unroll
      for (int dt = 0; dt < DT; ++dt) {
        const v8s a = tr_frag<LD>(vs, 32 * k2 + 4 * g, 32 * k2 + 16 + 4 * g, 16 * dt);
        acc[dt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, pf, acc[dt], 0, 0, 0);
      }
    }
  }
  l += __shfl_xor(l, 16, 64);
  l += __shfl_xor(l, 32, 64);
  if (qok) {
    const float inv = l > 0.f ? 1.f / l : 0.f;
    bf16_t* orow = p.out + ((long long)b * p.Lq + qi) * p.ldo + h * D + 4 * g;
#pragma unroll
    for (int dt = 0; dt < DT; ++dt) store4(orow + 16 * dt, acc[dt], inv);
    if (g == 0) p.lse[((long long)b * p.Hh + h) * p.Lq + qi] = l > 0.f ? m + log2f(l) : -INFINITY;
  }
}

// ------------------------------------------------------------------------------------ backward dQ
template <int D>
__global__ void __launch_bounds__(256) k_attn_bwd_dq(AttnParams p) {
  constexpr int LD = D + 8, KS = D / 32, DT = D / 16;
  __shared__ __attribute__((aligned(16))) bf16_t ks[64 * LD];
  __shared__ __attribute__((aligned(16))) bf16_t vs[64 * LD];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, fr = lane & 15, g = lane >> 4;
  const int b = blockIdx.z, h = blockIdx.y, q0 = blockIdx.x * 64;
  const int qi = q0 + 16 * w + fr;
  const bool qok = qi < p.Lq;
  const long long qrow = (long long)b * p.Lq + (qok ? qi : 0);
  const bf16_t* kb = p.k + (long long)b * p.Lk * p.ldk + h * D;
  const bf16_t* vb = p.v + (long long)b * p.Lk * p.ldv + h * D;
  v8s qf[KS], df[KS];
  float dl = 0.f;
#pragma unroll
  for (int s = 0; s < KS; ++s) {
    const v8s z = v8s{0, 0, 0, 0, 0, 0, 0, 0};
    qf[s] = qok ? *reinterpret_cast<const v8s*>(p.q + qrow * p.ldq + h * D + 32 * s + 8 * g) : z;
    df[s] = qok ? *reinterpret_cast<const v8s*>(p.dout + qrow * p.ldd + h * D + 32 * s + 8 * g) : z;
    const v8s of = qok ? *reinterpret_cast<const v8s*>(p.o + qrow * p.ldo + h * D + 32 * s + 8 * g) : z;
#pragma unroll
    for (int j = 0; j < 8; ++j) dl = fmaf(bf2f((bf16_t)df[s][j]), bf2f((bf16_t)of[j]), dl);
  }
  dl += __shfl_xor(dl, 16, 64);
  dl += __shfl_xor(dl, 32, 64);
  const long long sidx = ((long long)b * p.Hh + h) * p.Lq + (qok ? qi : 0);
  if (qok && g == 0) p.delta[sidx] = dl;
  const float lse = qok ? p.lse[sidx] : 0.f;
  const uint32_t sd = bh_seed(p, b, h);
  const long long brow = (long long)b * p.sbb + (long long)h * p.sbh + (long long)(qok ? qi : 0) * p.sbq;
  int nkt = (p.Lk + 63) / 64;
  if (p.causal) nkt = min(nkt, q0 / 64 + 1);
  v4f acc[DT];
#pragma unroll
  for (int i = 0; i < DT; ++i) acc[i] = v4f{0.f, 0.f, 0.f, 0.f};
  uint4 kr[D / 32], vr[D / 32];
  ld_rows<D>(kb, p.ldk, 0, p.Lk, kr);
  ld_rows<D>(vb, p.ldv, 0, p.Lk, vr);
  for (int kt = 0; kt < nkt; ++kt) {
    __syncthreads();
    st_rows<D>(ks, kr);
    st_rows<D>(vs, vr);
    __syncthreads();
    if (kt + 1 < nkt) {
      ld_rows<D>(kb, p.ldk, (kt + 1) * 64, p.Lk, kr);
      ld_rows<D>(vb, p.ldv, (kt + 1) * 64, p.Lk, vr);
    }
    v4f s[4], dp[4];
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      s[t] = v4f{0.f, 0.f, 0.f, 0.f};
      dp[t] = v4f{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int ss = 0; ss < KS; ++ss) {
        const v8s a = *reinterpret_cast<const v8s*>(&ks[(16 * t + fr) * LD + 32 * ss + 8 * g]);
        s[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, qf[ss], s[t], 0, 0, 0);
        const v8s c = *reinterpret_cast<const v8s*>(&vs[(16 * t + fr) * LD + 32 * ss + 8 * g]);
        dp[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(c, df[ss], dp[t], 0, 0, 0);
      }
    }
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      const int key0 = kt * 64 + 16 * t + 4 * g;
      float bv[4] = {0.f, 0.f, 0.f, 0.f};
      if (p.bias) bias4(p, brow, key0, bv);
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int key = key0 + r;
        const bool dead = key >= p.Lk || (p.causal && key > qi);
        const float pr = dead ? 0.f : exp2f(fmaf(s[t][r], p.scale_log2, bv[r] * kLog2e) - lse);
        float f = 1.f;
        if (p.dropout) f = akeep(sd, qi, key, p.keep_thr) ? p.inv_keep : 0.f;
        s[t][r] = pr * fmaf(dp[t][r], f, -dl);  // dS (natural-scale logits)
      }
    }
#pragma unroll
    for (int k2 = 0; k2 < 2; ++k2) {
      const v8s sf = pack8(s[2 * k2], s[2 * k2 + 1]);
#pragma unroll
      for (int dt = 0; dt < DT; ++dt) {
        const v8s a = tr_frag<LD>(ks, 32 * k2 + 4 * g, 32 * k2 + 16 + 4 * g, 16 * dt);
        acc[dt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, sf, acc[dt], 0, 0, 0);
      }
    }
  }
  if (qok) {
    bf16_t* grow = p.out + qrow * p.ldg + h * D + 4 * g;
#pragma unroll
    for (int dt = 0; dt < DT; ++dt) store4(grow + 16 * dt, acc[dt], p.scale);
  }
}

// --------------------------------------------------------------------------------- backward dK, dV
template <int D>
__global__ void __launch_bounds__(256) k_attn_bwd_dkdv(AttnParams p) {
  constexpr int LD = D + 8, KS = D / 32, DT = D / 16;
  __shared__ __attribute__((aligned(16))) bf16_t qs[64 * LD];
  __shared__ __attribute__((aligned(16))) bf16_t ds[64 * LD];
  __shared__ float lse_s[64], dl_s[64];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, fr = lane & 15, g = lane >> 4;
  const int b = blockIdx.z, h = blockIdx.y, k0 = blockIdx.x * 64;
  const int kj = k0 + 16 * w + fr;
  const bool kok = kj < p.Lk;
  const long long krow = (long long)b * p.Lk + (kok ? kj : 0);
  v8s kf[KS], vf[KS];
#pragma unroll
  for (int s = 0; s < KS; ++s) {
    const v8s z = v8s{0, 0, 0, 0, 0, 0, 0, 0};
    kf[s] = kok ? *reinterpret_cast<const v8s*>(p.k + krow * p.ldk + h * D + 32 * s + 8 * g) : z;
    vf[s] = kok ? *reinterpret_cast<const v8s*>(p.v + krow * p.ldv + h * D + 32 * s + 8 * g) : z;
  }
  const bf16_t* qb = p.q + (long long)b * p.Lq * p.ldq + h * D;
  const bf16_t* db = p.dout + (long long)b * p.Lq * p.ldd + h * D;
  const float* lseb = p.lse + ((long long)b * p.Hh + h) * p.Lq;
  const float* dlb = p.delta + ((long long)b * p.Hh + h) * p.Lq;
  const uint32_t sd = bh_seed(p, b, h);
  const long long bcol = (long long)b * p.sbb + (long long)h * p.sbh + (long long)(kok ? kj : 0) * p.sbk;
  const int nqt = (p.Lq + 63) / 64;
  const int qt0 = p.causal ? min(k0 / 64, nqt) : 0;
  v4f adk[DT], adv[DT];
#pragma unroll
  for (int i = 0; i < DT; ++i) {
    adk[i] = v4f{0.f, 0.f, 0.f, 0.f};
    adv[i] = v4f{0.f, 0.f, 0.f, 0.f};
  }
  uint4 qr[D / 32], dr[D / 32];
  // threads 0-63 carry the tile's LSE₂ values, 64-127 its δ values
  const float* sb = threadIdx.x < 64 ? lseb : dlb;
  const int si = threadIdx.x & 63;
  float sr = 0.f;
  if (qt0 < nqt) {
    ld_rows<D>(qb, p.ldq, qt0 * 64, p.Lq, qr);
    ld_rows<D>(db, p.ldd, qt0 * 64, p.Lq, dr);
    if (threadIdx.x < 128) sr = qt0 * 64 + si < p.Lq ? sb[qt0 * 64 + si] : 0.f;
  }
  for (int qt = qt0; qt < nqt; ++qt) {
    __syncthreads();
    st_rows<D>(qs, qr);
    st_rows<D>(ds, dr);
    if (threadIdx.x < 64) lse_s[si] = sr;
    else if (threadIdx.x < 128) dl_s[si] = sr;
    __syncthreads();
    if (qt + 1 < nqt) {
      ld_rows<D>(qb, p.ldq, (qt + 1) * 64, p.Lq, qr);
      ld_rows<D>(db, p.ldd, (qt + 1) * 64, p.Lq, dr);
      if (threadIdx.x < 128) sr = (qt + 1) * 64 + si < p.Lq ? sb[(qt + 1) * 64 + si] : 0.f;
    }
    v4f s[4], dp[4];
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      s[t] = v4f{0.f, 0.f, 0.f, 0.f};
      dp[t] = v4f{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int ss = 0; ss < KS; ++ss) {
        const v8s a = *reinterpret_cast<const v8s*>(&qs[(16 * t + fr) * LD + 32 * ss + 8 * g]);
        s[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, kf[ss], s[t], 0, 0, 0);
        const v8s c = *reinterpret_cast<const v8s*>(&ds[(16 * t + fr) * LD + 32 * ss + 8 * g]);
        dp[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(c, vf[ss], dp[t], 0, 0, 0);
      }
    }
    // lane: entries (query qt·64 + 16t + 4g + r, key kj); s ← P∘m (for dV), dp ← dS (for dK)
#pragma unroll
    for (int t = 0; t < 4; ++t) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int ql = 16 * t + 4 * g + r, qq = qt * 64 + ql;
        const bool dead = qq >= p.Lq || !kok || (p.causal && kj > qq);
        float bv = 0.f;
        if (p.bias && !dead) bv = p.bias[bcol + (long long)qq * p.sbq];
        const float pr = dead ? 0.f : exp2f(fmaf(s[t][r], p.scale_log2, bv * kLog2e) - lse_s[ql]);
        float f = 1.f;
        if (p.dropout) f = akeep(sd, qq, kj, p.keep_thr) ? p.inv_keep : 0.f;
        s[t][r] = pr * f;
        dp[t][r] = pr * fmaf(dp[t][r], f, -dl_s[ql]);
      }
    }
#pragma unroll
    for (int k2 = 0; k2 < 2; ++k2) {
      const v8s pf = pack8(s[2 * k2], s[2 * k2 + 1]);
      const v8s sf = pack8(dp[2 * k2], dp[2 * k2 + 1]);
#pragma unroll
      for (int dt = 0; dt < DT; ++dt) {
        const v8s ad = tr_frag<LD>(ds, 32 * k2 + 4 * g, 32 * k2 + 16 + 4 * g, 16 * dt);
        adv[dt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ad, pf, adv[dt], 0, 0, 0);
        const v8s aq = tr_frag<LD>(qs, 32 * k2 + 4 * g, 32 * k2 + 16 + 4 * g, 16 * dt);
        adk[dt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(aq, sf, adk[dt], 0, 0, 0);
      }
    }
  }
  if (kok) {
    bf16_t* dkr = p.dk + krow * p.ldgk + h * D + 4 * g;
    bf16_t* dvr = p.dv + krow * p.ldgv + h * D + 4 * g;
#pragma unroll
    for (int dt = 0; dt < DT; ++dt) {
      store4(dkr + 16 * dt, adk[dt], p.scale);
      store4(dvr + 16 * dt, adv[dt], 1.f);
    }
  }
}

// ------------------------------------------------------------------------------------------ host
static bool a16(const void* q) { return ((uintptr_t)q & 15) == 0; }

static int attn_setup(AttnParams& p, const void* q, long long ldq, const void* k, long long ldk, const void* v,
                      long long ldv, const float* bias, long long sbb, long long sbh, long long sbq, long long sbk,
                      int B, int Hh, int Lq, int Lk, int D, float scale, int causal, float keep, unsigned seed,
                      const void* seed_dev) {
  if (B <= 0 || Hh <= 0 || Lq <= 0 || Lk <= 0 || D <= 0 || D > 128 || D % 32) return (int)hipErrorInvalidValue;
  if (!a16(q) || !a16(k) || !a16(v) || ldq % 8 || ldk % 8 || ldv % 8) return (int)hipErrorInvalidValue;
  if (ldq < (long long)Hh * D || ldk < (long long)Hh * D || ldv < (long long)Hh * D) return (int)hipErrorInvalidValue;
  if (causal && Lq != Lk) return (int)hipErrorInvalidValue;
  if (!(keep > 0.f && keep <= 1.f)) return (int)hipErrorInvalidValue;
  if (B > 65535 || Hh > 65535) return (int)hipErrorInvalidValue;
  p.q = (const bf16_t*)q; p.k = (const bf16_t*)k; p.v = (const bf16_t*)v;
  p.ldq = ldq; p.ldk = ldk; p.ldv = ldv;
  p.bias = bias; p.sbb = sbb; p.sbh = sbh; p.sbq = sbq; p.sbk = sbk;
  p.bias_vec = bias && sbk == 1 && a16(bias) && sbb % 4 == 0 && sbh % 4 == 0 && sbq % 4 == 0;
  p.B = B; p.Hh = Hh; p.Lq = Lq; p.Lk = Lk;
  p.scale = scale;
  p.scale_log2 = scale * kLog2e;
  p.causal = causal;
  p.dropout = keep < 1.f;
  const double thr = (double)keep * 4294967296.0;
  p.keep_thr = thr >= 4294967295.0 ? 0xFFFFFFFFu : (uint32_t)thr;
  p.inv_keep = 1.f / keep;
  p.seed = seed;
  p.seed_dev = (const uint32_t*)seed_dev;
  return 0;
}

// O (and LSE₂, fp32 [B][Hh][Lq]) of softmax(scale·Q·Kᵀ + bias [+ causal]) ∘ dropout · V.
// q/k/v/out: [B·L][ld] bf16 rows, head h at columns h·D (16-B aligned, ld % 8 == 0), D ∈ {32, 64, 96, 128}.
BIGDL_EXPORT int bigdl_attn_fwd(const void* q, long long ldq, const void* k, long long ldk, const void* v,
                                long long ldv, void* out, long long ldo, float* lse, const float* bias, long long sbb,
                                long long sbh, long long sbq, long long sbk, int B, int Hh, int Lq, int Lk, int D,
                                float scale, int causal, float keep, unsigned seed, const void* seed_dev,
                                hipStream_t s) {
  AttnParams p{};
  int rc = attn_setup(p, q, ldq, k, ldk, v, ldv, bias, sbb, sbh, sbq, sbk, B, Hh, Lq, Lk, D, scale, causal, keep, seed,
                      seed_dev);
  if (rc) return rc;
  if (!a16(out) || ldo % 8 || ldo < (long long)Hh * D || !lse) return (int)hipErrorInvalidValue;
  p.out = (bf16_t*)out; p.ldo = ldo; p.lse = lse;
  const dim3 grid((unsigned)((Lq + 63) / 64), (unsigned)Hh, (unsigned)B);
  // head dims 32 / 64 / 96 / 128: every loop of the kernels runs over D / 32 k-slices and D / 16
  // output slices, and the [64][D + 8] LDS rows keep the 8-B alignment the transposed reads need
  switch (D) {
    case 32: hipLaunchKernelGGL(k_attn_fwd<32>, grid, dim3(256), 0, s, p); break;
    case 64: hipLaunchKernelGGL(k_attn_fwd<64>, grid, dim3(256), 0, s, p); break;
    case 96: hipLaunchKernelGGL(k_attn_fwd<96>, grid, dim3(256), 0, s, p); break;
    default: hipLaunchKernelGGL(k_attn_fwd<128>, grid, dim3(256), 0, s, p); break;
  }
  BIGDL_CHECK_LAUNCH();
}

// dQ, dK, dV (bf16, same row layout as q/k/v) from dO; delta: fp32 [B][Hh][Lq] workspace.
BIGDL_EXPORT int bigdl_attn_bwd(const void* q, long long ldq, const void* k, long long ldk, const void* v,
                                long long ldv, const void* o, long long ldo, const void* dout, long long ldd,
                                const float* lse, float* delta, const float* bias, long long sbb, long long sbh,
                                long long sbq, long long sbk, void* dq, long long ldg, void* dk, long long ldgk,
                                void* dv, long long ldgv, int B, int Hh, int Lq, int Lk, int D, float scale,
                                int causal, float keep, unsigned seed, const void* seed_dev, hipStream_t s) {
  AttnParams p{};
  int rc = attn_setup(p, q, ldq, k, ldk, v, ldv, bias, sbb, sbh, sbq, sbk, B, Hh, Lq, Lk, D, scale, causal, keep, seed,
                      seed_dev);
  if (rc) return rc;
  const long long hd = (long long)Hh * D;
  if (!a16(o) || !a16(dout) || !a16(dq) || !a16(dk) || !a16(dv) || !lse || !delta) return (int)hipErrorInvalidValue;
  if (ldo % 8 || ldd % 8 || ldg % 8 || ldgk % 8 || ldgv % 8) return (int)hipErrorInvalidValue;
  if (ldo < hd || ldd < hd || ldg < hd || ldgk < hd || ldgv < hd) return (int)hipErrorInvalidValue;
  p.o = (const bf16_t*)o; p.ldo = ldo; p.dout = (const bf16_t*)dout; p.ldd = ldd;
  p.lse = (float*)lse; p.delta = delta;
  p.out = (bf16_t*)dq; p.ldg = ldg; p.dk = (bf16_t*)dk; p.ldgk = ldgk; p.dv = (bf16_t*)dv; p.ldgv = ldgv;
  const dim3 gq((unsigned)((Lq + 63) / 64), (unsigned)Hh, (unsigned)B);
  const dim3 gk((unsigned)((Lk + 63) / 64), (unsigned)Hh, (unsigned)B);
  switch (D) {  // k_attn_bwd_dq also writes delta
    case 32:
      hipLaunchKernelGGL(k_attn_bwd_dq<32>, gq, dim3(256), 0, s, p);
      hipLaunchKernelGGL(k_attn_bwd_dkdv<32>, gk, dim3(256), 0, s, p);
      break;
    case 64:
      hipLaunchKernelGGL(k_attn_bwd_dq<64>, gq, dim3(256), 0, s, p);
      hipLaunchKernelGGL(k_attn_bwd_dkdv<64>, gk, dim3(256), 0, s, p);
      break;
    case 96:
      hipLaunchKernelGGL(k_attn_bwd_dq<96>, gq, dim3(256), 0, s, p);
      hipLaunchKernelGGL(k_attn_bwd_dkdv<96>, gk, dim3(256), 0, s, p);
      break;
    default:
      hipLaunchKernelGGL(k_attn_bwd_dq<128>, gq, dim3(256), 0, s, p);
      hipLaunchKernelGGL(k_attn_bwd_dkdv<128>, gk, dim3(256), 0, s, p);
      break;
  }
  BIGDL_CHECK_LAUNCH();
}
