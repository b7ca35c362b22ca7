// Relation-matrix passes of the fused step (gfx950 fp32 MFMA).
//
// RESCAL scores h^T R_r t with a dense d x d matrix per relation
// (RESCAL.py:140-174). Every triple of a positive shares (h, R_r) or
// (R_r, t), so the matrix work is per POSITIVE, not per negative: the score
// kernel's waves form a positive's context rows u = R^T h, v = R t and, after
// its merge, the positive's own row gradients g_h = R A, g_t = R^T B
// (rel_gemv_pair, kge_step_impl.h). This file holds the per-relation passes:
//
//   KR  rank      positives stably sorted by relation (one pass, no atomics),
//                 so every relation's positives are contiguous.
//   KP  dR        per relation dR_r = sum_i h_i (x) A_i + b_i (x) t_i as
//                 [d x 2n] x [2n x d] MFMA tiles, plus the dense regulariser
//                 term (2 lambda / R) R_r of every relation (RESCAL.py:190-198)
//                 and the dense gradient's norm^2.
//   KL  reg loss  lambda (mean_e ||e||^2 + mean_r ||R_r||_F^2) added to the loss
//                 (validation steps; train steps fold it into KP and the update).
//
// MFMA operand maps (v_mfma_f32_16x16x4_f32, one f32 per lane): lane l holds
// A[l & 15][k = l >> 4] and B[k = l >> 4][l & 15]; the 4 accumulators hold
// C[(l >> 4) * 4 + reg][l & 15]. fp32 in, fp32 accumulate (a k-ordered fmaf
// chain): the same arithmetic as the reference's fp32 matmul up to summation
// order.
#include <algorithm>

#include "kge_step.h"

namespace kge {

using f32x4 = __attribute__((ext_vector_type(4))) float;

__device__ __forceinline__ f32x4 mfma16(float a, float b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

__device__ __forceinline__ int64_t pos_id(const RelArgs& P, int64_t i, int c) {
  const int64_t v = load_idx(P.pos, i * 3 + c, P.i64);
  const int64_t lim = c == 1 ? P.rel.rows : P.ent.rows;
  return (v < 0 || v >= lim) ? 0 : v;   // the score kernel reports KGE_ERANGE
}

// ------------------------------------------------------------ KR rank
// Thread t plays positive i = t and relation r = t:
//   rank_i = #{j : r_j < r_i} + #{j < i : r_j == r_i};  sorted[rank_i] = i
//   rel_beg[r] = #{j : r_j < r}, rel_cnt[r] = #{j : r_j == r}
// Relation ids are staged 256 at a time in LDS and read back as int4
// broadcasts (every lane reads the same address).
__global__ __launch_bounds__(256) void rel_rank_kernel(RelArgs P) {
  __shared__ __attribute__((aligned(16))) int32_t s_r[256];
  const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int32_t ri = t < P.B ? (int32_t)pos_id(P, t, 1) : -1;
  const int32_t rr = (int32_t)t;
  int32_t lt = 0, eq = 0, rlt = 0, rcnt = 0;
  for (int64_t j0 = 0; j0 < P.B; j0 += 256) {
    __syncthreads();
    const int64_t j = j0 + threadIdx.x;
    s_r[threadIdx.x] = j < P.B ? (int32_t)pos_id(P, j, 1) : 0x7fffffff;   // sentinel: never < or ==
    __syncthreads();
    const int64_t before = t - j0;   // entries q < before precede positive t
#pragma unroll 4
    for (int q = 0; q < 256; q += 4) {
      const int4 x = *reinterpret_cast<const int4*>(s_r + q);
      lt += (x.x < ri) + (x.y < ri) + (x.z < ri) + (x.w < ri);
      eq += (x.x == ri && q < before) + (x.y == ri && q + 1 < before) + (x.z == ri && q + 2 < before) +
            (x.w == ri && q + 3 < before);
      rlt += (x.x < rr) + (x.y < rr) + (x.z < rr) + (x.w < rr);
      rcnt += (x.x == rr) + (x.y == rr) + (x.z == rr) + (x.w == rr);
    }
  }
  if (t < P.B) {
    P.sorted[lt + eq] = (int32_t)t;
    P.srel[lt + eq] = ri;
  }
  if (t < P.rel.rows) {
    P.rel_beg[t] = rlt;
    P.rel_cnt[t] = rcnt;
  }
}

// Small batches: a wave per item (positive t and relation t), its lanes
// sweeping the batch's relation ids straight from the triples (L2 hits after
// the first wave) and summing the four counts with integer butterflies --
// B / 64 loads per lane instead of a B-long serial loop per thread in two
// workgroups. Same counts, so the same stable order.
__device__ __forceinline__ int wave_isum(int x) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) x += __shfl_xor(x, o, KGE_WAVE);
  return x;
}
__global__ __launch_bounds__(256) void rel_rank_wave_kernel(RelArgs P) {
  const int lane = lane_id();
  const int64_t t = (int64_t)blockIdx.x * 4 + wave_id();
  const bool doi = t < P.B, dor = t < P.rel.rows;
  if (!doi && !dor) return;
  const int32_t ri = doi ? (int32_t)pos_id(P, t, 1) : -1;
  const int32_t rr = (int32_t)t;
  int lt = 0, eq = 0, rlt = 0, rcnt = 0;
#pragma unroll 8
  for (int64_t j = lane; j < P.B; j += KGE_WAVE) {
    const int32_t x = (int32_t)pos_id(P, j, 1);
    lt += x < ri;
    eq += x == ri && j < t;
    rlt += x < rr;
    rcnt += x == rr;
  }
  lt = wave_isum(lt);
  eq = wave_isum(eq);
  rlt = wave_isum(rlt);
  rcnt = wave_isum(rcnt);
  if (lane == 0) {
    if (doi) {
      P.sorted[lt + eq] = (int32_t)t;
      P.srel[lt + eq] = ri;
    }
    if (dor) {
      P.rel_beg[t] = rlt;
      P.rel_cnt[t] = rcnt;
    }
  }
}

// ------------------------------------------------------------ KP relation gradient
// Workgroup (r, ti): rows [16 ti, 16 ti + 16) of dR_r = X^T Y with
// X = [h_i ; b_i], Y = [A_i ; t_i] over the relation's positives (16 per
// chunk -> inner dimension 32), plus dense_rel * R_r; writes the dense
// gradient and reduces its norm^2 (last workgroup, fixed order).
__global__ __launch_bounds__(256) void rel_dr_kernel(RelArgs P) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  if (ws_refused(P.ctl, P.sig, P.status, P.loss_out)) return;
  const int d = P.d, nct = (d + 15) / 16, D16 = nct * 16;
  const int64_t r = blockIdx.x / nct;
  const int ti = (int)(blockIdx.x % nct), i0 = ti * 16;
  const int lane = lane_id(), wv = wave_id();
  float* Xc = sm;             // [32][16]
  float* Yc = sm + 32 * 16;   // [32][D16]
  __shared__ const float* s_x[32];
  __shared__ const float* s_y[32];
  __shared__ float s_n2[4], s_m2[4];
  // the strip's rows [i0, i0 + 16) are one contiguous run of 16 d floats in
  // both R_r and dR_r
  const int run = min(16, d - i0) * d;
  const float* Rm = P.rel.row(r) + (int64_t)i0 * d;
  const bool v4 = d % 4 == 0 && P.rel.ld % 4 == 0 && ((uintptr_t)P.rel.p % 16) == 0 && ((uintptr_t)P.grel % 16) == 0;
  constexpr int kRunV = 16 * 256 / 4 / 256;
  const int64_t beg = P.rel_beg[r], end = beg + P.rel_cnt[r];
  f32x4 acc[4];
#pragma unroll
  for (int t = 0; t < 4; ++t) acc[t] = f32x4{0.f, 0.f, 0.f, 0.f};
  // staged rows: every load of a chunk issued before any is stored (a float4
  // per lane when the rows allow) -- one L2 round trip per chunk, where a
  // scalar load-store loop took ~13 and made this pass 47 us at C4
  const bool vy = d % 4 == 0 && P.ent.ld % 4 == 0 && P.gcols % 4 == 0 && ((uintptr_t)P.ent.p % 16) == 0 &&
                  ((uintptr_t)P.gpos % 16) == 0;
  constexpr int kYV = 8;   // float4 per thread: 8 threads x 8 float4 cover a row (D16 <= 256)
  for (int64_t c0 = beg; c0 < end; c0 += 16) {
    const int nrow = (int)min<int64_t>(16, end - c0);
    __syncthreads();   // the previous chunk's MFMA reads of Xc / Yc
    if (threadIdx.x < 32) {   // each staged row's source, resolved once: h | b rows, A | t rows
      const int q = threadIdx.x & 15;
      const int64_t i = q < nrow ? P.sorted[c0 + q] : 0;
      const float* gr = P.gpos + i * 3 * (int64_t)P.gcols;
      if (threadIdx.x < 16) {
        s_x[q] = P.ent.row(pos_id(P, i, 0));
        s_y[q] = gr;
      } else {
        s_x[16 + q] = gr + P.gcols;
        s_y[16 + q] = P.ent.row(pos_id(P, i, 2));
      }
    }
    __syncthreads();
    float xv[2];
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int e = threadIdx.x + u * 256, q = e >> 4, c = i0 + (e & 15);
      xv[u] = ((q & 15) < nrow && c < d) ? s_x[q][c] : 0.f;
    }
    if (vy) {   // 8 threads per staged row (one row pointer each), float4 columns 32 apart
      const int q = threadIdx.x >> 3, l8 = threadIdx.x & 7;
      const float* src = s_y[q];
      const bool live = (q & 15) < nrow;
      float4 yv[kYV];
#pragma unroll
      for (int u = 0; u < kYV; ++u) {
        const int c = 4 * (l8 + 8 * u);
        yv[u] = (live && c < d) ? *reinterpret_cast<const float4*>(src + c) : make_float4(0.f, 0.f, 0.f, 0.f);
      }
#pragma unroll
      for (int u = 0; u < kYV; ++u) {
        const int c = 4 * (l8 + 8 * u);
        if (c < D16) *reinterpret_cast<float4*>(Yc + q * D16 + c) = yv[u];
      }
    } else {
      for (int e = threadIdx.x; e < 32 * D16; e += blockDim.x) {
        const int q = e / D16, c = e - q * D16;
        Yc[e] = ((q & 15) < nrow && c < d) ? s_y[q][c] : 0.f;
      }
    }
#pragma unroll
    for (int u = 0; u < 2; ++u) Xc[threadIdx.x + u * 256] = xv[u];
    __syncthreads();
    // k = 0..15: h_i with A_i, k = 16..31: b_i with t_i (positive order)
#pragma unroll 1
    for (int k0 = 0; k0 < 32; k0 += 4) {
      const int k = k0 + (lane >> 4);
      const float a = Xc[k * 16 + (lane & 15)];
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        const int jt = wv + 4 * t;
        if (jt < nct) acc[t] = mfma16(a, Yc[k * D16 + jt * 16 + (lane & 15)], acc[t]);
      }
    }
  }
  // epilogue: the accumulators go through LDS and the run is written a float4
  // per lane. Relations absent from the batch (most workgroups) have no
  // MFMA part: their strip is dense_rel * R_r -- not even written when the
  // apply pass re-derives it (lazy_absent: the norm partials only)
  // the strip's R_r part (<= 4 float4 per thread, d <= 256), loaded after the
  // loop: live across it, its 16 registers cost the pass half its occupancy
  float4 m[kRunV];
#pragma unroll
  for (int k = 0; k < kRunV; ++k) {
    const int e = 4 * (threadIdx.x + k * 256);
    m[k] = (v4 && e < run) ? *reinterpret_cast<const float4*>(Rm + e) : make_float4(0.f, 0.f, 0.f, 0.f);
  }
  const bool absent = beg == end;
  const bool store = !(absent && P.lazy_absent);
  float* G = P.grel + r * (int64_t)d * d + (int64_t)i0 * d;
  float* S = Yc;   // [16][D16] of the [32][D16] image
  if (!absent) {
    __syncthreads();   // the MFMA loop's last reads of Yc
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      const int jt = wv + 4 * t;
      if (jt >= nct) continue;
#pragma unroll
      for (int g = 0; g < 4; ++g) S[((lane >> 4) * 4 + g) * D16 + jt * 16 + (lane & 15)] = acc[t][g];
    }
    __syncthreads();
  }
  float n2 = 0.f, m2 = 0.f;   // gradient norm^2 | ||R_r||^2 (regulariser loss)
  if (v4) {
#pragma unroll
    for (int k = 0; k < kRunV; ++k) {
      const int e = 4 * (threadIdx.x + k * 256);
      if (e >= run) continue;
      const int row = e / d, col = e - row * d;
      float4 sv = make_float4(0.f, 0.f, 0.f, 0.f);
      if (!absent) sv = make_float4(S[row * D16 + col], S[row * D16 + col + 1], S[row * D16 + col + 2],
                                    S[row * D16 + col + 3]);
      float4 v;
      v.x = sv.x + P.dense_rel * m[k].x;
      v.y = sv.y + P.dense_rel * m[k].y;
      v.z = sv.z + P.dense_rel * m[k].z;
      v.w = sv.w + P.dense_rel * m[k].w;
      if (store) *reinterpret_cast<float4*>(G + e) = v;
      n2 += v.x * v.x + v.y * v.y + v.z * v.z + v.w * v.w;
      m2 += m[k].x * m[k].x + m[k].y * m[k].y + m[k].z * m[k].z + m[k].w * m[k].w;
    }
  } else {
    for (int e = threadIdx.x; e < run; e += blockDim.x) {
      const int row = e / d, col = e - row * d;
      const float rm = Rm[e];
      const float v = (absent ? 0.f : S[row * D16 + col]) + P.dense_rel * rm;
      G[e] = v;
      n2 += v * v;
      m2 += rm * rm;
    }
  }
  n2 = wave_sum(n2);
  m2 = wave_sum(m2);
  if (lane == 0) { s_n2[wv] = n2; s_m2[wv] = m2; }
  __syncthreads();
  // the strip's partials ([grid] gradient norm^2 | [grid] ||R||^2);
  // rescal_norms_kernel (after the dense entity update) sums them in a fixed
  // order -- no grid-wide ticket: 3 k workgroups taking turns on one counter
  // cost more than a one-workgroup launch
  if (threadIdx.x < 2) {
    const float* q = threadIdx.x ? s_m2 : s_n2;
    P.rpart[threadIdx.x * gridDim.x + blockIdx.x] = q[0] + q[1] + q[2] + q[3];
  }
}

// RESCAL train step, after the dR pass and the dense entity update: one
// workgroup sums both passes' partials in a fixed order -- the dense
// gradients' norm^2 (clip_by_norm of each dense tensor), ||R||^2 and ||e||^2
// for the regulariser loss lambda (mean_e ||e||^2 + mean_r ||R_r||_F^2)
// (RESCAL.py:190-198) -- and publishes the two SGD scales for the apply.
__global__ __launch_bounds__(256) void rescal_norms_kernel(RelArgs P, int nr, const float* upart, int nu, float lam,
                                                           float lr, float clip, float* loss_accum) {
  if (ws_refused(P.ctl, P.sig, P.status, P.loss_out)) return;
  __shared__ float s_w[4][4];
  const int lane = lane_id(), wv = wave_id();
  float a[4] = {0.f, 0.f, 0.f, 0.f};   // rel grad^2 | ||R||^2 | ent grad^2 | ||e||^2
  // eight partials of each sum in flight per thread (a serial load-add chain
  // of ~25 L2 round trips made this one-workgroup pass ~10 us); fixed order
  constexpr int U = 8;
  auto sum2 = [&](const float* x, int n, float& s0, float& s1) {
    for (int w0 = threadIdx.x; w0 < n; w0 += U * blockDim.x) {
      float q0[U], q1[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int w = w0 + u * blockDim.x;
        q0[u] = w < n ? x[w] : 0.f;
        q1[u] = w < n ? x[n + w] : 0.f;
      }
#pragma unroll
      for (int u = 0; u < U; ++u) { s0 += q0[u]; s1 += q1[u]; }
    }
  };
  sum2(P.rpart, nr, a[0], a[1]);
  sum2(upart, nu, a[2], a[3]);
#pragma unroll
  for (int k = 0; k < 4; ++k) a[k] = wave_sum(a[k]);
  if (lane == 0) {
#pragma unroll
    for (int k = 0; k < 4; ++k) s_w[wv][k] = a[k];
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    float t[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) t[k] = s_w[0][k] + s_w[1][k] + s_w[2][k] + s_w[3][k];
    P.ctl->dn2[0] = t[2];
    P.ctl->dn2[1] = t[0];
    P.ctl->reg_r2 = t[1];
    P.ctl->scale[0] = -lr * (clip / fmaxf(sqrtf(t[2]), clip));
    P.ctl->scale[1] = -lr * (clip / fmaxf(sqrtf(t[0]), clip));
    if (P.norm2_out) { P.norm2_out[0] = t[2]; P.norm2_out[1] = t[0]; }
    if (lam != 0.f) {
      const float add = lam * (t[3] / (float)P.ent.rows + t[1] / (float)P.rel.rows);
      P.loss_out[0] += add;
      if (loss_accum) loss_accum[0] += add;
    }
  }
}

// RESCAL in-step SGD of both dense gradients in one launch (keras SGD after
// clip_by_norm, BaseModel.py:327-328): blocks [0, be) stream the entity
// table a float4 per thread (w + (g * cs) * -lr), the rest go relation by
// relation over 1024-float chunks of R_r -- a relation absent from the batch
// has the gradient dense_rel * R_r, re-derived here (the dR pass wrote none
// of it), the same arithmetic as when it is stored.
__global__ __launch_bounds__(256) void rescal_apply_kernel(RelArgs P, float* ent, const float* gent, int64_t n4e,
                                                           int64_t be, int64_t bpr, float lr, float clip) {
  if (ws_refused(P.ctl, P.sig, P.status, P.loss_out)) return;
  if ((int64_t)blockIdx.x < be) {
    const float cs = clip / fmaxf(sqrtf(P.ctl->dn2[0]), clip);
    const int64_t q = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (q >= n4e) return;
    float4 w = reinterpret_cast<float4*>(ent)[q];
    const float4 g = reinterpret_cast<const float4*>(gent)[q];
    w.x = w.x + (g.x * cs) * (-lr); w.y = w.y + (g.y * cs) * (-lr);
    w.z = w.z + (g.z * cs) * (-lr); w.w = w.w + (g.w * cs) * (-lr);
    reinterpret_cast<float4*>(ent)[q] = w;
    return;
  }
  const int64_t b = blockIdx.x - be;
  const int64_t r = b / bpr, ch = b - r * bpr;
  const int64_t dd = (int64_t)P.d * P.d;
  const int64_t e = ch * 1024 + 4 * threadIdx.x;
  if (e >= dd) return;
  const float cs = clip / fmaxf(sqrtf(P.ctl->dn2[1]), clip);
  float4* wp = reinterpret_cast<float4*>(P.rel.p + r * P.rel.ld + e);
  float4 w = *wp;
  float4 g;
  if (P.rel_cnt[r] == 0) {
    g.x = 0.f + P.dense_rel * w.x; g.y = 0.f + P.dense_rel * w.y;
    g.z = 0.f + P.dense_rel * w.z; g.w = 0.f + P.dense_rel * w.w;
  } else {
    g = *reinterpret_cast<const float4*>(P.grel + r * dd + e);
  }
  w.x = w.x + (g.x * cs) * (-lr); w.y = w.y + (g.y * cs) * (-lr);
  w.z = w.z + (g.z * cs) * (-lr); w.w = w.w + (g.w * cs) * (-lr);
  *wp = w;
}

// ------------------------------------------------------------ KL regulariser loss
// lambda * (sum_e ||e||^2 / E + sum_r ||R_r||_F^2 / R): per-workgroup
// partials, the last workgroup adds the term to the step loss. Balanced
// sweep: the unit of work is a 256-float chunk of a row (a float4 per lane),
// so the R relation matrices (d^2 floats each) spread over every wave instead
// of one wave per matrix; units are dealt to waves in a fixed order
// (deterministic sums).
__device__ __forceinline__ float chunk_sq(const float* x, int64_t c0, int cols, int lane, bool a16) {
  const int64_t c = c0 + 4 * lane;
  float s = 0.f;
  if (a16 && c + 3 < cols) {
    const float4 v = *reinterpret_cast<const float4*>(x + c);
    s = v.x * v.x + v.y * v.y + v.z * v.z + v.w * v.w;
  } else {
    for (int64_t k = c; k < c0 + 4 * lane + 4 && k < cols; ++k) s += x[k] * x[k];
  }
  return s;
}

__global__ __launch_bounds__(256) void reg_loss_kernel(TabView ent, TabView rel, float lam, float* part,
                                                        StepCtl* ctl, float* loss_out, float* loss_accum,
                                                        uint32_t sig, int32_t* status) {
  if (ws_refused(ctl, sig, status, loss_out)) return;
  __shared__ float s_p[4][2];
  __shared__ int s_last;
  const int lane = lane_id(), wv = wave_id();
  const int64_t nw = (int64_t)gridDim.x * 4;
  const int64_t upe = (ent.cols + 255) / 256, upr = (rel.cols + 255) / 256;   // chunks per row
  const int64_t ue = ent.rows * upe, ur = rel.rows * upr;
  const bool ae = ((uintptr_t)ent.p % 16 == 0) && ent.ld % 4 == 0;
  const bool ar = ((uintptr_t)rel.p % 16 == 0) && rel.ld % 4 == 0;
  float se = 0.f, sr = 0.f;
  // four units in flight per wave (their loads issued before any is summed)
  for (int64_t u0 = (int64_t)blockIdx.x * 4 + wv; u0 < ue + ur; u0 += 4 * nw) {
    float q[4];
    bool isr[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int64_t u = u0 + k * nw;
      q[k] = 0.f;
      isr[k] = u >= ue;
      if (u < ue) {
        const int64_t row = u / upe;
        q[k] = chunk_sq(ent.row(row), (u - row * upe) * 256, ent.cols, lane, ae);
      } else if (u < ue + ur) {
        const int64_t v = u - ue, row = v / upr;
        q[k] = chunk_sq(rel.row(row), (v - row * upr) * 256, rel.cols, lane, ar);
      }
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      if (isr[k]) sr += q[k]; else se += q[k];
    }
  }
  se = wave_sum(se);
  sr = wave_sum(sr);
  if (lane == 0) { s_p[wv][0] = se; s_p[wv][1] = sr; }
  __syncthreads();
  if (threadIdx.x < 2) {
    const float w = s_p[0][threadIdx.x] + s_p[1][threadIdx.x] + s_p[2][threadIdx.x] + s_p[3][threadIdx.x];
    __hip_atomic_store(&part[blockIdx.x * 2 + threadIdx.x], w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    __builtin_amdgcn_s_waitcnt(0);   // the partial stores (this wave's) are drained
    const uint32_t prev = __hip_atomic_fetch_add(&ctl->reg_ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    s_last = prev == gridDim.x - 1;
  }
  __syncthreads();
  if (s_last && wv == 0) {
    float a = 0.f, b = 0.f;
    for (int w = lane; w < (int)gridDim.x; w += KGE_WAVE) {
      a += __hip_atomic_load(&part[w * 2], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      b += __hip_atomic_load(&part[w * 2 + 1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    a = wave_sum(a);
    b = wave_sum(b);
    if (lane == 0) {
      const float add = lam * (a / (float)ent.rows + b / (float)rel.rows);
      loss_out[0] += add;
      if (loss_accum) loss_accum[0] += add;
      ctl->reg_ticket = 0u;
    }
  }
}

// ------------------------------------------------------------ launchers
void launch_rel_rank(const RelArgs& P, hipStream_t st) {
  const int64_t n = std::max<int64_t>(P.B, P.rel.rows);
  if (n <= 8192)   // wave per item: n * B / 64 lane-loads, all in parallel
    hipLaunchKernelGGL(rel_rank_wave_kernel, dim3((unsigned)((n + 3) / 4)), dim3(256), 0, st, P);
  else
    hipLaunchKernelGGL(rel_rank_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, P);
}
void launch_rescal_norms(const RelArgs& P, const float* upart, int nu, float lam, float lr, float clip,
                         float* loss_accum, hipStream_t st) {
  const int nct = (P.d + 15) / 16;
  hipLaunchKernelGGL(rescal_norms_kernel, dim3(1), dim3(256), 0, st, P, (int)(P.rel.rows * nct), upart, nu, lam, lr,
                     clip, loss_accum);
}
bool rescal_apply_fused_ok(const RelArgs& P, const TabView& ent, const float* gent) {
  const int64_t dd = (int64_t)P.d * P.d;
  return dd % 4 == 0 && P.rel.ld % 4 == 0 && ((uintptr_t)P.rel.p % 16) == 0 && ((uintptr_t)P.grel % 16) == 0 &&
         ent.ld == ent.cols && ((int64_t)ent.rows * ent.cols) % 4 == 0 && ((uintptr_t)ent.p % 16) == 0 &&
         ((uintptr_t)gent % 16) == 0;
}
void launch_rescal_apply(const RelArgs& P, const TabView& ent, const float* gent, float lr, float clip,
                         hipStream_t st) {
  const int64_t n4e = ent.rows * (int64_t)ent.cols / 4;
  const int64_t be = (n4e + 255) / 256;
  const int64_t bpr = ((int64_t)P.d * P.d + 1023) / 1024;
  hipLaunchKernelGGL(rescal_apply_kernel, dim3((unsigned)(be + P.rel.rows * bpr)), dim3(256), 0, st, P, ent.p, gent,
                     n4e, be, bpr, lr, clip);
}
void launch_rel_post(const RelArgs& P, hipStream_t st) {
  // (g_h, g_t: the score kernel's waves, Rescal::SELF_CTX)
  const int nct = (P.d + 15) / 16;
  const size_t lds2 = (32 * 16 + 32 * (size_t)nct * 16) * sizeof(float);
  hipLaunchKernelGGL(rel_dr_kernel, dim3((unsigned)(P.rel.rows * nct)), dim3(256), lds2, st, P);
}
void launch_reg_loss(const TabView& ent, const TabView& rel, float lam, float* part, StepCtl* ctl,
                     float* loss_out, float* loss_accum, uint32_t sig, int32_t* status, hipStream_t st) {
  hipLaunchKernelGGL(reg_loss_kernel, dim3(kRegWGs), dim3(256), 0, st, ent, rel, lam, part, ctl, loss_out,
                     loss_accum, sig, status);
}

}  // namespace kge
