// Relation-matrix passes of the fused step (gfx950 fp32 MFMA).
//
// RESCAL scores h^T R_r t with a dense d x d matrix per relation
// (RESCAL.py:140-174). Every triple of a positive shares (h, R_r) or
// (R_r, t), so the matrix work is per POSITIVE, not per negative:
//
//   KR  rank      positives stably sorted by relation (one pass, no atomics),
//                 so every relation's positives are contiguous.
//   KC  context   u_i = R^T h_i and v_i = R t_i for 16 positives of one
//                 relation at a time: two [16 x d] x [d x d] products on
//                 v_mfma_f32_16x16x4_f32. The score kernel then streams the
//                 negatives as dot products (u . e, e . v).
//   KP  post      the positives' own row gradients g_h = R A_i, g_t = R^T B_i
//                 (same tile shape), and per relation dR_r = sum_i h_i (x) A_i
//                 + b_i (x) t_i as [d x 2n] x [2n x d] MFMA tiles, plus the
//                 dense regulariser term (2 lambda / R) R_r of every relation
//                 (RESCAL.py:190-198) and the dense gradient's norm^2.
//   KL  reg loss  lambda (mean_e ||e||^2 + mean_r ||R_r||_F^2) added to the loss.
//
// MFMA operand maps (v_mfma_f32_16x16x4_f32, one f32 per lane): lane l holds
// A[l & 15][k = l >> 4] and B[k = l >> 4][l & 15]; the 4 accumulators hold
// C[(l >> 4) * 4 + reg][l & 15]. fp32 in, fp32 accumulate (a k-ordered fmaf
// chain): the same arithmetic as the reference's fp32 matmul up to summation
// order.
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
// rank_i = #{j : r_j < r_i} + #{j < i : r_j == r_i}; sorted[rank_i] = i
__global__ __launch_bounds__(256) void rel_rank_kernel(RelArgs P) {
  __shared__ int32_t s_r[256];
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int32_t ri = i < P.B ? (int32_t)pos_id(P, i, 1) : -1;
  int64_t lt = 0, eq = 0;
  for (int64_t j0 = 0; j0 < P.B; j0 += 256) {
    __syncthreads();
    const int64_t j = j0 + threadIdx.x;
    s_r[threadIdx.x] = j < P.B ? (int32_t)pos_id(P, j, 1) : 0;
    __syncthreads();
    const int n = (int)min<int64_t>(256, P.B - j0);
    for (int q = 0; q < n; ++q) {
      const int32_t x = s_r[q];
      lt += x < ri ? 1 : 0;
      eq += (x == ri && j0 + q < i) ? 1 : 0;
    }
  }
  if (i < P.B) {
    P.sorted[lt + eq] = (int32_t)i;
    P.srel[lt + eq] = ri;
  }
}

// ------------------------------------------------------------ KC / KP pair products
// One workgroup per leading sorted position of a 16-positive tile of one
// relation (other positions exit at once). X1, X2 = 16 staged input rows.
//   MODE 0 (context): X1 = h rows, X2 = t rows; out0 = X1 R (u), out1 = X2 R^T (v)
//   MODE 1 (post):    X1 = B rows, X2 = A rows; out0 = X1 R (g_t), out1 = X2 R^T (g_h)
template <int MODE>
__global__ __launch_bounds__(256) void rel_pair_kernel(RelArgs P) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  const int d = P.d, D4 = (d + 3) & ~3;
  const int64_t p = blockIdx.x;
  const int64_t r = P.srel[p];
  const int64_t g0 = rel_lower(P.srel, 0, p + 1, r);
  if ((p - g0) % 16 != 0) return;
  const int64_t g1 = rel_lower(P.srel, p, P.B, r + 1);
  const int n = (int)min<int64_t>(16, g1 - p);
  float* X1 = sm;
  float* X2 = sm + 16 * D4;
  __shared__ int64_t s_i[16];
  if (threadIdx.x < 16) s_i[threadIdx.x] = threadIdx.x < n ? P.sorted[p + threadIdx.x] : 0;
  __syncthreads();
  for (int e = threadIdx.x; e < 16 * D4; e += blockDim.x) {
    const int q = e / D4, k = e - q * D4;
    float x1 = 0.f, x2 = 0.f;
    if (q < n && k < d) {
      const int64_t i = s_i[q];
      if (MODE == 0) {
        x1 = P.ent.row(pos_id(P, i, 0))[k];
        x2 = P.ent.row(pos_id(P, i, 2))[k];
      } else {
        const float* g = P.gpos + i * 3 * (int64_t)P.gcols;
        x1 = g[2 * P.gcols + k];   // B_i
        x2 = g[k];                 // A_i
      }
    }
    X1[e] = x1;
    X2[e] = x2;
  }
  __syncthreads();
  const float* Rm = P.rel.row(r);
  const int lane = lane_id(), wv = wave_id();
  const int nct = (d + 15) / 16;
  const int ar = lane & 15, kq = lane >> 4;
  for (int job = wv; job < 2 * nct; job += 4) {
    const int prod = job & 1, jt = job >> 1;
    const int col = jt * 16 + (lane & 15);
    const float* X = prod ? X2 : X1;
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
    for (int k0 = 0; k0 < D4; k0 += 4) {
      const int k = k0 + kq;
      const float a = X[ar * D4 + k];
      float b = 0.f;
      if (k < d && col < d) b = prod == 0 ? Rm[(int64_t)k * d + col] : Rm[(int64_t)col * d + k];
      acc = mfma16(a, b, acc);
    }
    if (col < d) {
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int row = kq * 4 + g;
        if (row >= n) continue;
        const int64_t i = s_i[row];
        float* out;
        if (MODE == 0) out = P.snap + i * 2 * (int64_t)d + (prod ? d : 0);
        else out = P.gproj + i * 2 * (int64_t)d + (prod ? 0 : d);
        out[col] = acc[g];
      }
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
  const int d = P.d, nct = (d + 15) / 16, D16 = nct * 16;
  const int64_t r = blockIdx.x / nct;
  const int ti = (int)(blockIdx.x % nct), i0 = ti * 16;
  const int lane = lane_id(), wv = wave_id();
  float* Xc = sm;             // [32][16]
  float* Yc = sm + 32 * 16;   // [32][D16]
  __shared__ int64_t s_i[16];
  __shared__ float s_n2[4];
  __shared__ int s_last;
  const int64_t beg = rel_lower(P.srel, 0, P.B, r), end = rel_lower(P.srel, beg, P.B, r + 1);
  f32x4 acc[4];
#pragma unroll
  for (int t = 0; t < 4; ++t) acc[t] = f32x4{0.f, 0.f, 0.f, 0.f};
  for (int64_t c0 = beg; c0 < end; c0 += 16) {
    const int nrow = (int)min<int64_t>(16, end - c0);
    __syncthreads();
    if (threadIdx.x < 16) s_i[threadIdx.x] = threadIdx.x < nrow ? P.sorted[c0 + threadIdx.x] : 0;
    __syncthreads();
    for (int e = threadIdx.x; e < 32 * 16; e += blockDim.x) {
      const int q = e >> 4, c = i0 + (e & 15);
      float x = 0.f;
      if ((q & 15) < nrow && c < d) {
        const int64_t i = s_i[q & 15];
        x = q < 16 ? P.ent.row(pos_id(P, i, 0))[c] : P.gpos[i * 3 * (int64_t)P.gcols + P.gcols + c];   // h | b
      }
      Xc[e] = x;
    }
    for (int e = threadIdx.x; e < 32 * D16; e += blockDim.x) {
      const int q = e / D16, c = e - q * D16;
      float y = 0.f;
      if ((q & 15) < nrow && c < d) {
        const int64_t i = s_i[q & 15];
        y = q < 16 ? P.gpos[i * 3 * (int64_t)P.gcols + c] : P.ent.row(pos_id(P, i, 2))[c];   // A | t
      }
      Yc[e] = y;
    }
    __syncthreads();
#pragma unroll
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
  const float* Rm = P.rel.row(r);
  float* G = P.grel + r * (int64_t)d * d;
  float n2 = 0.f;
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    const int jt = wv + 4 * t;
    const int col = jt * 16 + (lane & 15);
    if (jt >= nct || col >= d) continue;
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const int row = i0 + (lane >> 4) * 4 + g;
      if (row >= d) continue;
      const float v = acc[t][g] + P.dense_rel * Rm[(int64_t)row * d + col];
      G[(int64_t)row * d + col] = v;
      n2 += v * v;
    }
  }
  n2 = wave_sum(n2);
  if (lane == 0) s_n2[wv] = n2;
  __syncthreads();
  if (threadIdx.x == 0) {
    const float w = s_n2[0] + s_n2[1] + s_n2[2] + s_n2[3];
    __hip_atomic_store(&P.rpart[blockIdx.x], w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __builtin_amdgcn_s_waitcnt(0);
    const uint32_t prev = __hip_atomic_fetch_add(&P.ctl->rel_ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    s_last = prev == gridDim.x - 1;
  }
  __syncthreads();
  if (s_last) {
    float s = 0.f;
    for (int w = threadIdx.x; w < (int)gridDim.x; w += blockDim.x)
      s += __hip_atomic_load(&P.rpart[w], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    s = wave_sum(s);
    if (lane == 0) s_n2[wv] = s;
    __syncthreads();
    if (threadIdx.x == 0) {
      const float t = s_n2[0] + s_n2[1] + s_n2[2] + s_n2[3];
      P.ctl->dn2[1] = t;
      if (P.norm2_out) P.norm2_out[1] = t;
      P.ctl->rel_ticket = 0u;
    }
  }
}

// ------------------------------------------------------------ KL regulariser loss
// lambda * (sum_e ||e||^2 / E + sum_r ||R_r||_F^2 / R): per-workgroup
// partials, the last workgroup adds the term to the step loss.
__global__ __launch_bounds__(256) void reg_loss_kernel(TabView ent, TabView rel, float lam, float* part,
                                                        StepCtl* ctl, float* loss_out, float* loss_accum) {
  __shared__ float s_p[4][2];
  __shared__ int s_last;
  const int lane = lane_id(), wv = wave_id();
  const int64_t nw = (int64_t)gridDim.x * 4;
  float se = 0.f, sr = 0.f;
  for (int64_t row = (int64_t)blockIdx.x * 4 + wv; row < ent.rows + rel.rows; row += nw) {
    const bool is_e = row < ent.rows;
    const float* x = is_e ? ent.row(row) : rel.row(row - ent.rows);
    const int cols = is_e ? ent.cols : rel.cols;
    float s = 0.f;
    for (int c = lane; c < cols; c += KGE_WAVE) s += x[c] * x[c];
    if (is_e) se += s; else sr += s;
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
  hipLaunchKernelGGL(rel_rank_kernel, dim3((unsigned)((P.B + 255) / 256)), dim3(256), 0, st, P);
}
void launch_rel_ctx(const RelArgs& P, hipStream_t st) {
  const size_t lds = 2 * 16 * (size_t)((P.d + 3) & ~3) * sizeof(float);
  hipLaunchKernelGGL(rel_pair_kernel<0>, dim3((unsigned)P.B), dim3(256), lds, st, P);
}
void launch_rel_post(const RelArgs& P, hipStream_t st) {
  const size_t lds = 2 * 16 * (size_t)((P.d + 3) & ~3) * sizeof(float);
  hipLaunchKernelGGL(rel_pair_kernel<1>, dim3((unsigned)P.B), dim3(256), lds, st, P);
  const int nct = (P.d + 15) / 16;
  const size_t lds2 = (32 * 16 + 32 * (size_t)nct * 16) * sizeof(float);
  hipLaunchKernelGGL(rel_dr_kernel, dim3((unsigned)(P.rel.rows * nct)), dim3(256), lds2, st, P);
}
void launch_reg_loss(const TabView& ent, const TabView& rel, float lam, float* part, StepCtl* ctl,
                     float* loss_out, float* loss_accum, hipStream_t st) {
  hipLaunchKernelGGL(reg_loss_kernel, dim3(kRegWGs), dim3(256), 0, st, ent, rel, lam, part, ctl, loss_out,
                     loss_accum);
}

}  // namespace kge
