// Fused KGE training step for gfx950 -- element-wise model family.
//
// One reference batch step (KGEModel.__run_single_batch, BaseModel.py:293-330)
// runs as stream-ordered kernels:
//
//   K0  constrain   full-table row renormalisation of ent_emb when the model's
//                   _constraint_loss assigns it (TransE.py:171-172,
//                   DistMult.py:162-163).
//   KS  score       8-wave workgroups; `wpp` waves per positive. In-register
//                   Philox negative draws (ns_strategy.py:39-64 in the layout
//                   of BaseModel.py:332-408); each wave issues the gathers of
//                   ALL its sampled rows at once (up to 32 rows in flight per
//                   wave, kept in registers through the loss epilogue, so no
//                   row is read twice); batched wave64 shuffle reductions for
//                   the scores (score.py); the loss epilogue per positive in
//                   LDS (loss.py; SANS softmax); analytic gradients: the
//                   positive's own rows are reduced on chip, every negative
//                   leaves one scalar coefficient. Finally the workgroup's
//                   destination keys (entities AND the positive's relation)
//                   are grouped by destination bucket (stable LDS counting
//                   sort) for the update kernel.
//   KU  update      destination-major, one workgroup per bucket: merges every
//                   score workgroup's keys for its rows (LDS bitonic sort,
//                   parallel segment scan), re-derives each negative's row
//                   gradient from ONE frozen context row + its coefficient
//                   (4 entries' loads in flight per wave), sums in registers,
//                   applies clip_by_norm(5) per variable (BaseModel.py:327,
//                   TF-2.5 IndexedSlices: norm over un-deduplicated slices)
//                   and the SGD update (BaseModel.py:328, keras SGD
//                   ResourceScatterAdd) with ONE read-modify-write per touched
//                   row. No float atomics; fixed summation order, so results
//                   are bit-reproducible.
#include "kge_step.h"

namespace kge {

// ------------------------------------------------------------ K0 constrain
// kind 0: normalized_embeddings(p=2) -> X / pow(sum X^2, 1/2) * value
// kind 1: clip_constraint(p=2)       -> rows with norm >= value rescaled
// Each wave owns 4 rows and issues all their loads before reducing.
__global__ __launch_bounds__(256) void constrain_rows_kernel(float* __restrict__ t, int64_t rows,
                                                              int32_t cols, int64_t ld, int kind,
                                                              float value) {
  constexpr int RPW = 4;
  const int64_t nw = (int64_t)gridDim.x * (blockDim.x / KGE_WAVE);
  const bool v4 = (cols % 4 == 0) && (ld % 4 == 0) && (((uintptr_t)t & 15) == 0) && cols <= 4 * KGE_WAVE;
  for (int64_t r0 = ((int64_t)blockIdx.x * (blockDim.x / KGE_WAVE) + wave_id()) * RPW; r0 < rows;
       r0 += nw * RPW) {
    if (v4) {
      float4 x[RPW];
      float s[RPW];
      const int e0 = lane_id() * 4;
#pragma unroll
      for (int u = 0; u < RPW; ++u) {
        x[u] = make_float4(0.f, 0.f, 0.f, 0.f);
        if (r0 + u < rows && e0 < cols) x[u] = *reinterpret_cast<const float4*>(t + (r0 + u) * ld + e0);
      }
#pragma unroll
      for (int u = 0; u < RPW; ++u) s[u] = x[u].x * x[u].x + x[u].y * x[u].y + x[u].z * x[u].z + x[u].w * x[u].w;
#pragma unroll
      for (int o = 32; o >= 1; o >>= 1) {
#pragma unroll
        for (int u = 0; u < RPW; ++u) s[u] += __shfl_xor(s[u], o, KGE_WAVE);
      }
#pragma unroll
      for (int u = 0; u < RPW; ++u) {
        if (r0 + u >= rows || e0 >= cols) continue;
        const float n = sqrtf(s[u]);
        float4 y = x[u];
        if (kind == 0) {
          y.x = y.x / n * value; y.y = y.y / n * value; y.z = y.z / n * value; y.w = y.w / n * value;
        } else if (!(n < value)) {
          const float d = fmaxf(n, 1e-9f);
          y.x = y.x / d * value; y.y = y.y / d * value; y.z = y.z / d * value; y.w = y.w / d * value;
        } else {
          continue;
        }
        *reinterpret_cast<float4*>(t + (r0 + u) * ld + e0) = y;
      }
    } else {
      for (int u = 0; u < RPW && r0 + u < rows; ++u) {
        float* row = t + (r0 + u) * ld;
        float s = 0.f;
        for (int e = lane_id(); e < cols; e += KGE_WAVE) s += row[e] * row[e];
        s = wave_sum(s);
        const float n = sqrtf(s);
        if (kind == 0) {
          for (int e = lane_id(); e < cols; e += KGE_WAVE) row[e] = row[e] / n * value;
        } else if (!(n < value)) {
          const float d = fmaxf(n, 1e-9f);
          for (int e = lane_id(); e < cols; e += KGE_WAVE) row[e] = row[e] / d * value;
        }
      }
    }
  }
}

// ------------------------------------------------------------ helpers
__device__ __forceinline__ float log_sigmoid(float x) {
  return fminf(x, 0.f) - log1pf(expf(-fabsf(x)));
}
__device__ __forceinline__ float sigmoid(float x) { return 1.f / (1.f + expf(-x)); }

// slot j of positive i -> corruption kind (BaseModel.py:353-356: 'h+t' rows
// alternate [h-corrupt j/2, t-corrupt j/2]), draw index within its side's
// counter plane, plane offset (0 = h side / single side, 1 = t side)
__device__ __forceinline__ void slot_layout(int side_mode, int Kside, int64_t i, int j, int* kind,
                                            uint64_t* n, uint64_t* plane_off) {
  if (side_mode == KGE_SIDE_HT) {
    *kind = (j & 1) ? KIND_TC : KIND_HC;
    *n = (uint64_t)(i * Kside + (j >> 1));
    *plane_off = (j & 1);
  } else {
    *kind = side_mode == KGE_SIDE_H ? KIND_HC : KIND_TC;
    *n = (uint64_t)(i * Kside + j);
    *plane_off = 0;
  }
}
__device__ __forceinline__ int slot_kind(int side_mode, int j) {
  if (side_mode == KGE_SIDE_HT) return (j & 1) ? KIND_TC : KIND_HC;
  return side_mode == KGE_SIDE_H ? KIND_HC : KIND_TC;
}

template <int N>
__device__ __forceinline__ void wave_sum_n(float (&x)[N]) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) {
#pragma unroll
    for (int u = 0; u < N; ++u) x[u] += __shfl_xor(x[u], o, KGE_WAVE);
  }
}
template <int N>
__device__ __forceinline__ void wave_max_n(float (&x)[N]) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) {
#pragma unroll
    for (int u = 0; u < N; ++u) x[u] = fmaxf(x[u], __shfl_xor(x[u], o, KGE_WAVE));
  }
}

// exclusive scan of one int per thread over the whole (kStepThreads) block
__device__ __forceinline__ int block_scan_excl(int v, int* s_w, int* total) {
  const int lane = lane_id(), wv = wave_id();
  int x = v;
#pragma unroll
  for (int o = 1; o < KGE_WAVE; o <<= 1) {
    const int y = __shfl_up(x, o, KGE_WAVE);
    if (lane >= o) x += y;
  }
  if (lane == KGE_WAVE - 1) s_w[wv] = x;
  __syncthreads();
  int off = 0, tot = 0;
#pragma unroll
  for (int k = 0; k < kStepWaves; ++k) {
    const int t = s_w[k];
    off += k < wv ? t : 0;
    tot += t;
  }
  __syncthreads();
  *total = tot;
  return off + x - v;
}

// relation-row fragments: full layout, or RotatE's half layout
template <bool HALF, int VEC>
struct RelV { static constexpr int n = HALF ? (VEC / 2 > 0 ? VEC / 2 : 1) : VEC; };

template <bool HALF, int VEC, int NC>
__device__ __forceinline__ void load_rel_row(float (&v)[(HALF ? (VEC / 2 > 0 ? VEC / 2 : 1) : VEC) * NC], const float* row, int cols) {
  if constexpr (HALF) {
    load_row_half<VEC, NC>(v, row, cols);
  } else {
    Frag<VEC, NC> f;
    load_row(f, row, cols);
#pragma unroll
    for (int q = 0; q < VEC * NC; ++q) v[q] = f.v[q];
  }
}
template <bool HALF, int VEC, int NC>
__device__ __forceinline__ void store_rel_row(const float (&v)[(HALF ? (VEC / 2 > 0 ? VEC / 2 : 1) : VEC) * NC], float* row, int cols) {
  if constexpr (HALF) {
    store_row_half<VEC, NC>(v, row, cols);
  } else {
    Frag<VEC, NC> f;
#pragma unroll
    for (int q = 0; q < VEC * NC; ++q) f.v[q] = v[q];
    store_row(f, row, cols);
  }
}

// ------------------------------------------------------------ KS score
template <template <int, int, int> class Model, int VEC, int NC, int SK>
__global__ __launch_bounds__(kStepThreads) void score_kernel(StepArgs A) {
  using M = Model<VEC, NC, SK>;
  using F = Frag<VEC, NC>;
  constexpr int W = kStepWaves;
  constexpr int FL = KGE_WAVE * VEC * NC;   // floats per fragment image
  constexpr int ROWS = 32 / NC;             // sampled rows resident per wave
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];

  const int Keff = A.Keff, nP = A.nP, wpp = A.wpp, Kp = A.Kp;
  const ScoreLds L = score_lds(FL, nP, Kp, Keff, A.slotmax, A.P);
  float* red = reinterpret_cast<float*>(smem + L.red);      // [W][3][FL]
  float* s_R = reinterpret_cast<float*>(smem + L.sR);       // [nP][Kp] reduced value
  float* s_ti = reinterpret_cast<float*>(smem + L.sti);     // [nP][Kp] p=inf ties
  float* s_sc = reinterpret_cast<float*>(smem + L.ssc);     // [nP][Kp] score -> alpha
  float* s_M = reinterpret_cast<float*>(smem + L.sM);       // [nP][Kp] lp -> reduced value
  int32_t* s_ids = reinterpret_cast<int32_t*>(smem + L.ids);
  int32_t* s_bkt = reinterpret_cast<int32_t*>(smem + L.bkt);
  float* s_misc = reinterpret_cast<float*>(smem + L.misc);
  int32_t* s_w = reinterpret_cast<int32_t*>(smem + L.sw);
  int64_t* s_pos = reinterpret_cast<int64_t*>(smem + L.pos);
  int32_t* s_cnt = reinterpret_cast<int32_t*>(smem + L.cnt);

  const int tid = threadIdx.x, lane = lane_id(), wv = wave_id();
  const int grp = wv / wpp, gw = wv % wpp;
  const MP mp{A.limit};
  float nrm[4] = {0.f, 0.f, 0.f, 0.f};
  float loss_acc = 0.f;
  int err = 0;

  const int64_t i0 = (int64_t)blockIdx.x * nP;
  const int nValid = (int)min<int64_t>((int64_t)nP, A.B - i0);

  // positive ids of the workgroup
  if (tid < nValid * 3) {
    const int p = tid / 3, c = tid % 3;
    int64_t v = load_idx(A.pos, (i0 + p) * 3 + c, A.i64);
    const int64_t lim = c == 1 ? A.rel.rows : A.ent.rows;
    if (v < 0 || v >= lim) { err = KGE_ERANGE; v = 0; }
    s_pos[tid] = v;
  }
  // negative ids (draw or read), bounds-checked
  for (int s = tid; s < nValid * Keff; s += blockDim.x) {
    const int p = s / Keff, j = s % Keff;
    const int64_t i = i0 + p;
    int kind; uint64_t n, poff;
    slot_layout(A.side_mode, A.Kside, i, j, &kind, &n, &poff);
    int64_t e;
    if (A.given) {
      e = load_idx(A.neg_user, i * Keff + j, A.i64);
    } else {
      const int64_t x = load_idx(A.pos, i * 3 + (kind == KIND_HC ? 0 : 2), A.i64);
      if (A.smp.kind == KGE_SAMPLER_TYPED && (x < 0 || x >= A.ent.rows)) { e = 0; err = KGE_ERANGE; }
      else {
        e = sample_entity(A.smp, A.smp.offset + poff, n, x, &err);   // plane offset (+1 for the t side)
        if (e < 0) e = 0;
      }
      if (A.neg_user) store_idx(A.neg_user, i * Keff + j, e, A.i64);
    }
    if (e < 0 || e >= A.ent.rows) { err = KGE_ERANGE; e = 0; }
    s_ids[s] = (int32_t)e;
  }
  __syncthreads();

  const bool active = grp < nValid;
  const int64_t i = i0 + grp;
  typename M::Ctx ctx;
  if (active) {
    M::load_ctx(ctx, A.ent, A.rel, s_pos[grp * 3 + 0], s_pos[grp * 3 + 1], s_pos[grp * 3 + 2], mp);
  }
  const int jbeg = gw * A.SW;
  const int jend = min(Keff, jbeg + A.SW);
  const int nchunk = (A.SW + ROWS - 1) / ROWS;
  const int32_t* ids = s_ids + grp * Keff;
  float* gR = s_R + grp * Kp;
  float* gT = s_ti + grp * Kp;
  float* gS = s_sc + grp * Kp;
  float* gM = s_M + grp * Kp;

  F E[ROWS];
  // ---- phase A: scores (slot Keff = the positive, done by the group's last wave)
  if (active) {
    if (gw == wpp - 1) {
      F a, b, E0;
      E0.zero();
      M::fwd(ctx, KIND_POS, E0, a, b);
      const float part = score_partial<SK, M::CPLX>(a, b);
      const float Rv = SK == SK_PINF ? wave_max(part) : wave_sum(part);
      float ti = 1.f;
      if (SK == SK_PINF) ti = wave_sum(tie_partial<M::CPLX>(a, Rv));
      if (lane == 0) { gR[Keff] = Rv; gT[Keff] = ti; }
    }
    for (int c = 0; c < nchunk; ++c) {
      const int j0 = jbeg + c * ROWS;
#pragma unroll
      for (int u = 0; u < ROWS; ++u)
        if (j0 + u < jend) load_row(E[u], A.ent.row(ids[j0 + u]), A.ent.cols);
      float part[ROWS];
#pragma unroll
      for (int u = 0; u < ROWS; ++u) {
        part[u] = 0.f;
        if (j0 + u < jend) {
          F a, b;
          M::fwd(ctx, slot_kind(A.side_mode, j0 + u), E[u], a, b);
          part[u] = score_partial<SK, M::CPLX>(a, b);
        }
      }
      if (SK == SK_PINF) {
        wave_max_n(part);
        float tp[ROWS];
#pragma unroll
        for (int u = 0; u < ROWS; ++u) {
          tp[u] = 0.f;
          if (j0 + u < jend) {
            F a, b;
            M::fwd(ctx, slot_kind(A.side_mode, j0 + u), E[u], a, b);
            tp[u] = tie_partial<M::CPLX>(a, part[u]);
          }
        }
        wave_sum_n(tp);
        if (lane == 0) {
#pragma unroll
          for (int u = 0; u < ROWS; ++u)
            if (j0 + u < jend) { gR[j0 + u] = part[u]; gT[j0 + u] = tp[u]; }
        }
      } else {
        wave_sum_n(part);
        if (lane == 0) {
#pragma unroll
          for (int u = 0; u < ROWS; ++u)
            if (j0 + u < jend) { gR[j0 + u] = part[u]; gT[j0 + u] = 1.f; }
        }
      }
    }
  }
  __syncthreads();

  // ---- loss epilogue (first wave of each group): c_j = dL/ds_j -> alpha_j
  if (active && gw == 0) {
    float lpp;
    const float sp = score_value<SK>(gR[Keff], A.pw, &lpp);
    float zmax = -INFINITY;
    for (int j = lane; j < Keff; j += KGE_WAVE) {
      float lpj;
      const float sj = score_value<SK>(gR[j], A.pw, &lpj);
      gS[j] = sj;
      gM[j] = lpj;   // keep lp for alpha
      zmax = fmaxf(zmax, A.temperature * sj);
    }
    zmax = wave_max(zmax);
    float Z = 0.f;
    if (A.loss_kind == KGE_LOSS_SANS)
      for (int j = lane; j < Keff; j += KGE_WAVE) Z += expf(A.temperature * gS[j] - zmax);
    Z = wave_sum(Z);
    float lsum = 0.f, csum = 0.f;
    for (int j = lane; j < Keff; j += KGE_WAVE) {
      const float sj = gS[j];
      float c = 0.f;
      switch (A.loss_kind) {
        case KGE_LOSS_HINGE: {
          const float m = A.margin + sj - sp;
          lsum += fmaxf(m, 0.f);
          c = (m >= 0.f) ? A.inv_bk : 0.f;
        } break;
        case KGE_LOSS_LOGISTIC: {
          const float ex = expf(sj - sp);
          lsum += logf(1.f + ex);
          c = ex / (1.f + ex);
        } break;
        case KGE_LOSS_BCE:
          lsum += log_sigmoid(-sj);
          c = sigmoid(sj) * A.inv_b;
          break;
        case KGE_LOSS_SANS: {
          const float pj = expf(A.temperature * sj - zmax) / Z;
          lsum += pj * log_sigmoid(-sj - A.margin);
          c = pj * sigmoid(sj + A.margin) * A.inv_b;
        } break;
        default:  // SQERR
          lsum += sj * sj;
          c = sj * A.inv_b;
          break;
      }
      csum += c;
      const float al = score_alpha<SK>(c, gR[j], gM[j], gT[j], A.pw);
      const float Mj = gR[j];
      if (A.train) A.coef[i * Keff + j] = make_float2(al, Mj);
      gM[j] = Mj;
      gS[j] = al;   // alpha (scores already consumed)
      if (A.neg_score_out) A.neg_score_out[i * Keff + j] = sj;
    }
    lsum = wave_sum(lsum);
    csum = wave_sum(csum);
    // DistMult constraint term lambda * mean_i ||r_i||^2 (DistMult.py:164-165)
    float rreg = 0.f;
    if (A.rel_reg != 0.f) {
      F Rr;
      load_row(Rr, A.rel.row(s_pos[grp * 3 + 1]), A.rel.cols);
      rreg = wave_sum(sq_partial(Rr)) * A.rel_reg * A.inv_b;
    }
    if (lane == 0) {
      loss_acc += rreg;
      float cp, lossp;
      switch (A.loss_kind) {
        case KGE_LOSS_HINGE:
          lossp = lsum * A.inv_bk;
          cp = -csum;
          if (Keff == 0) lossp = NAN;   // sum([]) / 0 (loss.py:81-82)
          break;
        case KGE_LOSS_LOGISTIC: lossp = lsum; cp = -csum; break;
        case KGE_LOSS_BCE:
          lossp = -(log_sigmoid(sp) + lsum) * A.inv_b;
          cp = -sigmoid(-sp) * A.inv_b;
          break;
        case KGE_LOSS_SANS:
          lossp = -(log_sigmoid(sp + A.margin) + lsum) * A.inv_b;
          cp = -sigmoid(-(sp + A.margin)) * A.inv_b;
          break;
        default:
          lossp = ((sp - 1.f) * (sp - 1.f) + lsum) * 0.5f * A.inv_b;
          cp = (sp - 1.f) * A.inv_b;
          break;
      }
      loss_acc += lossp;
      gS[Keff] = score_alpha<SK>(cp, gR[Keff], lpp, gT[Keff], A.pw);
      gM[Keff] = gR[Keff];
      if (A.pos_score_out) A.pos_score_out[i] = sp;
    }
  }
  __syncthreads();

  if (A.train) {
    // ---- phase B: analytic gradients (rows still resident when nchunk == 1)
    F accH, accR, accT;
    accH.zero(); accR.zero(); accT.zero();
    if (active) {
      if (gw == wpp - 1) {
        F a, b, E0;
        E0.zero();
        M::fwd(ctx, KIND_POS, E0, a, b);
        M::bwd(ctx, KIND_POS, E0, a, b, gS[Keff], gM[Keff], accH, accR, accT, nrm, mp);
      }
      if (A.rel_reg != 0.f && gw == 0) {
        // its own IndexedSlices block: (lambda / B) * 2 r  (pow-2 gradient)
        F Rr;
        load_row(Rr, A.rel.row(s_pos[grp * 3 + 1]), A.rel.cols);
        const float gsc = A.rel_reg * A.inv_b;
#pragma unroll
        for (int q = 0; q < VEC * NC; ++q) {
          const float g = gsc * (2.f * Rr.v[q]);
          accR.v[q] += g;
          nrm[1] += g * g;
        }
      }
      for (int c = 0; c < nchunk; ++c) {
        const int j0 = jbeg + c * ROWS;
        if (nchunk > 1) {
#pragma unroll
          for (int u = 0; u < ROWS; ++u)
            if (j0 + u < jend) load_row(E[u], A.ent.row(ids[j0 + u]), A.ent.cols);
        }
#pragma unroll
        for (int u = 0; u < ROWS; ++u) {
          const int j = j0 + u;
          if (j < jend) {
            const int kind = slot_kind(A.side_mode, j);
            F a, b;
            M::fwd(ctx, kind, E[u], a, b);
            M::bwd(ctx, kind, E[u], a, b, gS[j], gM[j], accH, accR, accT, nrm, mp);
          }
        }
      }
    }
    // cross-wave reduction of the positive's row gradients
    float* my = red + wv * 3 * FL;
#pragma unroll
    for (int q = 0; q < VEC * NC; ++q) {
      const int c = q / VEC, k = q % VEC;
      const int e = (c * KGE_WAVE + lane) * VEC + k;
      my[e] = accH.v[q];
      my[FL + e] = accR.v[q];
      my[2 * FL + e] = accT.v[q];
    }
    if (active && gw == 0) M::write_snap(ctx, A.snap + i * (M::NSNAP * (int64_t)A.snap_cols), A.snap_cols);
    __syncthreads();
    for (int e = tid; e < nValid * 3 * FL; e += blockDim.x) {
      const int p = e / (3 * FL), rem = e % (3 * FL);
      const int v = rem / FL, k = rem % FL;
      const int cols = v == 1 ? A.rel_gcols : A.ent.cols;
      if (k >= cols) continue;
      // RotatE keeps the phase gradient of complex element k in float 2k
      const int src = (v == 1 && A.rel_half) ? 2 * k : k;
      float s = 0.f;
      for (int g = 0; g < wpp; ++g) s += red[((p * wpp + g) * 3 + v) * FL + src];
      A.gpos[(i0 + p) * 3 * (int64_t)A.gcols + v * (int64_t)A.gcols + k] = s;
    }
  }

  // ---- per-workgroup partials: loss, norm^2 per variable (fixed order)
#pragma unroll
  for (int v = 0; v < 4; ++v) nrm[v] = wave_sum(nrm[v]);
  if (lane == 0) {
    s_misc[wv * 8] = loss_acc;
#pragma unroll
    for (int v = 0; v < 4; ++v) s_misc[wv * 8 + 1 + v] = nrm[v];
  }
  if (err) set_status(A.status, err);
  __syncthreads();
  if (tid < 5) {
    float s = 0.f;
    for (int w = 0; w < W; ++w) s += s_misc[w * 8 + tid];
    A.part[(int64_t)blockIdx.x * 8 + tid] = s;
  }
  if (!A.train) return;

  // ---- group the workgroup's destination keys by bucket (stable counting sort)
  // key = dest << 32 | code; dest < E: entity, dest >= E: relation dest - E.
  // code < nP*Keff: negative slot; else nP*Keff + 3p + {0: h, 1: t, 2: r}.
  const int Kn = nP * Keff;
  const int nNeg = nValid * Keff;
  const int nKeys = nNeg + 3 * nValid;
  const int64_t E_ = A.ent.rows;
  auto key_of = [&](int s) -> uint64_t {
    if (s < nNeg) return ((uint64_t)(uint32_t)s_ids[s] << 32) | (uint32_t)s;
    const int q = s - nNeg, p = q / 3, c = q % 3;
    const int64_t dest = c == 0 ? s_pos[p * 3] : c == 1 ? s_pos[p * 3 + 2] : E_ + s_pos[p * 3 + 1];
    return ((uint64_t)dest << 32) | (uint32_t)(Kn + q);
  };
  for (int b = tid; b <= A.P; b += blockDim.x) s_cnt[b] = 0;
  __syncthreads();
  for (int s = tid; s < nKeys; s += blockDim.x) {
    const int b = (int)((int64_t)(key_of(s) >> 32) / A.bs);
    s_bkt[s] = b;
    atomicAdd(&s_cnt[b], 1);
  }
  __syncthreads();
  {
    const int CP = (A.P + blockDim.x - 1) / blockDim.x;
    const int b0 = tid * CP, b1 = min(A.P, b0 + CP);
    int local = 0;
    for (int b = b0; b < b1; ++b) local += s_cnt[b];
    int total;
    int run = block_scan_excl(local, s_w, &total);
    for (int b = b0; b < b1; ++b) {
      const int c = s_cnt[b];
      A.bmap[(int64_t)b * A.nWG + blockIdx.x] = ((uint32_t)run << 16) | (uint32_t)c;
      s_cnt[b] = run;
      run += c;
    }
  }
  __syncthreads();
  uint64_t* out = A.sorted + (int64_t)blockIdx.x * A.slotmax;
  for (int s = tid; s < nKeys; s += blockDim.x) {
    const int b = s_bkt[s];
    int rank = 0;
    for (int s2 = 0; s2 < s; ++s2) rank += s_bkt[s2] == b;   // LDS broadcast reads
    out[s_cnt[b] + rank] = key_of(s);
  }
}

// ------------------------------------------------------------ KU update
// blocks [0, P): destination buckets of bs consecutive destinations. Block 0
// also reduces the loss. Dynamic LDS: s_list [kUCap] u64, s_segs [kUCap+4],
// red [W][FL] (overflow path).
template <template <int, int, int> class Model, int VEC, int NC, int SK>
__global__ __launch_bounds__(kStepThreads) void update_kernel(StepArgs A) {
  using M = Model<VEC, NC, SK>;
  using F = Frag<VEC, NC>;
  constexpr int W = kStepWaves;
  constexpr int FL = KGE_WAVE * VEC * NC;
  constexpr int U = NC == 1 ? 4 : NC == 2 ? 2 : 1;   // entries in flight per wave
  constexpr int RV = RelV<M::CPLX, VEC>::n;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  uint64_t* s_list = reinterpret_cast<uint64_t*>(smem);
  int32_t* s_segs = reinterpret_cast<int32_t*>(s_list + kUCap);
  float* red = reinterpret_cast<float*>(s_segs + kUCap + 4);
  __shared__ float s_part[W * 8];
  __shared__ float s_scale[8];
  __shared__ int s_w[16];
  __shared__ int s_flag;

  const int tid = threadIdx.x, lane = lane_id(), wv = wave_id();

  // ---- clip_by_norm scale per variable: clip / max(||g||, clip), and the loss
  {
    float acc[5] = {0.f, 0.f, 0.f, 0.f, 0.f};
    for (int w = tid; w < A.nWG; w += blockDim.x) {
#pragma unroll
      for (int k = 0; k < 5; ++k) acc[k] += A.part[(int64_t)w * 8 + k];
    }
#pragma unroll
    for (int k = 0; k < 5; ++k) acc[k] = wave_sum(acc[k]);
    if (lane == 0) {
#pragma unroll
      for (int k = 0; k < 5; ++k) s_part[wv * 8 + k] = acc[k];
    }
    __syncthreads();
    if (tid < 5) {
      float s = 0.f;
      for (int w = 0; w < W; ++w) s += s_part[w * 8 + tid];
      if (tid == 0) {
        if (blockIdx.x == 0) {
          A.loss_out[0] = s;
          if (A.loss_accum) A.loss_accum[0] += s;
        }
      } else {
        s_scale[tid - 1] = -A.lr * (A.clip_norm / fmaxf(sqrtf(s), A.clip_norm));
        if (blockIdx.x == 0 && A.norm2_out) A.norm2_out[tid - 1] = s;
      }
    }
    __syncthreads();
  }
  if (!A.train) return;

  const int b = blockIdx.x;
  const int64_t lo = (int64_t)b * A.bs;
  const int64_t E_ = A.ent.rows;
  const int64_t ndest = E_ + A.rel.rows;
  const int Kn = A.nP * A.Keff;

  // ---- per-source-workgroup counts and a deterministic exclusive scan
  const int CW = (A.nWG + blockDim.x - 1) / blockDim.x;
  const int w0 = tid * CW, w1 = min(A.nWG, w0 + CW);
  int local = 0;
  for (int w = w0; w < w1; ++w) local += (int)(A.bmap[(int64_t)b * A.nWG + w] & 0xFFFFu);
  int L;
  const int base0 = block_scan_excl(local, s_w, &L);
  if (L == 0) return;

  // one key -> its positive's index i, and for a negative its slot j (c = -1);
  // for a positive's own row c = 0 (h), 1 (t), 2 (r)
  auto decode = [&](uint32_t lo32, int64_t* i, int* j, int* c) {
    const int w = (int)(lo32 >> 16), code = (int)(lo32 & 0xFFFFu);
    if (code < Kn) {
      *i = (int64_t)w * A.nP + code / A.Keff;
      *j = code % A.Keff;
      *c = -1;
    } else {
      const int q = code - Kn;
      *i = (int64_t)w * A.nP + q / 3;
      *j = 0;
      *c = q % 3;
    }
  };
  // entity destination: sum of the gradient rows of entries [s0, s1) of `src`
  auto entity_sum = [&](const uint64_t* src, int s0, int s1, const F& E, F& acc) {
    for (int s = s0; s < s1; s += U) {
      int64_t ii[U];
      int jj[U], cc[U];
      typename M::ECtx ec[U];
      float2 cf[U];
      F gp[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        if (s + u < s1) {
          decode((uint32_t)src[s + u], &ii[u], &jj[u], &cc[u]);
          if (cc[u] < 0) {
            cf[u] = A.coef[ii[u] * A.Keff + jj[u]];
            M::load_ectx(A.snap + ii[u] * (M::NSNAP * (int64_t)A.snap_cols), A.snap_cols,
                         slot_kind(A.side_mode, jj[u]), ec[u]);
          } else {
            load_row(gp[u], A.gpos + ii[u] * 3 * (int64_t)A.gcols + (cc[u] == 0 ? 0 : 2) * (int64_t)A.gcols,
                     A.ent.cols);
          }
        }
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        if (s + u < s1) {
          if (cc[u] < 0) {
            F g;
            M::grad_entity(ec[u], slot_kind(A.side_mode, jj[u]), E, cf[u].x, cf[u].y, g);
            add_to(acc, g);
          } else {
            add_to(acc, gp[u]);
          }
        }
      }
    }
  };
  auto rel_sum = [&](const uint64_t* src, int s0, int s1, float (&acc)[RV * NC]) {
    for (int s = s0; s < s1; s += U) {
      float g[U][RV * NC];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        if (s + u < s1) {
          int64_t ii;
          int jj, cc;
          decode((uint32_t)src[s + u], &ii, &jj, &cc);
          load_rel_row<M::CPLX, VEC, NC>(g[u], A.gpos + ii * 3 * (int64_t)A.gcols + A.gcols, A.rel_gcols);
        }
      }
#pragma unroll
      for (int u = 0; u < U; ++u)
        if (s + u < s1) {
#pragma unroll
          for (int q = 0; q < RV * NC; ++q) acc[q] += g[u][q];
        }
    }
  };
  auto apply_entity = [&](int64_t e, F& E, const F& acc) {
    if (A.grad_mode) {
      store_row(acc, A.gent + e * (int64_t)A.ent.cols, A.ent.cols);
      return;
    }
    const float sc = s_scale[0];
#pragma unroll
    for (int q = 0; q < VEC * NC; ++q) E.v[q] = E.v[q] + acc.v[q] * sc;
    store_row(E, A.ent.row_w(e), A.ent.cols);
  };
  auto apply_rel = [&](int64_t r, const float (&acc)[RV * NC]) {
    if (A.grad_mode) {
      store_rel_row<M::CPLX, VEC, NC>(acc, A.grel + r * (int64_t)A.rel_gcols, A.rel.cols);
      return;
    }
    float row[RV * NC];
    load_rel_row<M::CPLX, VEC, NC>(row, A.rel.row(r), A.rel.cols);
    const float sc = s_scale[1];
#pragma unroll
    for (int q = 0; q < RV * NC; ++q) row[q] = row[q] + acc[q] * sc;
    store_rel_row<M::CPLX, VEC, NC>(row, A.rel.row_w(r), A.rel.cols);
  };

  if (L <= kUCap) {
    // ---- fast path: gather the bucket's keys into LDS, sort, segment.
    // key' = (dest - lo) << 32 | w << 16 | code
    int base = base0;
    for (int w = w0; w < w1; ++w) {
      const uint32_t pk = A.bmap[(int64_t)b * A.nWG + w];
      const int st = (int)(pk >> 16), cnt = (int)(pk & 0xFFFFu);
      const uint64_t* src = A.sorted + (int64_t)w * A.slotmax + st;
      for (int k = 0; k < cnt; ++k) {
        const uint64_t key = src[k];
        s_list[base++] = (((key >> 32) - (uint64_t)lo) << 32) | ((uint64_t)w << 16) | (key & 0xFFFFu);
      }
    }
    int Lp = 1;
    while (Lp < L) Lp <<= 1;
    for (int s = L + tid; s < Lp; s += blockDim.x) s_list[s] = ~0ull;
    __syncthreads();
    for (int k = 2; k <= Lp; k <<= 1) {
      for (int jj = k >> 1; jj > 0; jj >>= 1) {
        for (int s = tid; s < Lp; s += blockDim.x) {
          const int o = s ^ jj;
          if (o > s) {
            const uint64_t x = s_list[s], y = s_list[o];
            const bool up = (s & k) == 0;
            if ((x > y) == up) { s_list[s] = y; s_list[o] = x; }
          }
        }
        __syncthreads();
      }
    }
    // segment starts (ordered): block scan of head flags
    const int CL = (L + blockDim.x - 1) / blockDim.x;
    const int l0 = tid * CL, l1 = min(L, l0 + CL);
    int heads = 0;
    for (int s = l0; s < l1; ++s)
      heads += (s == 0 || (s_list[s] >> 32) != (s_list[s - 1] >> 32)) ? 1 : 0;
    int nseg;
    int sidx = block_scan_excl(heads, s_w, &nseg);
    for (int s = l0; s < l1; ++s)
      if (s == 0 || (s_list[s] >> 32) != (s_list[s - 1] >> 32)) s_segs[sidx++] = s;
    if (tid == 0) s_segs[nseg] = L;
    __syncthreads();
    for (int sg = wv; sg < nseg; sg += W) {
      const int s0 = s_segs[sg], s1 = s_segs[sg + 1];
      const int64_t dest = lo + (int64_t)(s_list[s0] >> 32);
      if (dest < E_) {
        F E, acc;
        load_row(E, A.ent.row(dest), A.ent.cols);
        acc.zero();
        entity_sum(s_list, s0, s1, E, acc);
        apply_entity(dest, E, acc);
      } else {
        float acc[RV * NC];
#pragma unroll
        for (int q = 0; q < RV * NC; ++q) acc[q] = 0.f;
        rel_sum(s_list, s0, s1, acc);
        apply_rel(dest - E_, acc);
      }
    }
    return;
  }

  // ---- overflow path: destination by destination; waves split the source
  // workgroups (w = wv mod W), partial sums combined in wave order.
  const int64_t d_hi = min<int64_t>(ndest, lo + A.bs);
  for (int64_t dest = lo; dest < d_hi; ++dest) {
    const bool is_ent = dest < E_;
    F E, acc;
    acc.zero();
    E.zero();
    if (is_ent) load_row(E, A.ent.row(dest), A.ent.cols);
    float racc[RV * NC];
#pragma unroll
    for (int q = 0; q < RV * NC; ++q) racc[q] = 0.f;
    bool any = false;
    for (int w = wv; w < A.nWG; w += W) {
      const uint32_t pk = A.bmap[(int64_t)b * A.nWG + w];
      const int st = (int)(pk >> 16), cnt = (int)(pk & 0xFFFFu);
      const uint64_t* src = A.sorted + (int64_t)w * A.slotmax + st;
      for (int k = 0; k < cnt; ++k) {
        const uint64_t key = src[k];
        if ((int64_t)(key >> 32) != dest) continue;
        const uint64_t k2 = ((uint64_t)w << 16) | (key & 0xFFFFu);
        if (is_ent) entity_sum(&k2, 0, 1, E, acc);
        else rel_sum(&k2, 0, 1, racc);
        any = true;
      }
    }
    if (tid == 0) s_flag = 0;
    __syncthreads();
    if (any && lane == 0) atomicOr(&s_flag, 1);
#pragma unroll
    for (int q = 0; q < VEC * NC; ++q) {
      const int c = q / VEC, k = q % VEC;
      const int idx = (c * KGE_WAVE + lane) * VEC + k;
      red[wv * FL + idx] = is_ent ? acc.v[q] : (q < RV * NC ? racc[q] : 0.f);
    }
    __syncthreads();
    if (wv == 0 && s_flag) {
      if (is_ent) {
#pragma unroll
        for (int q = 0; q < VEC * NC; ++q) {
          const int c = q / VEC, k = q % VEC;
          const int idx = (c * KGE_WAVE + lane) * VEC + k;
          float s = 0.f;
          for (int w = 0; w < W; ++w) s += red[w * FL + idx];
          acc.v[q] = s;
        }
        apply_entity(dest, E, acc);
      } else {
#pragma unroll
        for (int q = 0; q < RV * NC; ++q) {
          const int c = q / VEC, k = q % VEC;
          const int idx = (c * KGE_WAVE + lane) * VEC + k;
          float s = 0.f;
          for (int w = 0; w < W; ++w) s += red[w * FL + idx];
          racc[q] = s;
        }
        apply_rel(dest - E_, racc);
      }
    }
    __syncthreads();
  }
}

// ------------------------------------------------------------ dispatch
template <template <int, int, int> class Model, int VEC, int NC, int SK>
static kge_status launch_family(const StepArgs& A, const StepGeom& G, hipStream_t st, hipEvent_t const* ev) {
  hipLaunchKernelGGL((score_kernel<Model, VEC, NC, SK>), dim3(G.nWG), dim3(kStepThreads), G.lds_score, st, A);
  if (ev) (void)hipEventRecord(ev[2], st);
  hipLaunchKernelGGL((update_kernel<Model, VEC, NC, SK>), dim3(A.train ? G.gridU : 1), dim3(kStepThreads),
                     G.lds_update, st, A);
  return KGE_OK;
}

template <template <int, int, int> class Model, int VEC, int NC>
static kge_status by_sk(const StepArgs& A, const StepGeom& G, int sk, hipStream_t st, hipEvent_t const* ev) {
  switch (sk) {
    case SK_P1: return launch_family<Model, VEC, NC, SK_P1>(A, G, st, ev);
    case SK_P2: return launch_family<Model, VEC, NC, SK_P2>(A, G, st, ev);
    case SK_PINF: return launch_family<Model, VEC, NC, SK_PINF>(A, G, st, ev);
    default: return launch_family<Model, VEC, NC, SK_DOT>(A, G, st, ev);
  }
}

template <template <int, int, int> class Model, int VEC, int NC>
static kge_status by_sk_lp(const StepArgs& A, const StepGeom& G, int sk, hipStream_t st, hipEvent_t const* ev) {
  switch (sk) {
    case SK_P1: return launch_family<Model, VEC, NC, SK_P1>(A, G, st, ev);
    case SK_P2: return launch_family<Model, VEC, NC, SK_P2>(A, G, st, ev);
    case SK_PINF: return launch_family<Model, VEC, NC, SK_PINF>(A, G, st, ev);
    default: return KGE_EUNSUPPORTED;
  }
}

// TransE: every score kind, VEC 4 / 1
static kge_status transe(const StepArgs& A, const StepGeom& G, int sk, hipStream_t st, hipEvent_t const* ev) {
  if (G.vec == 4) {
    if (G.nc == 1) return by_sk<TransE, 4, 1>(A, G, sk, st, ev);
    if (G.nc == 2) return by_sk<TransE, 4, 2>(A, G, sk, st, ev);
    return by_sk<TransE, 4, 4>(A, G, sk, st, ev);
  }
  if (G.nc == 1) return by_sk<TransE, 1, 1>(A, G, sk, st, ev);
  if (G.nc == 2) return by_sk<TransE, 1, 2>(A, G, sk, st, ev);
  return by_sk<TransE, 1, 4>(A, G, sk, st, ev);
}

// DistMult: its own trilinear score (score_fn unused), VEC 4 / 1
static kge_status distmult(const StepArgs& A, const StepGeom& G, hipStream_t st, hipEvent_t const* ev) {
  if (G.vec == 4) {
    if (G.nc == 1) return launch_family<DistMult, 4, 1, SK_DOT>(A, G, st, ev);
    if (G.nc == 2) return launch_family<DistMult, 4, 2, SK_DOT>(A, G, st, ev);
    return launch_family<DistMult, 4, 4, SK_DOT>(A, G, st, ev);
  }
  if (G.nc == 1) return launch_family<DistMult, 1, 1, SK_DOT>(A, G, st, ev);
  if (G.nc == 2) return launch_family<DistMult, 1, 2, SK_DOT>(A, G, st, ev);
  return launch_family<DistMult, 1, 4, SK_DOT>(A, G, st, ev);
}

// RotatE: Lp kinds on complex rows, VEC 4 / 2 (a complex pair never splits)
static kge_status rotate(const StepArgs& A, const StepGeom& G, int sk, hipStream_t st, hipEvent_t const* ev) {
  if (G.vec == 4) {
    if (G.nc == 1) return by_sk_lp<RotatE, 4, 1>(A, G, sk, st, ev);
    if (G.nc == 2) return by_sk_lp<RotatE, 4, 2>(A, G, sk, st, ev);
    return by_sk_lp<RotatE, 4, 4>(A, G, sk, st, ev);
  }
  if (G.nc == 1) return by_sk_lp<RotatE, 2, 1>(A, G, sk, st, ev);
  if (G.nc == 2) return by_sk_lp<RotatE, 2, 2>(A, G, sk, st, ev);
  return by_sk_lp<RotatE, 2, 4>(A, G, sk, st, ev);
}

kge_status launch_step_elementwise(const StepArgs& A, const StepGeom& G, int model, int sk,
                                   hipStream_t st, hipEvent_t const* ev) {
  switch (model) {
    case KGE_MODEL_TRANSE: return transe(A, G, sk, st, ev);
    case KGE_MODEL_DISTMULT: return distmult(A, G, st, ev);
    case KGE_MODEL_ROTATE: return rotate(A, G, sk, st, ev);
    default: return KGE_EUNSUPPORTED;
  }
}

}  // namespace kge
