// Fused KGE training step for gfx950 -- element-wise model family.
//
// One reference batch step (KGEModel.__run_single_batch, BaseModel.py:293-330)
// runs as three stream-ordered kernels:
//
//   K0  constrain   full-table row renormalisation of ent_emb when the model's
//                   _constraint_loss assigns it (TransE.py:171-172,
//                   DistMult.py:162-163); one wave per row.
//   KS  score       one workgroup per nP positives. In-register Philox
//                   negative draws (ns_strategy.py:39-64 layout of
//                   BaseModel.py:332-408), gather of the sampled rows (one
//                   row per wave-instruction), wave64 shuffle reductions for
//                   the score (score.py), the loss epilogue in LDS
//                   (loss.py; SANS softmax per positive), then a second pass
//                   over the (L2-hot) rows for the analytic gradient: the
//                   positive's own rows are reduced on chip, the sampled
//                   rows' gradients are NOT scattered -- each negative only
//                   leaves a scalar coefficient, and the workgroup sorts its
//                   entity contributions by destination bucket.
//   KU  update      destination-major: one workgroup per entity bucket
//                   merges every score workgroup's contributions for its
//                   rows, re-derives each negative's row gradient from the
//                   positive's frozen context + the coefficient, sums in
//                   registers, applies clip_by_norm(5) per variable
//                   (BaseModel.py:327, TF-2.5 IndexedSlices semantics: norm
//                   over un-deduplicated slices) and the SGD update
//                   (BaseModel.py:328, keras SGD ResourceScatterAdd) with ONE
//                   plain read-modify-write per touched row -- no float
//                   atomics, deterministic summation order. Extra workgroups
//                   update the relation rows.
#include "kge_models.h"
#include "kge_step.h"

namespace kge {

// ------------------------------------------------------------ K0 constrain
// kind 0: normalized_embeddings(p=2) -> X / pow(sum X^2, 1/2) * value
// kind 1: clip_constraint(p=2)       -> rows with norm >= value rescaled
__global__ __launch_bounds__(256) void constrain_rows_kernel(float* __restrict__ t, int64_t rows,
                                                              int32_t cols, int64_t ld, int kind,
                                                              float value) {
  const int64_t nw = (int64_t)gridDim.x * (blockDim.x / KGE_WAVE);
  for (int64_t r = (int64_t)blockIdx.x * (blockDim.x / KGE_WAVE) + wave_id(); r < rows; r += nw) {
    float* row = t + r * ld;
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

// ------------------------------------------------------------ helpers
__device__ __forceinline__ float log_sigmoid(float x) {
  return fminf(x, 0.f) - log1pf(expf(-fabsf(x)));
}
__device__ __forceinline__ float sigmoid(float x) { return 1.f / (1.f + expf(-x)); }

// slot j of a positive -> (kind, draw index within its side's plane, plane)
__device__ __forceinline__ void slot_layout(int side_mode, int Kside, int64_t i, int j, int* kind,
                                            uint64_t* n, uint64_t* plane_off, int64_t B) {
  if (side_mode == KGE_SIDE_HT) {
    // rows alternate [h-corrupt j/2, t-corrupt j/2] (BaseModel.py:353-356)
    *kind = (j & 1) ? KIND_TC : KIND_HC;
    *n = (uint64_t)(i * Kside + (j >> 1));
    *plane_off = (j & 1);
  } else {
    *kind = side_mode == KGE_SIDE_H ? KIND_HC : KIND_TC;
    *n = (uint64_t)(i * Kside + j);
    *plane_off = 0;
  }
  (void)B;
}

// ------------------------------------------------------------ KS score
template <template <int, int, int> class Model, int VEC, int NC, int SK>
__global__ __launch_bounds__(256) void score_kernel(StepArgs A) {
  using M = Model<VEC, NC, SK>;
  using F = Frag<VEC, NC>;
  constexpr int W = 4;
  constexpr int FL = KGE_WAVE * VEC * NC;   // floats per fragment image
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];

  const int Keff = A.Keff;
  const int nP = A.nP;
  // LDS carve (16-byte aligned pieces)
  float* red = reinterpret_cast<float*>(smem);                       // [W][3][FL]
  float* s_sc = red + W * 3 * FL;                                     // [Keff+1] scores
  float* s_R = s_sc + A.Kpad;                                         // [Keff+1] reduced value
  float* s_M = s_R + A.Kpad;                                          // [Keff+1] max / alpha
  float* s_ti = s_M + A.Kpad;                                         // [Keff+1] ties
  int32_t* s_ids = reinterpret_cast<int32_t*>(s_ti + A.Kpad);         // [nP*Keff]
  float* s_misc = reinterpret_cast<float*>(s_ids + A.idpad);          // [64]
  uint64_t* s_keys = reinterpret_cast<uint64_t*>(s_misc + 64);        // [sortpad]
  int64_t* s_pos = reinterpret_cast<int64_t*>(s_keys + A.sortpad);    // [nP*3]

  const int tid = threadIdx.x, lane = lane_id(), wv = wave_id();
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
    slot_layout(A.side_mode, A.Kside, i, j, &kind, &n, &poff, A.B);
    int64_t e;
    if (A.given) {
      e = load_idx(A.neg_user, i * Keff + j, A.i64);
    } else {
      const int64_t x = load_idx(A.pos, i * 3 + (kind == KIND_HC ? 0 : 2), A.i64);
      if (A.smp.kind == KGE_SAMPLER_TYPED && (x < 0 || x >= A.ent.rows)) { e = 0; err = KGE_ERANGE; }
      else {
        // plane = offset (+1 for the tail side of 'h+t')
        e = sample_entity(A.smp, A.smp.offset + poff, n, x, &err);
        if (e < 0) e = 0;
      }
      if (A.neg_user) store_idx(A.neg_user, i * Keff + j, e, A.i64);
    }
    if (e < 0 || e >= A.ent.rows) { err = KGE_ERANGE; e = 0; }
    s_ids[s] = (int32_t)e;
    if (A.train) A.ids[i * Keff + j] = (int32_t)e;
  }
  __syncthreads();

  F accH, accR, accT;
  for (int p = 0; p < nValid; ++p) {
    const int64_t i = i0 + p;
    const int64_t h = s_pos[p * 3 + 0], r = s_pos[p * 3 + 1], t = s_pos[p * 3 + 2];
    typename M::Ctx ctx;
    M::load_ctx(ctx, A.ent, A.rel, h, r, t, mp);
    const int32_t* ids = s_ids + p * Keff;

    // ---- phase A: scores (slot Keff = the positive, done by the last wave)
    if (wv == W - 1) {
      F a, b, E;
      M::fwd(ctx, KIND_POS, E, a, b);
      const float part = score_partial<SK, M::CPLX>(a, b);
      const float Rv = SK == SK_PINF ? wave_max(part) : wave_sum(part);
      float ti = 1.f;
      if (SK == SK_PINF) ti = wave_sum(tie_partial<M::CPLX>(a, Rv));
      if (lane == 0) { s_R[Keff] = Rv; s_ti[Keff] = ti; }
    }
    constexpr int UN = 4;
    for (int j0 = wv * UN; j0 < Keff; j0 += W * UN) {
      F E[UN];
#pragma unroll
      for (int u = 0; u < UN; ++u)
        if (j0 + u < Keff) load_row(E[u], A.ent.row(ids[j0 + u]), A.ent.cols);
#pragma unroll
      for (int u = 0; u < UN; ++u) {
        const int j = j0 + u;
        if (j >= Keff) break;
        int kind; uint64_t n, poff;
        slot_layout(A.side_mode, A.Kside, i, j, &kind, &n, &poff, A.B);
        F a, b;
        M::fwd(ctx, kind, E[u], a, b);
        const float part = score_partial<SK, M::CPLX>(a, b);
        const float Rv = SK == SK_PINF ? wave_max(part) : wave_sum(part);
        float ti = 1.f;
        if (SK == SK_PINF) ti = wave_sum(tie_partial<M::CPLX>(a, Rv));
        if (lane == 0) { s_R[j] = Rv; s_ti[j] = ti; }
      }
    }
    __syncthreads();

    // ---- loss epilogue (wave 0): coefficients c_j = dL/ds_j -> alpha_j
    if (wv == 0) {
      float lpp;
      const float sp = score_value<SK>(s_R[Keff], A.pw, &lpp);
      // per-lane pass 1: scores + (SANS) max
      float zmax = -INFINITY;
      for (int j = lane; j < Keff; j += KGE_WAVE) {
        float lpj;
        const float sj = score_value<SK>(s_R[j], A.pw, &lpj);
        s_sc[j] = sj;
        s_M[j] = lpj;   // keep lp for alpha
        zmax = fmaxf(zmax, A.temperature * sj);
      }
      zmax = wave_max(zmax);
      float Z = 0.f;
      if (A.loss_kind == KGE_LOSS_SANS)
        for (int j = lane; j < Keff; j += KGE_WAVE) Z += expf(A.temperature * s_sc[j] - zmax);
      Z = wave_sum(Z);
      float lsum = 0.f, csum = 0.f;
      for (int j = lane; j < Keff; j += KGE_WAVE) {
        const float sj = s_sc[j];
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
        const float al = score_alpha<SK>(c, s_R[j], s_M[j], s_ti[j], A.pw);
        const float Mj = s_R[j];
        if (A.train) A.coef[i * Keff + j] = make_float2(al, Mj);
        s_M[j] = Mj;
        s_sc[j] = al;   // alpha (scores already consumed)
        if (A.neg_score_out) A.neg_score_out[i * Keff + j] = sj;
      }
      lsum = wave_sum(lsum);
      csum = wave_sum(csum);
      // DistMult constraint term lambda * mean_i ||r_i||^2 (DistMult.py:164-165)
      float rreg = 0.f;
      if (A.rel_reg != 0.f) {
        F Rr;
        load_row(Rr, A.rel.row(r), A.rel.cols);
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
        s_sc[Keff] = score_alpha<SK>(cp, s_R[Keff], lpp, s_ti[Keff], A.pw);
        s_M[Keff] = s_R[Keff];
        if (A.pos_score_out) A.pos_score_out[i] = sp;
      }
    }
    __syncthreads();

    if (A.train) {
      // ---- phase B: analytic gradients (rows re-read from L2)
      accH.zero(); accR.zero(); accT.zero();
      if (wv == W - 1) {
        F a, b, E;
        M::fwd(ctx, KIND_POS, E, a, b);
        M::bwd(ctx, KIND_POS, E, a, b, s_sc[Keff], s_M[Keff], accH, accR, accT, nrm, mp);
      }
      if (A.rel_reg != 0.f && wv == 0) {
        // its own IndexedSlices block: (lambda / B) * 2 r  (pow-2 gradient)
        F Rr;
        load_row(Rr, A.rel.row(r), A.rel.cols);
        const float gsc = A.rel_reg * A.inv_b;
#pragma unroll
        for (int q = 0; q < VEC * NC; ++q) {
          const float g = gsc * (2.f * Rr.v[q]);
          accR.v[q] += g;
          nrm[1] += g * g;
        }
      }
      for (int j0 = wv * UN; j0 < Keff; j0 += W * UN) {
        F E[UN];
#pragma unroll
        for (int u = 0; u < UN; ++u)
          if (j0 + u < Keff) load_row(E[u], A.ent.row(ids[j0 + u]), A.ent.cols);
#pragma unroll
        for (int u = 0; u < UN; ++u) {
          const int j = j0 + u;
          if (j >= Keff) break;
          int kind; uint64_t n, poff;
          slot_layout(A.side_mode, A.Kside, i, j, &kind, &n, &poff, A.B);
          F a, b;
          M::fwd(ctx, kind, E[u], a, b);
          M::bwd(ctx, kind, E[u], a, b, s_sc[j], s_M[j], accH, accR, accT, nrm, mp);
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
      if (wv == 0) {
        float* sb = A.snap + i * 3 * (int64_t)A.snap_cols;
        M::write_snap(ctx, sb, sb + A.snap_cols, sb + 2 * A.snap_cols, A.snap_cols);
      }
      __syncthreads();
      float* gp = A.gpos + i * 3 * (int64_t)A.gcols;
      for (int e = tid; e < 3 * FL; e += blockDim.x) {
        const int v = e / FL, k = e % FL;
        int cols = v == 1 ? A.rel_gcols : A.ent.cols;
        // RotatE keeps the phase gradient of complex element k in float 2k
        const int src = (v == 1 && A.rel_half) ? 2 * k : k;
        if (k >= cols) continue;
        float s = 0.f;
#pragma unroll
        for (int w = 0; w < W; ++w) s += red[w * 3 * FL + v * FL + src];
        gp[v * A.gcols + k] = s;
      }
      __syncthreads();
    }
  }

  // ---- per-workgroup partials: loss, norm^2 per variable
#pragma unroll
  for (int v = 0; v < 4; ++v) nrm[v] = wave_sum(nrm[v]);
  if (lane == 0) {
#pragma unroll
    for (int v = 0; v < 4; ++v) s_misc[wv * 4 + v] = nrm[v];
  }
  if (err) set_status(A.status, err);
  __syncthreads();
  if (tid == 0) {
    float* pt = A.part + (int64_t)blockIdx.x * 8;
    pt[0] = loss_acc;
#pragma unroll
    for (int v = 0; v < 4; ++v) {
      float s = 0.f;
      for (int w = 0; w < W; ++w) s += s_misc[w * 4 + v];
      pt[1 + v] = s;
    }
  }
  if (!A.train) return;

  // ---- bucket the workgroup's entity contributions by destination
  // key = entity << 32 | code; code < nP*Keff: negative slot, else positive
  // h / t vector (nP*Keff + 2p + {0,1}).
  const int nNeg = nValid * Keff;
  const int nEnt = nNeg + 2 * nValid;
  for (int s = tid; s < A.sortpad; s += blockDim.x) {
    uint64_t key = ~0ull;
    if (s < nNeg) key = ((uint64_t)(uint32_t)s_ids[s] << 32) | (uint32_t)s;
    else if (s < nEnt) {
      const int q = s - nNeg, p = q >> 1;
      const int64_t e = s_pos[p * 3 + ((q & 1) ? 2 : 0)];
      key = ((uint64_t)(uint32_t)e << 32) | (uint32_t)(nP * Keff + q);
    }
    s_keys[s] = key;
  }
  __syncthreads();
  // bitonic sort (ascending) of sortpad (power of two) keys
  for (int k = 2; k <= A.sortpad; k <<= 1) {
    for (int jj = k >> 1; jj > 0; jj >>= 1) {
      for (int s = tid; s < A.sortpad; s += blockDim.x) {
        const int o = s ^ jj;
        if (o > s) {
          const uint64_t x = s_keys[s], y = s_keys[o];
          const bool up = (s & k) == 0;
          if ((x > y) == up) { s_keys[s] = y; s_keys[o] = x; }
        }
      }
      __syncthreads();
    }
  }
  uint64_t* out = A.sorted + (int64_t)blockIdx.x * A.slotmax;
  for (int s = tid; s < nEnt; s += blockDim.x) out[s] = s_keys[s];
  // starts[b] = first index with entity >= b*bs   (b = 0..P)
  int32_t* st = A.starts + (int64_t)blockIdx.x * (A.P + 1);
  for (int b = tid; b <= A.P; b += blockDim.x) {
    const uint64_t lo = (uint64_t)((int64_t)b * A.bs) << 32;
    int l = 0, hgh = nEnt;
    while (l < hgh) {
      const int m = (l + hgh) >> 1;
      if (s_keys[m] < lo) l = m + 1; else hgh = m;
    }
    st[b] = l;
  }
}

// relation-row fragments: full layout, or RotatE's half layout
template <bool HALF, int VEC, int NC>
__device__ __forceinline__ void load_rel_row(float (&v)[(HALF ? (VEC / 2 > 0 ? VEC / 2 : 1) : VEC) * NC],
                                             const float* row, int cols) {
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
__device__ __forceinline__ void store_rel_row(const float (&v)[(HALF ? (VEC / 2 > 0 ? VEC / 2 : 1) : VEC) * NC],
                                              float* row, int cols) {
  if constexpr (HALF) {
    store_row_half<VEC, NC>(v, row, cols);
  } else {
    Frag<VEC, NC> f;
#pragma unroll
    for (int q = 0; q < VEC * NC; ++q) f.v[q] = v[q];
    store_row(f, row, cols);
  }
}

// ------------------------------------------------------------ KU update
// blocks [0, P): entity buckets; [P, P + Pr): relation groups (one wave per
// relation). Block 0 also reduces the loss.
template <template <int, int, int> class Model, int VEC, int NC, int SK>
__global__ __launch_bounds__(256) void update_kernel(StepArgs A) {
  using M = Model<VEC, NC, SK>;
  using F = Frag<VEC, NC>;
  constexpr int W = 4;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  uint64_t* s_list = reinterpret_cast<uint64_t*>(smem);                   // [cap]
  int32_t* s_cnt = reinterpret_cast<int32_t*>(s_list + A.ucap);           // [256+1]
  float* s_red = reinterpret_cast<float*>(s_cnt + 264);                   // [W][FL] + misc
  __shared__ float s_scale[4];
  __shared__ int s_seg[2];

  const int tid = threadIdx.x, lane = lane_id(), wv = wave_id();
  constexpr int FL = KGE_WAVE * VEC * NC;

  // clip_by_norm scale per variable: clip / max(||g||, clip)
  if (wv == 0) {
    for (int v = 0; v < 4; ++v) {
      float s = 0.f;
      for (int w = lane; w < A.nWG; w += KGE_WAVE) s += A.part[(int64_t)w * 8 + 1 + v];
      s = wave_sum(s);
      if (lane == 0) {
        const float n = sqrtf(s);
        s_scale[v] = -A.lr * (A.clip_norm / fmaxf(n, A.clip_norm));
        if (blockIdx.x == 0 && A.norm2_out) A.norm2_out[v] = s;
      }
    }
    if (blockIdx.x == 0) {
      float l = 0.f;
      for (int w = lane; w < A.nWG; w += KGE_WAVE) l += A.part[(int64_t)w * 8];
      l = wave_sum(l);
      if (lane == 0) {
        A.loss_out[0] = l;
        if (A.loss_accum) A.loss_accum[0] += l;
      }
    }
  }
  __syncthreads();
  if (!A.train) return;

  if ((int)blockIdx.x >= A.P) {
    // ---------------- relation rows: one wave per relation, positives in order
    const int64_t r = (int64_t)(blockIdx.x - A.P) * W + wv;
    if (r >= A.rel.rows) return;
    // RotatE phase rows use the half-width layout (phase k beside complex k)
    constexpr int RV = M::CPLX ? (VEC / 2 > 0 ? VEC / 2 : 1) : VEC;
    float acc[RV * NC];
#pragma unroll
    for (int q = 0; q < RV * NC; ++q) acc[q] = 0.f;
    bool any = false;
    for (int64_t i0 = 0; i0 < A.B; i0 += KGE_WAVE) {
      const int64_t i = i0 + lane;
      bool m = false;
      if (i < A.B) m = load_idx(A.pos, i * 3 + 1, A.i64) == r;
      unsigned long long bal = __ballot(m);
      while (bal) {
        const int l = __ffsll((long long)bal) - 1;
        bal &= bal - 1;
        const float* g = A.gpos + (i0 + l) * 3 * (int64_t)A.gcols + A.gcols;
        float gv[RV * NC];
        load_rel_row<M::CPLX, VEC, NC>(gv, g, A.rel_gcols);
#pragma unroll
        for (int q = 0; q < RV * NC; ++q) acc[q] += gv[q];
        any = true;
      }
    }
    if (!any) return;
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
    return;
  }

  // ---------------- entity bucket b
  const int b = blockIdx.x;
  const int64_t e_lo = (int64_t)b * A.bs;
  // per-source-workgroup counts and a deterministic exclusive scan
  int local = 0;
  for (int w = tid; w < A.nWG; w += blockDim.x) {
    const int32_t* st = A.starts + (int64_t)w * (A.P + 1);
    local += st[b + 1] - st[b];
  }
  // block scan of per-thread totals (thread order == w order within thread)
  s_cnt[tid] = local;
  __syncthreads();
  if (tid == 0) {
    int run = 0;
    for (int k = 0; k < (int)blockDim.x; ++k) { const int c = s_cnt[k]; s_cnt[k] = run; run += c; }
    s_cnt[blockDim.x] = run;
  }
  __syncthreads();
  const int L = s_cnt[blockDim.x];
  if (L == 0) return;

  const int Kn = A.nP * A.Keff;   // code boundary between negative and positive entries
  auto apply_entry = [&](uint64_t key, const F& E, F& acc) {
    const uint32_t lo = (uint32_t)key;
    const int w = (int)(lo >> 16), code = (int)(lo & 0xFFFF);
    if (code < Kn) {
      const int p = code / A.Keff, j = code % A.Keff;
      const int64_t i = (int64_t)w * A.nP + p;
      int kind; uint64_t n, poff;
      slot_layout(A.side_mode, A.Kside, i, j, &kind, &n, &poff, A.B);
      const float2 cf = A.coef[i * A.Keff + j];
      const float* sb = A.snap + i * 3 * (int64_t)A.snap_cols;
      F g;
      M::grad_entity(sb, sb + A.snap_cols, sb + 2 * A.snap_cols, A.snap_cols, kind, E, cf.x, cf.y, g);
      add_to(acc, g);
    } else {
      const int q = code - Kn, p = q >> 1;
      const int64_t i = (int64_t)w * A.nP + p;
      F g;
      load_row(g, A.gpos + i * 3 * (int64_t)A.gcols + ((q & 1) ? 2 * A.gcols : 0), A.ent.cols);
      add_to(acc, g);
    }
  };

  if (L <= A.ucap) {
    // fast path: gather the bucket's entries into LDS, sort, segment.
    // key' = (entity - e_lo) << 32 | w << 16 | code
    int base = s_cnt[tid];
    for (int w = tid; w < A.nWG; w += blockDim.x) {
      const int32_t* st = A.starts + (int64_t)w * (A.P + 1);
      const int s0 = st[b], s1 = st[b + 1];
      const uint64_t* src = A.sorted + (int64_t)w * A.slotmax;
      for (int k = s0; k < s1; ++k) {
        const uint64_t key = src[k];
        const uint64_t ent = (key >> 32) - (uint64_t)e_lo;
        s_list[base++] = (ent << 32) | ((uint64_t)w << 16) | (key & 0xFFFF);
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
    // segment heads -> each wave walks the list and owns every W-th segment
    int seg = 0;
    for (int s0 = 0; s0 < L;) {
      const uint32_t ent = (uint32_t)(s_list[s0] >> 32);
      // segment end: first index with a different entity (wave-parallel scan)
      int s1 = s0 + 1;
      while (s1 < L) {
        const int idx = s1 + lane;
        const bool diff = idx < L ? (uint32_t)(s_list[idx] >> 32) != ent : true;
        const unsigned long long bal = __ballot(diff);
        if (bal) { s1 += __ffsll((long long)bal) - 1; break; }
        s1 += KGE_WAVE;
      }
      if ((seg % W) == wv) {
        const int64_t e = e_lo + ent;
        F E, acc;
        load_row(E, A.ent.row(e), A.ent.cols);
        acc.zero();
        for (int s = s0; s < s1; ++s) apply_entry(s_list[s], E, acc);
        if (A.grad_mode) {
          store_row(acc, A.gent + e * (int64_t)A.ent.cols, A.ent.cols);
          ++seg;
          s0 = s1;
          continue;
        }
        const float sc = s_scale[0];
#pragma unroll
        for (int q = 0; q < VEC * NC; ++q) E.v[q] = E.v[q] + acc.v[q] * sc;
        store_row(E, A.ent.row_w(e), A.ent.cols);
      }
      ++seg;
      s0 = s1;
    }
    return;
  }

  // slow path (bucket overflow): entity by entity, waves split the sources
  const int64_t e_hi = min<int64_t>(A.ent.rows, e_lo + A.bs);
  float* red = s_red;
  for (int64_t e = e_lo; e < e_hi; ++e) {
    F E, acc;
    load_row(E, A.ent.row(e), A.ent.cols);
    acc.zero();
    bool any = false;
    for (int w = wv; w < A.nWG; w += W) {
      const int32_t* st = A.starts + (int64_t)w * (A.P + 1);
      const uint64_t* src = A.sorted + (int64_t)w * A.slotmax;
      int l = st[b], hgh = st[b + 1];
      const uint64_t lo = (uint64_t)e << 32;
      while (l < hgh) { const int m = (l + hgh) >> 1; if (src[m] < lo) l = m + 1; else hgh = m; }
      for (int k = l; k < st[b + 1] && (src[k] >> 32) == (uint64_t)e; ++k) {
        const uint64_t key = src[k];
        apply_entry(((uint64_t)0 << 32) | ((uint64_t)w << 16) | (key & 0xFFFF), E, acc);
        any = true;
      }
    }
    // cross-wave sum
#pragma unroll
    for (int q = 0; q < VEC * NC; ++q) {
      const int c = q / VEC, k = q % VEC;
      red[wv * FL + (c * KGE_WAVE + lane) * VEC + k] = acc.v[q];
    }
    if (lane == 0) s_seg[0] = 0;
    __syncthreads();
    if (any && lane == 0) atomicOr(&s_seg[0], 1);
    __syncthreads();
    if (wv == 0 && s_seg[0]) {
#pragma unroll
      for (int q = 0; q < VEC * NC; ++q) {
        const int c = q / VEC, k = q % VEC;
        const int idx = (c * KGE_WAVE + lane) * VEC + k;
        float s = 0.f;
        for (int w = 0; w < W; ++w) s += red[w * FL + idx];
        if (A.grad_mode) E.v[q] = s;
        else E.v[q] = E.v[q] + s * s_scale[0];
      }
      store_row(E, A.grad_mode ? A.gent + e * (int64_t)A.ent.cols : A.ent.row_w(e), A.ent.cols);
    }
    __syncthreads();
  }
}

// ------------------------------------------------------------ dispatch
template <template <int, int, int> class Model, int VEC, int NC, int SK>
static kge_status launch_family(const StepArgs& A, const StepGeom& G, hipStream_t st, hipEvent_t const* ev) {
  hipLaunchKernelGGL((score_kernel<Model, VEC, NC, SK>), dim3(G.nWG), dim3(256), G.lds_score, st, A);
  if (ev) (void)hipEventRecord(ev[2], st);
  hipLaunchKernelGGL((update_kernel<Model, VEC, NC, SK>), dim3(A.train ? G.gridU : 1), dim3(256),
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
