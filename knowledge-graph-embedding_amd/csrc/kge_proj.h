// Projection-family fused training step for gfx950: TransH (TransH.py:149-213)
// and TransD (TransD.py:170-242).
//
// Both models project every entity row of a triple through a per-relation
// rank-1 map before scoring s(P(h) + r, P(t)):
//   TransH  P(e) = e - (w_r . e) w_r                     (w_r = rel_hyper[r])
//   TransD  P(e) = clip(r_p (e_p . e) + I e)             (e_p = ent_proj[e],
//                  r_p = rel_proj[r], I the [k, d] identity; clip to norm <= 1
//                  when `constraint`, constraint.py:70-99)
// so the projection is element-wise work plus one or two wave reductions per
// row -- VALU, no MFMA. One workgroup (4 waves) owns one positive:
//
//   setup     slot ids (in-register Philox draws, ns_strategy.py:39-64), the
//             positive's rows and their projections, kept in registers
//   forward   each wave streams its slots in batches of U rows (all U rows'
//             loads issued first), projects them with batched (transposed)
//             reductions, scores; per-slot value / dot / norm to LDS
//   weights   one wave: loss terms and dL/ds per slot (IEEE transcendentals;
//             each weight decided once, the backward reuses it)
//   backward  the same batches again (rows re-read from L2): gradients in the
//             projected space, back through the clip and the projection, every
//             slice's norm^2 (clip_by_norm sees IndexedSlices, BaseModel.py:327);
//             each negative's entity-row gradient(s) materialised at gneg[code]
//             (and gnegp[code], TransD ent_proj); the positive's rows
//             accumulated in registers, merged over the 4 waves in wave order
//   keys      every destination key filed into its list (kge_step_impl.h bin_key)
//
// The update passes are the shared destination-major kernel in its
// materialised mode: the aux tables first (TransD ent_proj + rel_proj, TransH
// rel_hyper) over the same lists without clearing them, then ent_emb +
// rel_emb. TransH with `constraint` has dense gradients (soft_constraint over
// every entity row, the orthogonality term over every relation,
// TransH.py:200-211): the passes write summed gradients, transh_dense_kernel
// adds the dense terms and reduces the dense norms, apply_kernel clips / SGDs.
#pragma once
#include "kge_step_impl.h"

namespace kge {

constexpr int kPjWaves = 4;
constexpr int kPjThreads = kPjWaves * KGE_WAVE;

struct PjArgs {
  TabView raux;     // TransH rel_hyper [R, d] / TransD rel_proj [R, k]
  TabView eaux;     // TransD ent_proj [E, d]
  float* gnegp;     // TransD: [B << kshift, d] negatives' ent_proj row gradients
  float* gpos2;     // [B, 3, gcols] the positive's aux rows: TransH row 1 = rel_hyper;
                    // TransD 0 = ent_proj[h], 1 = rel_proj[r], 2 = ent_proj[t]
  bool clip;        // TransD `constraint`: projected rows clipped to norm <= 1
  int32_t kmin;     // TransD: min(d, k), the identity block of r_p e_p^T + I
};

// LDS carve (floats) of proj_kernel
struct PjLds {
  int ids, sR, sT, sS, sA, sD, sN, mrg, wn, misc, total;
};
__host__ __device__ inline PjLds pj_lds(int K, int FL, bool td) {
  PjLds L;
  int o = 0;
  auto take = [&](int n) { const int r = o; o += (n + 3) & ~3; return r; };
  L.ids = take(K);
  L.sR = take(K + 1);
  L.sT = take(K + 1);
  L.sS = take(K + 1);
  L.sA = take(K + 1);
  L.sD = take(K);
  L.sN = take(K);
  L.mrg = take(kPjWaves * (td ? 6 : 4) * FL);   // every wave's accumulator images
  L.wn = take(kPjWaves * 4);
  L.misc = take(16);
  L.total = o;
  return L;
}

// N wave-wide sums (N a power of two <= 16), every lane gets every sum:
// one transposed multi-reduction, then a readlane per value
template <int N, bool MAX = false>
__device__ __forceinline__ void wave_sums(float (&x)[N]) {
  if constexpr (N == 1) {
    x[0] = lane_reduce<5, MAX>(x[0]);
  } else {
    constexpr int SH = N == 2 ? 5 : N == 4 ? 4 : N == 8 ? 3 : 2;
    const float r = multi_reduce<N, MAX>(x);
#pragma unroll
    for (int u = 0; u < N; ++u) x[u] = bcast(r, u << SH);
  }
}

template <int VEC, int NC>
__device__ __forceinline__ float dot_partial(const Frag<VEC, NC>& a, const Frag<VEC, NC>& b) {
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < VEC * NC; ++i) s += a.v[i] * b.v[i];
  return s;
}

// TransD identity block: element e < kmin of the row
template <int VEC, int NC>
__device__ __forceinline__ float id_mask(int i, int kmin) {
  return frag_elem<VEC>(i / VEC, i % VEC) < kmin ? 1.f : 0.f;
}

// Projections of N rows E[u] (TransD: with their ent_proj rows Q[u]) through
// the relation's aux row W. Returns P[u] (clipped), dt[u] (w.e or e_p.e) and
// nr[u] (TransD pre-clip norm).
template <bool TD, int N, int VEC, int NC>
__device__ __forceinline__ void project_rows(const Frag<VEC, NC> (&E)[N], const Frag<VEC, NC> (&Q)[N],
                                             const Frag<VEC, NC>& W, const PjArgs& P, Frag<VEC, NC> (&Pr)[N],
                                             float (&dt)[N], float (&nr)[N]) {
#pragma clang fp contract(off)
#pragma unroll
  for (int u = 0; u < N; ++u) dt[u] = TD ? dot_partial(Q[u], E[u]) : dot_partial(W, E[u]);
  wave_sums<N>(dt);
#pragma unroll
  for (int u = 0; u < N; ++u) {
#pragma unroll
    for (int i = 0; i < VEC * NC; ++i) {
      if (TD) Pr[u].v[i] = W.v[i] * dt[u] + id_mask<VEC, NC>(i, P.kmin) * E[u].v[i];
      else Pr[u].v[i] = E[u].v[i] - dt[u] * W.v[i];
    }
    nr[u] = 0.f;
  }
  if (TD) {
#pragma unroll
    for (int u = 0; u < N; ++u) nr[u] = sq_partial(Pr[u]);
    wave_sums<N>(nr);
#pragma unroll
    for (int u = 0; u < N; ++u) {
      nr[u] = sqrtf(nr[u]);
      if (P.clip && !(nr[u] < 1.f)) {
        const float dv = fmaxf(nr[u], 1e-9f);
#pragma unroll
        for (int i = 0; i < VEC * NC; ++i) Pr[u].v[i] = Pr[u].v[i] / dv;
      }
    }
  }
}

// the same projection from a stored dot / norm (no reductions; identical bits)
template <bool TD, int VEC, int NC>
__device__ __forceinline__ void reproject(const Frag<VEC, NC>& E, const Frag<VEC, NC>& W, float dt, float nr,
                                          const PjArgs& P, Frag<VEC, NC>& Pr) {
#pragma clang fp contract(off)
#pragma unroll
  for (int i = 0; i < VEC * NC; ++i) {
    if (TD) Pr.v[i] = W.v[i] * dt + id_mask<VEC, NC>(i, P.kmin) * E.v[i];
    else Pr.v[i] = E.v[i] - dt * W.v[i];
  }
  if (TD && P.clip && !(nr < 1.f)) {
    const float dv = fmaxf(nr, 1e-9f);
#pragma unroll
    for (int i = 0; i < VEC * NC; ++i) Pr.v[i] = Pr.v[i] / dv;
  }
}

// Back through the projection of ONE row for NS rows at once: gP[s] is
// dL/dP (projected space) of row s with raw row E[s] (TransD: ent_proj row
// Q[s]), projected row Pr[s], dot dt[s] and pre-clip norm nr[s]. Produces the
// entity-row gradient gE[s], TransD's ent_proj gradient gQ[s], and adds the
// relation aux row's slice term of row s to gW[s]:
//   TransH  gE = g - (w.g) w ;           gW += -(w.e) g - (w.g) e
//   TransD  g' = clip'(g) ; gE = I^T g' + e_p (r_p.g') ; gQ = e (r_p.g') ;
//           gW += (e_p.e) g'
template <bool TD, int NS, int VEC, int NC>
__device__ __forceinline__ void project_back(Frag<VEC, NC> (&gP)[NS], const Frag<VEC, NC>* const (&E)[NS],
                                             const Frag<VEC, NC>* const (&Q)[NS], const Frag<VEC, NC>* const (&Pr)[NS],
                                             const float (&dt)[NS], const float (&nr)[NS], const Frag<VEC, NC>& W,
                                             const PjArgs& P, Frag<VEC, NC> (&gE)[NS], Frag<VEC, NC> (&gQ)[NS],
                                             Frag<VEC, NC> (&gW)[NS]) {
  float s[NS];
  if (TD) {
    // through clip_constraint: rows with norm >= 1 were divided by it
    if (P.clip) {
#pragma unroll
      for (int u = 0; u < NS; ++u) s[u] = dot_partial(gP[u], *Pr[u]);
      wave_sums<NS>(s);
#pragma unroll
      for (int u = 0; u < NS; ++u) {
        if (!(nr[u] < 1.f)) {
#pragma unroll
          for (int i = 0; i < VEC * NC; ++i) gP[u].v[i] = (gP[u].v[i] - s[u] * Pr[u]->v[i]) / nr[u];
        }
      }
    }
#pragma unroll
    for (int u = 0; u < NS; ++u) s[u] = dot_partial(W, gP[u]);
    wave_sums<NS>(s);
#pragma unroll
    for (int u = 0; u < NS; ++u) {
#pragma unroll
      for (int i = 0; i < VEC * NC; ++i) {
        gE[u].v[i] = id_mask<VEC, NC>(i, P.kmin) * gP[u].v[i] + Q[u]->v[i] * s[u];
        gQ[u].v[i] = E[u]->v[i] * s[u];
        gW[u].v[i] += dt[u] * gP[u].v[i];
      }
    }
  } else {
#pragma unroll
    for (int u = 0; u < NS; ++u) s[u] = dot_partial(W, gP[u]);
    wave_sums<NS>(s);
#pragma unroll
    for (int u = 0; u < NS; ++u) {
#pragma unroll
      for (int i = 0; i < VEC * NC; ++i) {
        gE[u].v[i] = gP[u].v[i] - s[u] * W.v[i];
        gW[u].v[i] += -(dt[u] * gP[u].v[i]) - s[u] * E[u]->v[i];
      }
    }
  }
}

// element gradients of the score wrt x and y (a = x - y for the Lp kinds)
template <int SK, int VEC, int NC>
__device__ __forceinline__ void score_xy_grad(const Frag<VEC, NC>& x, const Frag<VEC, NC>& y, float alpha, float M,
                                              Frag<VEC, NC>& gx, Frag<VEC, NC>& gy) {
  if (SK == SK_DOT) {
#pragma unroll
    for (int i = 0; i < VEC * NC; ++i) { gx.v[i] = alpha * y.v[i]; gy.v[i] = alpha * x.v[i]; }
  } else {
    Frag<VEC, NC> a;
#pragma unroll
    for (int i = 0; i < VEC * NC; ++i) a.v[i] = x.v[i] - y.v[i];
    score_grad<SK, false>(a, alpha, M, gx);
#pragma unroll
    for (int i = 0; i < VEC * NC; ++i) gy.v[i] = -gx.v[i];
  }
}

template <int SK, int VEC, int NC>
__device__ __forceinline__ float score_xy_partial(const Frag<VEC, NC>& x, const Frag<VEC, NC>& y, float p) {
  if (SK == SK_DOT) return dot_partial(x, y);
  Frag<VEC, NC> a;
#pragma unroll
  for (int i = 0; i < VEC * NC; ++i) a.v[i] = x.v[i] - y.v[i];
  return score_partial<SK, false>(a, a, p);
}

template <int VEC, int NC>
__device__ __forceinline__ void stash(const Frag<VEC, NC>& f, float* img) {
#pragma unroll
  for (int q = 0; q < VEC * NC; ++q) img[frag_elem<VEC>(q / VEC, q % VEC)] = f.v[q];
}

template <bool TD, int VEC, int NC, int SK>
__global__ __launch_bounds__(kPjThreads) void proj_kernel(StepArgs A, PjArgs P) {
  if (ws_refused(A.ctl, A.sig, A.status, A.loss_out)) return;
  using F = Frag<VEC, NC>;
  constexpr int FL = KGE_WAVE * VEC * NC;
  constexpr int U = NC == 1 ? 4 : 2;                 // slots per batch
  constexpr int NACC = TD ? 6 : 4;
  extern __shared__ __attribute__((aligned(16))) float sm[];
  __shared__ int s_last;
  const int K = A.Keff;
  const PjLds L = pj_lds(K, FL, TD);
  int32_t* ids = reinterpret_cast<int32_t*>(sm + L.ids);
  float* sR = sm + L.sR;
  float* sT = sm + L.sT;
  float* sS = sm + L.sS;
  float* sA = sm + L.sA;
  float* sD = sm + L.sD;
  float* sN = sm + L.sN;
  float* misc = sm + L.misc;

  const int tid = threadIdx.x, lane = lane_id(), wv = wave_id();
  const int64_t i = blockIdx.x;
  int err = 0;
  int64_t ph = load_idx(A.pos, i * 3 + 0, A.i64);
  int64_t pr = load_idx(A.pos, i * 3 + 1, A.i64);
  int64_t pt = load_idx(A.pos, i * 3 + 2, A.i64);
  ph = ent_row(A, ph, &err);
  if (pr < 0 || pr >= A.rel.rows) { err = KGE_ERANGE; pr = 0; }
  pt = ent_row(A, pt, &err);
  for (int j = tid; j < K; j += kPjThreads) ids[j] = slot_entity(A, i, j, &err);

  // ---- the positive's rows and projections (every wave keeps its own copy)
  F H, T, Rv, W, QH, QT;
  load_row(H, A.ent.row(ph), A.ent.cols);
  load_row(T, A.ent.row(pt), A.ent.cols);
  load_row(Rv, A.rel.row(pr), A.rel.cols);
  load_row(W, P.raux.row(pr), P.raux.cols);
  if (TD) {
    load_row(QH, P.eaux.row(ph), P.eaux.cols);
    load_row(QT, P.eaux.row(pt), P.eaux.cols);
  } else {
    QH.zero();
    QT.zero();
  }
  F PH, PT;        // projected (clipped) h and t
  float dth, dtt, nrh, nrt;
  {
    const F E2[2] = {H, T};
    const F Q2[2] = {QH, QT};
    F P2[2];
    float d2[2], n2[2];
    project_rows<TD, 2>(E2, Q2, W, P, P2, d2, n2);
    PH = P2[0]; PT = P2[1];
    dth = d2[0]; dtt = d2[1]; nrh = n2[0]; nrt = n2[1];
  }
  F X;             // x side of the positive / t-corrupted triples: P(h) + r
#pragma unroll
  for (int q = 0; q < VEC * NC; ++q) X.v[q] = PH.v[q] + Rv.v[q];
  __syncthreads();   // ids

  // ---- forward: scores of the negatives (wave w: batches w, w + 4, ...)
  for (int q0 = wv * U; q0 < K; q0 += kPjWaves * U) {
    int qq[U];
    F E[U], Q[U], Pr[U];
    float dt[U], nr[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      qq[u] = min(q0 + u, K - 1);
      const int64_t e = ids[qq[u]];
      load_row(E[u], A.ent.row(e), A.ent.cols);
      if (TD) load_row(Q[u], P.eaux.row(e), P.eaux.cols);
      else Q[u].zero();
    }
    project_rows<TD, U>(E, Q, W, P, Pr, dt, nr);
    float part[U];
    F x[U], y[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const bool hc = slot_kind(A.side_mode, qq[u]) == KIND_HC;
#pragma unroll
      for (int q = 0; q < VEC * NC; ++q) {
        x[u].v[q] = hc ? Pr[u].v[q] + Rv.v[q] : X.v[q];
        y[u].v[q] = hc ? PT.v[q] : Pr[u].v[q];
      }
      part[u] = score_xy_partial<SK>(x[u], y[u], A.p);
    }
    wave_sums<U, SK == SK_PINF>(part);
    float tq[U];
#pragma unroll
    for (int u = 0; u < U; ++u) tq[u] = 1.f;
    if (SK == SK_PINF) {
#pragma unroll
      for (int u = 0; u < U; ++u) {
        F a;
#pragma unroll
        for (int q = 0; q < VEC * NC; ++q) a.v[q] = x[u].v[q] - y[u].v[q];
        tq[u] = tie_partial<false>(a, part[u]);
      }
      wave_sums<U>(tq);
    }
    if (lane == 0) {
#pragma unroll
      for (int u = 0; u < U; ++u) {
        if (q0 + u < K) {
          float lp;
          sR[q0 + u] = part[u];
          sT[q0 + u] = tq[u];
          sS[q0 + u] = score_value<SK>(part[u], A.pw, &lp, A.p);
          sD[q0 + u] = dt[u];
          sN[q0 + u] = nr[u];
        }
      }
    }
  }
  // the positive's score (wave 0)
  if (wv == 0) {
    float part[1] = {score_xy_partial<SK>(X, PT, A.p)};
    wave_sums<1, SK == SK_PINF>(part);
    float tq = 1.f;
    if (SK == SK_PINF) {
      F a;
#pragma unroll
      for (int q = 0; q < VEC * NC; ++q) a.v[q] = X.v[q] - PT.v[q];
      tq = lane_reduce<5, false>(tie_partial<false>(a, part[0]));
    }
    if (lane == 0) {
      float lp;
      sR[K] = part[0];
      sT[K] = tq;
      sS[K] = score_value<SK>(part[0], A.pw, &lp, A.p);
    }
  }
  __syncthreads();

  // ---- loss and dL/ds per triple (one wave, IEEE transcendentals)
  if (wv == 0) {
    const float sp = sS[K];
    const bool sans = A.loss_kind == KGE_LOSS_SANS;
    float Ms = -INFINITY;
    if (sans)
      for (int q = lane; q < K; q += KGE_WAVE) Ms = fmaxf(Ms, A.temperature * sS[q]);
    Ms = lane_reduce<5, true>(Ms);
    float Z = 0.f;
    if (sans)
      for (int q = lane; q < K; q += KGE_WAVE) Z += expf(A.temperature * sS[q] - Ms);
    Z = lane_reduce<5, false>(Z);
    const float invZ = sans ? (Z > 0.f ? 1.f / Z : 0.f) : 1.f;
    float lneg = 0.f, csum = 0.f;
    for (int q = lane; q < K; q += KGE_WAVE) {
      const float s = sS[q];
      float lp;
      score_value<SK>(sR[q], A.pw, &lp, A.p);
      const float c = neg_coef(A, s, sp, Ms, invZ);
      sA[q] = score_alpha<SK>(c, sR[q], lp, sT[q], A.pw, A.p);
      csum += c;
      switch (A.loss_kind) {
        case KGE_LOSS_HINGE: lneg += fmaxf(A.margin + s - sp, 0.f); break;
        case KGE_LOSS_LOGISTIC: lneg += logf(1.f + expf(s - sp)); break;
        case KGE_LOSS_BCE: lneg += log_sigmoid(-s); break;
        case KGE_LOSS_SANS: lneg += expf(A.temperature * s - Ms) * invZ * log_sigmoid(-s - A.margin); break;
        default: lneg += s * s; break;
      }
    }
    lneg = lane_reduce<5, false>(lneg);
    csum = lane_reduce<5, false>(csum);
    if (lane == 0) {
      float lossp, cp;
      switch (A.loss_kind) {
        case KGE_LOSS_HINGE: lossp = lneg * A.inv_bk; cp = -csum; if (K == 0) lossp = NAN; break;
        case KGE_LOSS_LOGISTIC: lossp = lneg; cp = -csum; break;
        case KGE_LOSS_BCE: lossp = -(log_sigmoid(sp) + lneg) * A.inv_b; cp = -sigmoid(-sp) * A.inv_b; break;
        case KGE_LOSS_SANS:
          lossp = -(log_sigmoid(sp + A.margin) + lneg) * A.inv_b;
          cp = -sigmoid(-(sp + A.margin)) * A.inv_b;
          break;
        default: lossp = ((sp - 1.f) * (sp - 1.f) + lneg) * 0.5f * A.inv_b; cp = (sp - 1.f) * A.inv_b; break;
      }
      float lpp;
      score_value<SK>(sR[K], A.pw, &lpp, A.p);
      sA[K] = score_alpha<SK>(cp, sR[K], lpp, sT[K], A.pw, A.p);
      misc[0] = lossp;
      if (A.pos_score_out) A.pos_score_out[i] = sp;
    }
  }
  if (A.neg_score_out)
    for (int q = tid; q < K; q += kPjThreads) A.neg_score_out[i * K + q] = sS[q];
  __syncthreads();

  // per-lane slice norm^2: 0 ent_emb, 1 rel_emb, 2 rel aux (rel_hyper / rel_proj), 3 ent_proj
  float nrm[4] = {0.f, 0.f, 0.f, 0.f};
  if (A.train) {
    F accH, accT, accR, accW, accQH, accQT;
    accH.zero(); accT.zero(); accR.zero(); accW.zero(); accQH.zero(); accQT.zero();
    // ---- backward over the same batches
    for (int q0 = wv * U; q0 < K; q0 += kPjWaves * U) {
      int qq[U];
      bool hc[U];
      F E[U], Q[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        qq[u] = min(q0 + u, K - 1);
        hc[u] = slot_kind(A.side_mode, qq[u]) == KIND_HC;
        const int64_t e = ids[qq[u]];
        load_row(E[u], A.ent.row(e), A.ent.cols);
        if (TD) load_row(Q[u], P.eaux.row(e), P.eaux.cols);
        else Q[u].zero();
      }
      F Pr[U];
      float dtn[U], nrn[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        dtn[u] = sD[qq[u]];
        nrn[u] = sN[qq[u]];
        reproject<TD>(E[u], W, dtn[u], nrn[u], P, Pr[u]);
      }
      // projected-space gradients: side 0 = x (head) row, side 1 = y (tail) row
      F g[2 * U];
      const F* er[2 * U];
      const F* qr[2 * U];
      const F* pp[2 * U];
      float dd[2 * U], nn[2 * U];
      F gW[2 * U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const float alpha = q0 + u < K ? sA[qq[u]] : 0.f;   // rows past the range: weight 0
        const float M = SK == SK_PGEN ? A.p : sR[qq[u]];
        F x, y;
#pragma unroll
        for (int q = 0; q < VEC * NC; ++q) {
          x.v[q] = hc[u] ? Pr[u].v[q] + Rv.v[q] : X.v[q];
          y.v[q] = hc[u] ? PT.v[q] : Pr[u].v[q];
        }
        score_xy_grad<SK>(x, y, alpha, M, g[2 * u], g[2 * u + 1]);
        // the r-lookup slice is d s / d x
        add_to(accR, g[2 * u]);
        nrm[1] += sq_partial(g[2 * u]);
        er[2 * u] = hc[u] ? &E[u] : &H;
        qr[2 * u] = hc[u] ? &Q[u] : &QH;
        pp[2 * u] = hc[u] ? &Pr[u] : &PH;
        dd[2 * u] = hc[u] ? dtn[u] : dth;
        nn[2 * u] = hc[u] ? nrn[u] : nrh;
        er[2 * u + 1] = hc[u] ? &T : &E[u];
        qr[2 * u + 1] = hc[u] ? &QT : &Q[u];
        pp[2 * u + 1] = hc[u] ? &PT : &Pr[u];
        dd[2 * u + 1] = hc[u] ? dtt : dtn[u];
        nn[2 * u + 1] = hc[u] ? nrt : nrn[u];
        gW[2 * u].zero();
        gW[2 * u + 1].zero();
      }
      F gE[2 * U], gQ[2 * U];
      project_back<TD, 2 * U>(g, er, qr, pp, dd, nn, W, P, gE, gQ, gW);
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const bool val = q0 + u < K;
        // rel aux slice of this triple: both sides' terms
        F sw;
#pragma unroll
        for (int q = 0; q < VEC * NC; ++q) sw.v[q] = gW[2 * u].v[q] + gW[2 * u + 1].v[q];
        add_to(accW, sw);
        nrm[2] += sq_partial(sw);
        nrm[0] += sq_partial(gE[2 * u]) + sq_partial(gE[2 * u + 1]);
        if (TD) nrm[3] += sq_partial(gQ[2 * u]) + sq_partial(gQ[2 * u + 1]);
        // the negative's row (materialised) and the positive's side
        const int ns = hc[u] ? 0 : 1, ps = 1 - ns;
        if (val) {
          const int64_t code = (int64_t)(((uint32_t)i << A.kshift) | (uint32_t)(q0 + u));
          store_row(gE[2 * u + ns], A.gneg + code * A.ent.cols, A.ent.cols);
          if (TD) store_row(gQ[2 * u + ns], P.gnegp + code * P.eaux.cols, P.eaux.cols);
        }
        if (hc[u]) {
          add_to(accT, gE[2 * u + ps]);
          if (TD) add_to(accQT, gQ[2 * u + ps]);
        } else {
          add_to(accH, gE[2 * u + ps]);
          if (TD) add_to(accQH, gQ[2 * u + ps]);
        }
      }
    }
    // the positive's own triple (wave 0)
    if (wv == 0) {
      F g[2], gW[2], gE[2], gQ[2];
      score_xy_grad<SK>(X, PT, sA[K], SK == SK_PGEN ? A.p : sR[K], g[0], g[1]);
      add_to(accR, g[0]);
      nrm[1] += sq_partial(g[0]);
      const F* er[2] = {&H, &T};
      const F* qr[2] = {&QH, &QT};
      const F* pp[2] = {&PH, &PT};
      const float dd[2] = {dth, dtt}, nn[2] = {nrh, nrt};
      gW[0].zero();
      gW[1].zero();
      project_back<TD, 2>(g, er, qr, pp, dd, nn, W, P, gE, gQ, gW);
      F sw;
#pragma unroll
      for (int q = 0; q < VEC * NC; ++q) sw.v[q] = gW[0].v[q] + gW[1].v[q];
      add_to(accW, sw);
      nrm[2] += sq_partial(sw);
      nrm[0] += sq_partial(gE[0]) + sq_partial(gE[1]);
      add_to(accH, gE[0]);
      add_to(accT, gE[1]);
      if (TD) {
        nrm[3] += sq_partial(gQ[0]) + sq_partial(gQ[1]);
        add_to(accQH, gQ[0]);
        add_to(accQT, gQ[1]);
      }
    }
    // ---- the positive's rows: the waves' accumulators summed in wave order
    {
      float* img = sm + L.mrg + wv * NACC * FL;
      stash(accH, img);
      stash(accR, img + FL);
      stash(accT, img + 2 * FL);
      stash(accW, img + 3 * FL);
      if (TD) {
        stash(accQH, img + 4 * FL);
        stash(accQT, img + 5 * FL);
      }
    }
    __syncthreads();
    float* gp = A.gpos + i * 3 * (int64_t)A.gcols;
    float* gp2 = P.gpos2 + i * 3 * (int64_t)A.gcols;
    for (int e = tid; e < NACC * FL; e += kPjThreads) {
      const int v = e / FL, k = e % FL;
      float s = 0.f;
#pragma unroll
      for (int w = 0; w < kPjWaves; ++w) s += sm[L.mrg + w * NACC * FL + e];
      // v: 0 h, 1 r, 2 t (ent_emb / rel_emb); 3 rel aux; 4, 5 ent_proj h, t
      if (v < 3) {
        if (k < (v == 1 ? A.rel.cols : A.ent.cols)) gp[v * A.gcols + k] = s;
      } else if (v == 3) {
        if (k < P.raux.cols) gp2[A.gcols + k] = s;
      } else if (k < P.eaux.cols) {
        gp2[(v == 4 ? 0 : 2) * A.gcols + k] = s;
      }
    }
    // ---- destination keys for the update passes
    for (int q = tid; q < K; q += kPjThreads) bin_key(A, ids[q], ((uint32_t)i << A.kshift) | (uint32_t)q);
    if (tid < 3) {
      const int64_t dest = tid == 0 ? ph : tid == 1 ? pt : A.ent.rows + pr;
      bin_key(A, dest, A.nkeyneg + ((uint32_t)i << 2) + (uint32_t)tid);
    }
  }
  if (err) set_status(A.status, err);

  // ---- partials: loss, slice norm^2 per variable; the last workgroup
  // reduces them in a fixed order
  wave_sums<4>(nrm);
  float* wn = sm + L.wn;
  if (lane == 0) {
#pragma unroll
    for (int v = 0; v < 4; ++v) wn[wv * 4 + v] = nrm[v];
  }
  __syncthreads();
  if (tid == 0) {
    float acc[5] = {misc[0], 0.f, 0.f, 0.f, 0.f};
    for (int w = 0; w < kPjWaves; ++w) {
#pragma unroll
      for (int v = 0; v < 4; ++v) acc[1 + v] += wn[w * 4 + v];
    }
#pragma unroll
    for (int c = 0; c < 5; ++c)
      __hip_atomic_store(&A.part[(int64_t)blockIdx.x * 8 + c], acc[c], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __builtin_amdgcn_s_waitcnt(0);
    const uint32_t prev = __hip_atomic_fetch_add(&A.ctl->score_ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    s_last = prev == (uint32_t)(gridDim.x - 1);
  }
  __syncthreads();
  if (s_last && wv == 0) {
    float acc[5] = {0.f, 0.f, 0.f, 0.f, 0.f};
    for (int w = lane; w < (int)gridDim.x; w += KGE_WAVE) {
#pragma unroll
      for (int c = 0; c < 5; ++c)
        acc[c] += __hip_atomic_load(&A.part[(int64_t)w * 8 + c], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
#pragma unroll
    for (int c = 0; c < 5; ++c) acc[c] = lane_reduce<5, false>(acc[c]);
    if (lane == 0) {
      A.loss_out[0] = acc[0];
      if (A.loss_accum) A.loss_accum[0] += acc[0];
      A.ctl->loss = acc[0];
      A.ctl->score_ticket = 0u;
      A.ctl->ovf_len = __hip_atomic_exchange(&A.ctl->ovf_count, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#pragma unroll
      for (int v = 0; v < 4; ++v) {
        A.ctl->scale[v] = -A.lr * (A.clip_norm / fmaxf(sqrtf(acc[1 + v]), A.clip_norm));
        if (A.norm2_out) A.norm2_out[v] = acc[1 + v];
      }
    }
  }
}

// host side (kge_proj.hip)
struct PjPlan {
  PjArgs P;
  bool td;
  bool dense;          // TransH + constraint: the regulariser term (loss, and dense gradients when training)
  bool grads;          // training step: dense gradients
  float lam;           // constraint_weight
  float* gdense[3];    // dense gradient buffers: ent, rel, rel_hyper
  float* dpart;        // [kPjDenseWGs * 4] dense-kernel partials
  TabView raux_tab;    // the aux tables as the update pass sees them
  TabView eaux_tab;
};
constexpr int kPjDenseWGs = 1024;
kge_status launch_step_proj(const StepArgs& A, const StepGeom& G, const PjPlan& J, int sk, hipStream_t st,
                            hipEvent_t const* ev);

}  // namespace kge
