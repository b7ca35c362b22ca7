// Per-model forward / backward policies for the element-wise model family
// (TransE, DistMult, RotatE). Each policy restates the reference's
// score_hrt and the TF-2.5 gradient of that op chain, on row fragments
// (kge_common.h): one wave owns one triple, a lane holds VEC*NC elements.
//
// Triple kinds: KIND_POS = the positive (h, r, t); KIND_HC = head-corrupted
// negative (E replaces h); KIND_TC = tail-corrupted negative (E replaces t)
// -- the corruption layout of BaseModel.py:360-408.
//
// Score element kinds SK (score.py): SK_P1 / SK_P2 / SK_PINF = LpDistance
// (or LpDistancePow) with p = 1, 2, inf; SK_DOT = Dot.
#pragma once

#include "kge_common.h"

namespace kge {

enum { KIND_POS = 0, KIND_HC = 1, KIND_TC = 2 };
enum { SK_P1 = 0, SK_P2 = 1, SK_PINF = 2, SK_DOT = 3, SK_PGEN = 4 };
// SK_PGEN: LpDistance(p) for any finite p > 0 (score.py:49-63); its runtime p
// travels in the `M` argument the p = inf kind uses for the row maximum

constexpr float kPiF = 3.14159265358979323846f;

// |z| of a complex element, evaluated identically at every call site (no
// contraction differences), so the p = inf arg-max test is exact.
__device__ __forceinline__ float cmod(float re, float im) {
#pragma clang fp contract(off)
  return sqrtf(re * re + im * im);
}

// ------------------------------------------------------------------ scores
// Per-lane partial of the score's reduction over the last axis, from
// a = x - y (Lp kinds) or a = x, b = y (Dot). CPLX: (re, im) interleaved and
// |.| is the complex modulus (score.py:59-63 on complex64 input).
template <int SK, bool CPLX, int VEC, int NC>
__device__ __forceinline__ float score_partial(const Frag<VEC, NC>& a, const Frag<VEC, NC>& b, float p = 2.f) {
  float acc = 0.f;
  if (SK == SK_DOT) {
#pragma unroll
    for (int i = 0; i < VEC * NC; ++i) acc += a.v[i] * b.v[i];
    return acc;
  }
  if (CPLX) {
#pragma unroll
    for (int i = 0; i < VEC * NC; i += 2) {
      if (SK == SK_P2) acc += a.v[i] * a.v[i] + a.v[i + 1] * a.v[i + 1];
      else if (SK == SK_P1) acc += cmod(a.v[i], a.v[i + 1]);
      else if (SK == SK_PGEN) acc += powf(cmod(a.v[i], a.v[i + 1]), p);
      else acc = fmaxf(acc, cmod(a.v[i], a.v[i + 1]));
    }
  } else {
#pragma unroll
    for (int i = 0; i < VEC * NC; ++i) {
      const float m = fabsf(a.v[i]);
      if (SK == SK_P2) acc += m * m;
      else if (SK == SK_P1) acc += m;
      else if (SK == SK_PGEN) acc += powf(m, p);
      else acc = fmaxf(acc, m);
    }
  }
  return acc;
}

// Number of elements attaining the max (for p = inf gradient ties).
template <bool CPLX, int VEC, int NC>
__device__ __forceinline__ float tie_partial(const Frag<VEC, NC>& a, float M) {
  float n = 0.f;
  if (CPLX) {
#pragma unroll
    for (int i = 0; i < VEC * NC; i += 2)
      n += (cmod(a.v[i], a.v[i + 1]) == M) ? 1.f : 0.f;
  } else {
#pragma unroll
    for (int i = 0; i < VEC * NC; ++i) n += (fabsf(a.v[i]) == M) ? 1.f : 0.f;
  }
  return n;
}

// Scalar score from the reduced value R:
//   LpDistance:    -pow(clip(R, 1e-9, inf), 1/p); p = inf: -R (max)
//   LpDistancePow: -(LpDistance)^2
//   Dot:           R
template <int SK>
__device__ __forceinline__ float score_value(float R, bool pw, float* lp_out, float p = 2.f) {
  if (SK == SK_DOT) { *lp_out = R; return R; }
  float lp;
  if (SK == SK_P2) lp = -sqrtf(fmaxf(R, 1e-9f));
  else if (SK == SK_P1) lp = -fmaxf(R, 1e-9f);
  else if (SK == SK_PGEN) lp = -powf(fmaxf(R, 1e-9f), 1.f / p);
  else lp = -R;
  *lp_out = lp;
  return pw ? -(lp * lp) : lp;
}

// dL/ds = c  ->  alpha such that the element gradient is
//   P2:   g_a = alpha * a                       (TF: pow/clip/sum/pow/abs chain)
//   P1:   g_a = alpha * sign(a) (complex: a/|a|)
//   PINF: g_a = alpha * sign(a) on the arg-max set (ties split evenly)
//   PGEN: g_a = alpha * |a|^(p-1) sign(a) (complex: |a|^(p-2) a),
//         alpha = -c R^(1/p - 1)   (d/dR of -R^(1/p) times d|a|^p/da / p)
//   DOT:  g_x = alpha * y, g_y = alpha * x
template <int SK>
__device__ __forceinline__ float score_alpha(float c, float R, float lp, float ties, bool pw, float p = 2.f) {
  if (SK == SK_DOT) return c;
  const float clp = pw ? c * (-2.f * lp) : c;   // d(-lp^2)/dlp = -2 lp
  if (SK == SK_P2) return R >= 1e-9f ? (-clp * 0.5f * rsqrtf(R)) * 2.f : 0.f;
  if (SK == SK_P1) return R >= 1e-9f ? -clp : 0.f;
  if (SK == SK_PGEN) return R >= 1e-9f ? -clp * powf(R, 1.f / p - 1.f) : 0.f;
  return -clp / ties;
}

// Hardware-rate forms (v_sqrt / v_rsq, ~1 ulp) of score_value / score_alpha
// for the score kernel's in-stream weights; the stored per-negative
// coefficients and scores use the IEEE forms above.
template <int SK>
__device__ __forceinline__ float score_value_fast(float R, bool pw, float* lp_out, float p = 2.f) {
  if (SK == SK_PGEN) return score_value<SK>(R, pw, lp_out, p);
  if (SK == SK_DOT) { *lp_out = R; return R; }
  float lp;
  if (SK == SK_P2) lp = -__builtin_amdgcn_sqrtf(fmaxf(R, 1e-9f));
  else if (SK == SK_P1) lp = -fmaxf(R, 1e-9f);
  else lp = -R;
  *lp_out = lp;
  return pw ? -(lp * lp) : lp;
}
template <int SK>
__device__ __forceinline__ float score_alpha_fast(float c, float R, float lp, float ties, bool pw, float p = 2.f) {
  if (SK == SK_PGEN) return score_alpha<SK>(c, R, lp, ties, pw, p);
  if (SK == SK_DOT) return c;
  const float clp = pw ? c * (-2.f * lp) : c;
  if (SK == SK_P2) return R >= 1e-9f ? -clp * __builtin_amdgcn_rsqf(R) : 0.f;
  if (SK == SK_P1) return R >= 1e-9f ? -clp : 0.f;
  return -clp * __builtin_amdgcn_rcpf(ties);
}
__device__ __forceinline__ float fast_exp(float x) { return __builtin_amdgcn_exp2f(x * 1.4426950408889634f); }
__device__ __forceinline__ float fast_sigmoid(float x) { return __builtin_amdgcn_rcpf(1.f + fast_exp(-x)); }

// Element gradient wrt a (Lp kinds). M = max |a| (PINF only).
template <int SK, bool CPLX, int VEC, int NC>
__device__ __forceinline__ void score_grad(const Frag<VEC, NC>& a, float alpha, float M,
                                           Frag<VEC, NC>& g) {
  if (SK == SK_P2) {
#pragma unroll
    for (int i = 0; i < VEC * NC; ++i) g.v[i] = alpha * a.v[i];
    return;
  }
  if (SK == SK_PGEN) {   // M carries p
#pragma unroll
    for (int i = 0; i < VEC * NC; i += (CPLX ? 2 : 1)) {
      if (CPLX) {
        const float m = cmod(a.v[i], a.v[i + 1]);
        const float s = m > 0.f ? alpha * powf(m, M - 2.f) : 0.f;
        g.v[i] = s * a.v[i];
        g.v[i + 1] = s * a.v[i + 1];
      } else {
        const float x = a.v[i];
        const float s = x > 0.f ? alpha : (x < 0.f ? -alpha : 0.f);
        g.v[i] = x != 0.f ? s * powf(fabsf(x), M - 1.f) : 0.f;
      }
    }
    return;
  }
  if (CPLX) {
#pragma unroll
    for (int i = 0; i < VEC * NC; i += 2) {
      const float m = cmod(a.v[i], a.v[i + 1]);
      float s = (m > 0.f) ? alpha / m : 0.f;
      if (SK == SK_PINF && m != M) s = 0.f;
      g.v[i] = s * a.v[i];
      g.v[i + 1] = s * a.v[i + 1];
    }
  } else {
#pragma unroll
    for (int i = 0; i < VEC * NC; ++i) {
      const float x = a.v[i];
      float s = x > 0.f ? alpha : (x < 0.f ? -alpha : 0.f);
      if (SK == SK_PINF && fabsf(x) != M) s = 0.f;
      g.v[i] = s;
    }
  }
}

template <int VEC, int NC>
__device__ __forceinline__ float sq_partial(const Frag<VEC, NC>& g) {
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < VEC * NC; ++i) s += g.v[i] * g.v[i];
  return s;
}

template <int VEC, int NC>
__device__ __forceinline__ void add_to(Frag<VEC, NC>& acc, const Frag<VEC, NC>& g) {
#pragma unroll
  for (int i = 0; i < VEC * NC; ++i) acc.v[i] += g.v[i];
}
template <int VEC, int NC>
__device__ __forceinline__ void sub_to(Frag<VEC, NC>& acc, const Frag<VEC, NC>& g) {
#pragma unroll
  for (int i = 0; i < VEC * NC; ++i) acc.v[i] -= g.v[i];
}

// Table view passed to kernels.
struct TabView {
  float* p;
  int64_t ld;
  int32_t cols;
  int64_t rows;
  __device__ __forceinline__ const float* row(int64_t i) const { return p + i * ld; }
  __device__ __forceinline__ float* row_w(int64_t i) const { return p + i * ld; }
};

// Model scalars shared by every policy call.
struct MP {
  float limit;       // RotatE phase range (RotatE.py:93)
  bool norm;         // fused full-table renormalisation: h / t context rows normalised on load
  const float* ctx;  // RESCAL: this positive's precomputed context rows (u = R^T h, v = R t)
};

// Context rows ("snap") written per positive by the score kernel and read
// back by the update kernel: everything a sampled row's gradient needs
// besides the row itself and its coefficient, frozen before any update.
// NSNAP rows of `cols` floats each. A negative's update-side context is ONE
// row for TransE / DistMult and at most two for RotatE.

// ======================================================================
// TransE: s(h + r, t)      (TransE.py:149-155)
//   positive      a = (h + r) - t            (the reference's op order)
//   t-corrupted   a = X - e,   X = h + r     (snap row 0)
//   h-corrupted   a = e + D,   D = r - t     (snap row 1)
// The update kernel rebuilds `a` from the same snap rows, so both kernels
// hold identical bits (the p = inf arg-max test depends on it).
// ======================================================================
template <int VEC, int NC, int SK>
struct TransE {
  static constexpr bool CPLX = false;
  static constexpr bool WIDE = false;   // score kernel fits 128 VGPRs at one chunk (4 waves / SIMD)
  static constexpr bool SELF_CTX = false;   // context rows computed by the score kernel itself (RESCAL)
  // owner-side scoring records carry the h and t accumulators only: an Lp
  // score is a function of h + r - t, so d/dr = d/dh for a t-corrupt slot and
  // -d/dt for an h-corrupt one -- the r accumulator is h - t (finish below);
  // Dot keeps all three
  static constexpr int REC_IMG = SK == SK_DOT ? 3 : 2;
  static constexpr bool FAST_STREAM = false;   // stream partial / gradient in hardware-rate forms (RotatE)
  static constexpr bool MAT = false;   // negatives' entity gradients re-derived, not materialised
  static constexpr int NSNAP = 2;
  using F = Frag<VEC, NC>;
  struct Ctx { F X, R, T, D; };
  struct ECtx { F c0; };

  __device__ static void load_ctx(Ctx& c, const TabView& ent, const TabView& rel, int64_t h,
                                  int64_t r, int64_t t, const MP& mp) {
    load_ctx_raw(c, ent, rel, h, r, t);
    ctx_finish(c, mp);
  }
  // load_ctx in two halves (the score kernel issues the context rows with
  // its first row batch and finishes them after): the raw rows (h parked
  // in X), then the normalisation and the combined rows
  __device__ static void load_ctx_raw(Ctx& c, const TabView& ent, const TabView& rel, int64_t h, int64_t r,
                                      int64_t t) {
    load_row(c.X, ent.row(h), ent.cols);
    load_row(c.R, rel.row(r), rel.cols);
    load_row(c.T, ent.row(t), ent.cols);
  }
  __device__ static void ctx_finish(Ctx& c, const MP& mp) {
    if (mp.norm) {
      normalize_row(c.X);
      normalize_row(c.T);
    }
#pragma unroll
    for (int i = 0; i < VEC * NC; ++i) {
      c.X.v[i] = c.X.v[i] + c.R.v[i];
      c.D.v[i] = c.R.v[i] - c.T.v[i];
    }
  }
  __device__ static void fwd(const Ctx& c, int kind, const F& E, F& a, F& b) {
#pragma unroll
    for (int i = 0; i < VEC * NC; ++i) {
      if (SK == SK_DOT) {
        a.v[i] = kind == KIND_HC ? E.v[i] + c.R.v[i] : c.X.v[i];
        b.v[i] = kind == KIND_TC ? E.v[i] : c.T.v[i];
      } else {
        a.v[i] = kind == KIND_HC ? E.v[i] + c.D.v[i] : c.X.v[i] - (kind == KIND_TC ? E.v[i] : c.T.v[i]);
      }
    }
  }
  __device__ static void grad_xy(const F& a, const F& b, float alpha, float M, F& gx, F& gy) {
    if (SK == SK_DOT) {
#pragma unroll
      for (int i = 0; i < VEC * NC; ++i) { gx.v[i] = alpha * b.v[i]; gy.v[i] = alpha * a.v[i]; }
    } else {
      score_grad<SK, false>(a, alpha, M, gx);
#pragma unroll
      for (int i = 0; i < VEC * NC; ++i) gy.v[i] = -gx.v[i];
    }
  }
  __device__ static void bwd(const Ctx& c, int kind, const F& E, const F& a, const F& b,
                             float alpha, float M, F& accH, F& accR, F& accT, float* nrm,
                             const MP&) {
    F gx, gy;
    grad_xy(a, b, alpha, M, gx, gy);
    const float sx = sq_partial(gx), sy = sq_partial(gy);
    nrm[0] += sx + sy;   // h-lookup slice + t-lookup slice
    nrm[1] += sx;        // r-lookup slice
    add_to(accR, gx);
    if (kind != KIND_HC) add_to(accH, gx);
    if (kind != KIND_TC) add_to(accT, gy);
  }
  // ---- score-kernel stream hooks (slot kind known at compile time)
  // Lp kinds: the t-slot gradient is minus the h-slot one, so a negative row
  // adds to ONE accumulator (t-corrupted -> h, h-corrupted -> t) and the
  // relation gradient is rebuilt once after the stream (finish): accR =
  // accH - accT. P2: the row gradient is alpha * a, so its norm^2 is
  // alpha^2 * R, accumulated from the reduced value (NRM_FROM_R).
  static constexpr bool NRM_FROM_R = SK == SK_P2;
  // update kernel: P2 negative gradient wrt its entity row E is
  // alpha (E + D) (h-corrupted) or alpha (E - X) (t-corrupted); Dot: alpha c0
  static constexpr bool LINEAR_E = SK == SK_P2 || SK == SK_DOT;
  __device__ static void lin_coefs(int kind, float alpha, float& aE, float& aC) {
    if (SK == SK_DOT) { aE = 0.f; aC = alpha; return; }
    aE = alpha;
    aC = kind == KIND_HC ? alpha : -alpha;
  }
  template <int KIND>
  __device__ static void fwdk(const Ctx& c, const F& E, F& a, F& b) {
#pragma unroll
    for (int i = 0; i < VEC * NC; ++i) {
      if (SK == SK_DOT) {
        a.v[i] = KIND == KIND_HC ? E.v[i] + c.R.v[i] : c.X.v[i];
        b.v[i] = KIND == KIND_TC ? E.v[i] : c.T.v[i];
      } else {
        a.v[i] = KIND == KIND_HC ? E.v[i] + c.D.v[i] : c.X.v[i] - (KIND == KIND_TC ? E.v[i] : c.T.v[i]);
      }
    }
  }
  template <int KIND>
  __device__ static void bwdk(const Ctx& c, const F& E, const F& a, const F& b, float alpha, float M,
                              F& accH, F& accR, F& accT, float* nrm, const MP& mp) {
    if (SK == SK_DOT) {
      bwd(c, KIND, E, a, b, alpha, M, accH, accR, accT, nrm, mp);
      return;
    }
    if (SK == SK_P2) {
#pragma unroll
      for (int i = 0; i < VEC * NC; ++i) {
        if (KIND == KIND_TC) accH.v[i] += alpha * a.v[i];
        else accT.v[i] -= alpha * a.v[i];
      }
      return;
    }
    F g;
    score_grad<SK, false>(a, alpha, M, g);
    const float s = sq_partial(g);
    nrm[0] += 2.f * s;
    nrm[1] += s;
    if (KIND == KIND_TC) add_to(accH, g);
    else sub_to(accT, g);
  }
  __device__ static void finish(F& accH, F& accR, F& accT) {
    if (SK == SK_DOT) return;
#pragma unroll
    for (int i = 0; i < VEC * NC; ++i) accR.v[i] = accH.v[i] - accT.v[i];
  }
  __device__ static void write_snap(const Ctx& c, float* sb, int cols) {
    store_row(c.X, sb, cols);
    if (SK == SK_DOT) {   // Dot: h-corrupted needs r and t separately -> keep r + t? use D slot for t
      store_row(c.T, sb + cols, cols);
    } else {
      store_row(c.D, sb + cols, cols);
    }
  }
  __device__ static void load_ectx(const float* sb, int cols, int kind, ECtx& ec) {
    load_row(ec.c0, sb + (kind == KIND_TC ? 0 : cols), cols);
  }
  // gradient of a negative wrt its sampled entity row E
  __device__ static void grad_entity(const ECtx& ec, int kind, const F& E, float alpha, float M, F& gE) {
    if (SK == SK_DOT) {
      // TC: d/dE (X . E) = alpha X ; HC: d/dE ((E + r) . t) = alpha t
#pragma unroll
      for (int i = 0; i < VEC * NC; ++i) gE.v[i] = alpha * ec.c0.v[i];
      return;
    }
    F a, g;
#pragma unroll
    for (int i = 0; i < VEC * NC; ++i) a.v[i] = kind == KIND_HC ? E.v[i] + ec.c0.v[i] : ec.c0.v[i] - E.v[i];
    score_grad<SK, false>(a, alpha, M, g);
    if (kind == KIND_HC) gE = g;
    else {
#pragma unroll
      for (int i = 0; i < VEC * NC; ++i) gE.v[i] = -g.v[i];
    }
  }
};

// ======================================================================
// DistMult: sum(h * r * t)     (DistMult.py:140-146); score_fn not used
//   positive / t-corrupted: a = h*r (snap row 0), b = t-side row
//   h-corrupted:            a = e,   b = t*r (snap row 1)
// ======================================================================
template <int VEC, int NC, int SK_UNUSED>
struct DistMult {
  static constexpr bool CPLX = false;
  static constexpr bool WIDE = true;    // five context rows: 256-VGPR budget (2 waves / SIMD)
  static constexpr bool SELF_CTX = false;
  static constexpr bool FAST_STREAM = false;
  static constexpr bool MAT = false;   // negatives' entity gradients re-derived, not materialised
  static constexpr int NSNAP = 2;
  using F = Frag<VEC, NC>;
  struct Ctx { F H, R, T, HR, TR; };
  struct ECtx { F c0; };

  __device__ static void load_ctx(Ctx& c, const TabView& ent, const TabView& rel, int64_t h,
                                  int64_t r, int64_t t, const MP& mp) {
    load_ctx_raw(c, ent, rel, h, r, t);
    ctx_finish(c, mp);
  }
  // the two halves (the score kernel's KGE_CTX_LATE): raw rows, then the
  // normalisation and the products
  __device__ static void load_ctx_raw(Ctx& c, const TabView& ent, const TabView& rel, int64_t h, int64_t r,
                                      int64_t t) {
    load_row(c.H, ent.row(h), ent.cols);
    load_row(c.R, rel.row(r), rel.cols);
    load_row(c.T, ent.row(t), ent.cols);
  }
  __device__ static void ctx_finish(Ctx& c, const MP& mp) {
    if (mp.norm) {
      normalize_row(c.H);
      normalize_row(c.T);
    }
#pragma unroll
    for (int i = 0; i < VEC * NC; ++i) {
      c.HR.v[i] = c.H.v[i] * c.R.v[i];
      c.TR.v[i] = c.T.v[i] * c.R.v[i];
    }
  }
  __device__ static void fwd(const Ctx& c, int kind, const F& E, F& a, F& b) {
#pragma unroll
    for (int i = 0; i < VEC * NC; ++i) {
      a.v[i] = kind == KIND_HC ? E.v[i] : c.HR.v[i];
      b.v[i] = kind == KIND_HC ? c.TR.v[i] : (kind == KIND_TC ? E.v[i] : c.T.v[i]);
    }
  }
  __device__ static void bwd(const Ctx& c, int kind, const F& E, const F& a, const F& b,
                             float alpha, float M, F& accH, F& accR, F& accT, float* nrm,
                             const MP&) {
    F gH, gR, gT;
    const F& Hv = kind == KIND_HC ? E : c.H;
    const F& Tv = kind == KIND_TC ? E : c.T;
#pragma unroll
    for (int i = 0; i < VEC * NC; ++i) {
      gH.v[i] = kind == KIND_HC ? alpha * c.TR.v[i] : (alpha * Tv.v[i]) * c.R.v[i];
      gR.v[i] = (alpha * Tv.v[i]) * Hv.v[i];
      gT.v[i] = kind == KIND_HC ? (alpha * E.v[i]) * c.R.v[i] : alpha * c.HR.v[i];
    }
    nrm[0] += sq_partial(gH) + sq_partial(gT);
    nrm[1] += sq_partial(gR);
    add_to(accR, gR);
    if (kind != KIND_HC) add_to(accH, gH);
    if (kind != KIND_TC) add_to(accT, gT);
  }
  // score-kernel stream hooks: slot kind known at compile time
  static constexpr bool NRM_FROM_R = false;   // row-gradient norm^2 from the reduced value
  // update kernel: a negative's entity gradient is aE * E + aC * c0 (scalars)
  static constexpr bool LINEAR_E = true;    // gradient wrt the entity row is alpha * c0
  __device__ static void lin_coefs(int kind, float alpha, float& aE, float& aC) { aE = 0.f; aC = alpha; }
  template <int KIND>
  __device__ static void fwdk(const Ctx& c, const F& E, F& a, F& b) { fwd(c, KIND, E, a, b); }
  template <int KIND>
  __device__ static void bwdk(const Ctx& c, const F& E, const F& a, const F& b, float alpha, float M,
                              F& accH, F& accR, F& accT, float* nrm, const MP& mp) {
    bwd(c, KIND, E, a, b, alpha, M, accH, accR, accT, nrm, mp);
  }
  __device__ static void finish(F& accH, F& accR, F& accT) {}
  __device__ static void write_snap(const Ctx& c, float* sb, int cols) {
    store_row(c.HR, sb, cols);
    store_row(c.TR, sb + cols, cols);
  }
  __device__ static void load_ectx(const float* sb, int cols, int kind, ECtx& ec) {
    load_row(ec.c0, sb + (kind == KIND_TC ? 0 : cols), cols);
  }
  __device__ static void grad_entity(const ECtx& ec, int kind, const F& E, float alpha, float M, F& gE) {
#pragma unroll
    for (int i = 0; i < VEC * NC; ++i) gE.v[i] = alpha * ec.c0.v[i];
  }
};

// ======================================================================
// RotatE: s(h o e^{i theta}, t), theta = r / limit * pi   (RotatE.py:148-165)
// ent rows are [d, 2] (re, im interleaved) -> 2d floats; rel rows d phases.
// VEC must be 2 or 4 (complex pairs stay inside one lane).
// snap rows: 0 = X = h o w, 1 = w = (cos, sin), 2 = t.
// ======================================================================
template <int VEC, int NC, int SK>
struct RotatE {
  static constexpr bool CPLX = true;
  static constexpr bool WIDE = true;
  static constexpr bool SELF_CTX = false;
  // C3's stream is VALU-bound on IEEE sqrt / divide per complex element
  // (PMC: 41 % of wave cycles issuing VALU, ~90 instructions per element):
  // LpDistance p = 1 / 2 stream rows use v_rsq once per element (|a| = s
  // rsq(s) for the score, a rsq(s) for the gradient, kept from forward to
  // backward in b); p = inf keeps the IEEE modulus (exact arg-max ties)
  static constexpr bool FAST_STREAM = SK == SK_P1 || SK == SK_P2;
  static constexpr bool MAT = false;
  static constexpr int NSNAP = 3;
  static constexpr int HV = VEC / 2;
  using F = Frag<VEC, NC>;
  struct Ctx { F H, X, CS, T; };   // CS = (cos, sin) interleaved, X = H o CS
  struct ECtx { F c0, c1; };
  __device__ static void load_ctx(Ctx& c, const TabView& ent, const TabView& rel, int64_t h,
                                  int64_t r, int64_t t, const MP& mp) {
    load_ctx_raw(c, ent, rel, h, r, t);
    ctx_finish(c, mp);
  }
  // the two halves (the score kernel's KGE_CTX_LATE): the raw rows (the
  // phases parked in CS's first half), then (cos, sin) and X = H o w
  __device__ static void load_ctx_raw(Ctx& c, const TabView& ent, const TabView& rel, int64_t h, int64_t r,
                                      int64_t t) {
    load_row(c.H, ent.row(h), ent.cols);
    load_row(c.T, ent.row(t), ent.cols);
    float ph[HV * NC];
    load_row_half<VEC, NC>(ph, rel.row(r), rel.cols);
#pragma unroll
    for (int k = 0; k < HV * NC; ++k) c.CS.v[k] = ph[k];
  }
  __device__ static void ctx_finish(Ctx& c, const MP& mp) {
    const float limit = mp.limit;
    float ph[HV * NC];
#pragma unroll
    for (int k = 0; k < HV * NC; ++k) ph[k] = c.CS.v[k];
#pragma unroll
    for (int k = 0; k < HV * NC; ++k) {
      const float th = (ph[k] / limit) * kPiF;
      c.CS.v[2 * k] = cosf(th);
      c.CS.v[2 * k + 1] = sinf(th);
    }
    cmul(c.H, c.CS, c.X);
  }
  // complex product, rounded op by op (no contraction): the update kernel
  // re-derives it and must get the same bits as the score kernel did
  __device__ static void cmul(const F& A, const F& W, F& out) {
#pragma clang fp contract(off)
#pragma unroll
    for (int i = 0; i < VEC * NC; i += 2) {
      out.v[i] = A.v[i] * W.v[i] - A.v[i + 1] * W.v[i + 1];
      out.v[i + 1] = A.v[i] * W.v[i + 1] + A.v[i + 1] * W.v[i];
    }
  }
  __device__ static void fwd(const Ctx& c, int kind, const F& E, F& a, F& b) {
    F x;
    if (kind == KIND_HC) cmul(E, c.CS, x); else x = c.X;
    const F& y = kind == KIND_TC ? E : c.T;
#pragma unroll
    for (int i = 0; i < VEC * NC; ++i) a.v[i] = x.v[i] - y.v[i];
  }
  // stream partial of a row (FAST_STREAM): b.v[2k] <- rsq(|a_k|^2) for bwdk
  template <int SKK>
  __device__ static float fast_partial(const F& a, F& b) {
    float acc = 0.f;
#pragma unroll
    for (int i = 0; i < VEC * NC; i += 2) {
      const float s = a.v[i] * a.v[i] + a.v[i + 1] * a.v[i + 1];
      if (SKK == SK_P2) {
        acc += s;
      } else {
        const float r = s > 0.f ? __builtin_amdgcn_rsqf(s) : 0.f;
        b.v[i] = r;
        acc += s * r;
      }
    }
    return acc;
  }
  // g_h = g_x * conj(w); g_theta = gxi * x_re - gxr * x_im
  // (FAST: the stream rows' element gradients from fast_partial's rsq in b,
  // and x of an h-corrupted row as a + t instead of a second complex product)
  template <bool FAST = false>
  __device__ static void bwd(const Ctx& c, int kind, const F& E, const F& a, const F& b,
                             float alpha, float M, F& accH, F& accR, F& accT, float* nrm,
                             const MP& mp) {
    const float plim = kPiF / mp.limit;
    F gx;
    if constexpr (FAST && SK == SK_P1) {
#pragma unroll
      for (int i = 0; i < VEC * NC; i += 2) {
        const float s = alpha * b.v[i];
        gx.v[i] = s * a.v[i];
        gx.v[i + 1] = s * a.v[i + 1];
      }
    } else {
      score_grad<SK, true>(a, alpha, M, gx);
    }
    F x;
    if (kind == KIND_HC) {
      if constexpr (FAST) {
#pragma unroll
        for (int i = 0; i < VEC * NC; ++i) x.v[i] = a.v[i] + c.T.v[i];
      } else {
        cmul(E, c.CS, x);
      }
    } else {
      x = c.X;
    }
    F gH;
    float gth2 = 0.f;
#pragma unroll
    for (int i = 0; i < VEC * NC; i += 2) {
      const float co = c.CS.v[i], si = c.CS.v[i + 1];
      gH.v[i] = gx.v[i] * co + gx.v[i + 1] * si;
      gH.v[i + 1] = gx.v[i + 1] * co - gx.v[i] * si;
      const float gth = gx.v[i + 1] * x.v[i] - gx.v[i] * x.v[i + 1];
      const float gr = gth * plim;
      accR.v[i] += gr;   // phase gradient kept in the even slot
      gth2 += gr * gr;
    }
    const float sx = sq_partial(gH), sy = sq_partial(gx);   // |g_t| = |g_u|
    nrm[0] += sx + sy;
    nrm[1] += gth2;
    if (kind != KIND_HC) add_to(accH, gH);
    if (kind != KIND_TC) sub_to(accT, gx);
  }
  // score-kernel stream hooks: slot kind known at compile time
  static constexpr bool NRM_FROM_R = false;   // row-gradient norm^2 from the reduced value
  // update kernel: a negative's entity gradient is aE * E + aC * c0 (scalars)
  static constexpr bool LINEAR_E = false;
  __device__ static void lin_coefs(int kind, float alpha, float& aE, float& aC) { aE = 0.f; aC = alpha; }
  template <int KIND>
  __device__ static void fwdk(const Ctx& c, const F& E, F& a, F& b) { fwd(c, KIND, E, a, b); }
  template <int KIND>
  __device__ static void bwdk(const Ctx& c, const F& E, const F& a, const F& b, float alpha, float M,
                              F& accH, F& accR, F& accT, float* nrm, const MP& mp) {
    bwd<FAST_STREAM>(c, KIND, E, a, b, alpha, M, accH, accR, accT, nrm, mp);
  }
  __device__ static void finish(F& accH, F& accR, F& accT) {}
  __device__ static void write_snap(const Ctx& c, float* sb, int cols) {
    store_row(c.X, sb, cols);
    store_row(c.CS, sb + cols, cols);
    store_row(c.T, sb + 2 * cols, cols);
  }
  // both rows loaded on every path (only the first one's address depends on
  // the kind): a branch-free shape keeps the update kernel's per-entry
  // contexts in registers (a half-filled struct array went to scratch)
  __device__ static void load_ectx(const float* sb, int cols, int kind, ECtx& ec) {
    load_row(ec.c0, sb + (kind == KIND_TC ? 0 : cols), cols);
    load_row(ec.c1, sb + 2 * cols, cols);
  }
  // element gradient of a row's score (the update kernel's re-derivation):
  // p = 1 with the stream's v_rsq form, else score_grad
  __device__ static void row_grad(const F& a, float alpha, float M, F& g) {
    if constexpr (SK == SK_P1) {
#pragma unroll
      for (int i = 0; i < VEC * NC; i += 2) {
        const float s = a.v[i] * a.v[i] + a.v[i + 1] * a.v[i + 1];
        const float k = s > 0.f ? alpha * __builtin_amdgcn_rsqf(s) : 0.f;
        g.v[i] = k * a.v[i];
        g.v[i + 1] = k * a.v[i + 1];
      }
    } else {
      score_grad<SK, true>(a, alpha, M, g);
    }
  }
  __device__ static void grad_entity(const ECtx& ec, int kind, const F& E, float alpha, float M, F& gE) {
    if (kind == KIND_TC) {
      F a, g;
#pragma unroll
      for (int i = 0; i < VEC * NC; ++i) a.v[i] = ec.c0.v[i] - E.v[i];
      row_grad(a, alpha, M, g);
#pragma unroll
      for (int i = 0; i < VEC * NC; ++i) gE.v[i] = -g.v[i];
    } else {
      F x, a, g;
      cmul(E, ec.c0, x);
#pragma unroll
      for (int i = 0; i < VEC * NC; ++i) a.v[i] = x.v[i] - ec.c1.v[i];
      row_grad(a, alpha, M, g);
#pragma unroll
      for (int i = 0; i < VEC * NC; i += 2) {
        const float co = ec.c0.v[i], si = ec.c0.v[i + 1];
        gE.v[i] = g.v[i] * co + g.v[i + 1] * si;
        gE.v[i + 1] = g.v[i + 1] * co - g.v[i] * si;
      }
    }
  }
};

// ======================================================================
// RESCAL: h^T R_r t     (RESCAL.py:140-174); score_fn not used
// A positive's score waves first compute its context rows u = R^T h and
// v = R t together (rel_gemv_pair, kge_step_impl.h: R_r streamed once per
// positive from L2, rows split over the waves), so every triple of the
// positive is a dot product of two d-vectors:
//   positive      u . t
//   t-corrupted   u . e          (gradient wrt e: alpha u)
//   h-corrupted   e . v          (gradient wrt e: alpha v)
// The positive's own rows need R again: g_h = R (c_p t + sum_tc alpha e),
// g_t = R^T (c_p h + sum_hc alpha e) -- the same waves after the merge, from
// the UN-projected sums in the positive-gradient rows (row 0: A = c_p t +
// sum_tc alpha e, row 1: b = sum_hc alpha e, row 2: B = c_p h + b). The MFMA
// pass after the score kernel forms dR_r = sum_i h_i (x) A_i + b_i (x) t_i.
// ======================================================================
template <int VEC, int NC, int SK_UNUSED>
struct Rescal {
  static constexpr bool CPLX = false;
  static constexpr bool WIDE = false;
  // u = R^T h, v = R t computed by the positive's own score waves (and the
  // post products g_h = R A, g_t = R^T B after the merge): no separate passes
  static constexpr bool SELF_CTX = true;
  static constexpr bool FAST_STREAM = false;
  static constexpr bool MAT = false;   // negatives' entity gradients re-derived, not materialised
  static constexpr int NSNAP = 2;
  using F = Frag<VEC, NC>;
  struct Ctx { F H, T, U, V; };
  struct ECtx { F c0; };

  __device__ static void load_ctx(Ctx& c, const TabView& ent, const TabView&, int64_t h, int64_t,
                                  int64_t t, const MP& mp) {
    load_row(c.H, ent.row(h), ent.cols);
    load_row(c.T, ent.row(t), ent.cols);
    load_row(c.U, mp.ctx, ent.cols);
    load_row(c.V, mp.ctx + ent.cols, ent.cols);
  }
  __device__ static void fwd(const Ctx& c, int kind, const F& E, F& a, F& b) {
#pragma unroll
    for (int i = 0; i < VEC * NC; ++i) {
      a.v[i] = kind == KIND_HC ? E.v[i] : c.U.v[i];
      b.v[i] = kind == KIND_HC ? c.V.v[i] : (kind == KIND_TC ? E.v[i] : c.T.v[i]);
    }
  }
  // POS (called at unit alpha): row 0 gets t, row 2 gets h (scaled by c_p
  // in the merge); TC: row 0 += alpha e; HC: rows 1 and 2 += alpha e
  __device__ static void bwd(const Ctx& c, int kind, const F& E, const F&, const F&, float alpha, float,
                             F& accH, F& accR, F& accT, float*, const MP&) {
#pragma unroll
    for (int i = 0; i < VEC * NC; ++i) {
      if (kind == KIND_POS) {
        accH.v[i] += alpha * c.T.v[i];
        accT.v[i] += alpha * c.H.v[i];
      } else if (kind == KIND_TC) {
        accH.v[i] += alpha * E.v[i];
      } else {
        accR.v[i] += alpha * E.v[i];
        accT.v[i] += alpha * E.v[i];
      }
    }
  }
  static constexpr bool NRM_FROM_R = false;
  static constexpr bool LINEAR_E = true;   // gradient wrt a sampled entity row: alpha * (u or v)
  __device__ static void lin_coefs(int, float alpha, float& aE, float& aC) { aE = 0.f; aC = alpha; }
  template <int KIND>
  __device__ static void fwdk(const Ctx& c, const F& E, F& a, F& b) { fwd(c, KIND, E, a, b); }
  template <int KIND>
  __device__ static void bwdk(const Ctx& c, const F& E, const F& a, const F& b, float alpha, float M,
                              F& accH, F& accR, F& accT, float* nrm, const MP& mp) {
    bwd(c, KIND, E, a, b, alpha, M, accH, accR, accT, nrm, mp);
  }
  __device__ static void finish(F&, F&, F&) {}
  __device__ static void write_snap(const Ctx&, float*, int) {}   // written by the context pass
  __device__ static void load_ectx(const float* sb, int cols, int kind, ECtx& ec) {
    load_row(ec.c0, sb + (kind == KIND_TC ? 0 : cols), cols);
  }
  __device__ static void grad_entity(const ECtx& ec, int, const F&, float alpha, float, F& gE) {
#pragma unroll
    for (int i = 0; i < VEC * NC; ++i) gE.v[i] = alpha * ec.c0.v[i];
  }
};

// ======================================================================
// Materialised-gradient family (TransR; kge_transr.hip): the score pass
// writes every negative's entity-row gradient to gneg[code] (it is a GEMM
// output, M_r g, not a function of one context row), so the update kernel
// only sums rows. Only the update-kernel hooks are defined.
// ======================================================================
template <int VEC, int NC, int SK_UNUSED>
struct Materialised {
  static constexpr bool CPLX = false;
  static constexpr bool WIDE = false;
  static constexpr bool SELF_CTX = false;
  static constexpr bool FAST_STREAM = false;
  static constexpr bool MAT = true;
  static constexpr int NSNAP = 0;
  static constexpr bool NRM_FROM_R = false;
  static constexpr bool LINEAR_E = false;
  using F = Frag<VEC, NC>;
  struct ECtx { F c0; };
  __device__ static void lin_coefs(int, float alpha, float& aE, float& aC) { aE = 0.f; aC = alpha; }
  __device__ static void load_ectx(const float*, int, int, ECtx&) {}
  __device__ static void grad_entity(const ECtx& ec, int, const F&, float, float, F& gE) { gE = ec.c0; }
};

}  // namespace kge
