// TransR fused training step for gfx950 (TransR.py:154-211) on fp32 MFMA.
//
// TransR projects every entity row of a triple through its relation's
// matrix M_r [d, k] before scoring:  s = score(clip(h M_r) + r, clip(t M_r)).
// All triples of a positive share M_r, so the projection work of one
// positive is three small GEMMs, done by ONE workgroup (8 waves):
//
//   X  [K+2, d]   its entity rows (h, t, the K negatives), gathered into LDS
//   P  = X M_r    GEMM1 [K+2, d] x [d, k]     -> projected rows, clipped in place
//   scores / loss / dL/dP per triple on the VALU (wave per slot); the
//   per-triple gradients wrt every projected row (slices), back through the clip
//   S  rows: summed h-slices, summed t-slices, each negative's slice, and
//            every positive-side slice on its own (clip_by_norm sees slices)
//   Y  = S M_r^T  GEMM2 [2K+4, k] x [k, d]  -> entity-row gradients (h, t to
//                 the positive-gradient rows, negatives to gneg[code]) and
//                 the entity slice norms ||M g||^2
//   dM = X^T S'   GEMM3 [d, K+2] x [K+2, k] -> this positive's rel_proj
//                 gradient (a per-positive partial; the apply pass sums a
//                 relation's partials in positive order)
//
// MFMA: v_mfma_f32_16x16x4_f32 (fp32 in / fp32 accumulate). Lane l holds
// A[l & 15][k = l >> 4], B[k = l >> 4][l & 15], C[(l >> 4) * 4 + reg][l & 15].
// Each wave owns 16-column tiles of the output and keeps that tile's whole
// B column (inner dimension <= 256 -> 64 registers) in registers while it
// walks the row tiles, so M_r is read from L2 once per GEMM per positive.
//
// The update pass is the shared destination-major kernel in its
// materialised mode (gradient rows summed in code order); rel_proj is
// updated by transr_proj_apply.
#include "kge_transr2.h"

namespace kge {

// (f32x4, mfma16, the MFMA tile helpers and the shared constants: kge_transr2.h)
extern template void launch_transr2<SK_P1>(const StepArgs&, const TrArgs&, hipStream_t);
extern template void launch_transr2<SK_P2>(const StepArgs&, const TrArgs&, hipStream_t);
extern template void launch_transr2<SK_PINF>(const StepArgs&, const TrArgs&, hipStream_t);
extern template void launch_transr2<SK_DOT>(const StepArgs&, const TrArgs&, hipStream_t);
extern template void launch_transr2<SK_PGEN>(const StepArgs&, const TrArgs&, hipStream_t);

template <int SK, int NC>
__global__ __launch_bounds__(kTrThreads) void transr_kernel(StepArgs A, TrArgs T) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  __shared__ float s_w[kTrWaves][4];
  __shared__ int s_last;
  if (ws_refused(A.ctl, A.sig, A.status, A.loss_out)) return;
  const int d = T.d, k = T.k, K = A.Keff, NR = K + 2, NS = 2 * K + 4;
  const TrLds L = tr_lds(d, k, K);
  constexpr int W = 16 * NC;   // padded row width (L.W)
  const int LX = L.LX, LP = L.LP, g4 = 4 * (lane_id() >> 4);
  float* X = sm;
  float* P = sm + L.NR16 * LX;
  float* S = sm;   // over X and P once both are consumed
  float* pn = sm + L.pn;
  float* xx = sm + L.xx;
  float* xh = sm + L.xh;
  float* xt = sm + L.xt;
  float* sS = sm + L.sS;
  float* sR = sm + L.sR;
  float* sT = sm + L.sT;
  float* sA = sm + L.sA;
  float* rp = sm + L.rp;
  int32_t* ids = reinterpret_cast<int32_t*>(sm + L.ids);
  float* misc = sm + L.misc;

  KGE_PROF_INIT();
  const int tid = threadIdx.x, lane = lane_id(), wv = wave_id();
  const int64_t i = blockIdx.x;
  int err = 0;
  int64_t ph = load_idx(A.pos, i * 3 + 0, A.i64);
  int64_t pr = load_idx(A.pos, i * 3 + 1, A.i64);
  int64_t pt = load_idx(A.pos, i * 3 + 2, A.i64);
  ph = ent_row(A, ph, &err);
  if (pr < 0 || pr >= A.rel.rows) { err = KGE_ERANGE; pr = 0; }
  pt = ent_row(A, pt, &err);
  for (int j = tid; j < K; j += kTrThreads) ids[j] = slot_entity(A, i, j, &err);
  __syncthreads();
  auto row_id = [&](int q) -> int64_t { return q == 0 ? ph : q == 1 ? pt : (int64_t)ids[q - 2]; };

  KGE_PROF(32);
  // ---- gather X (pad rows and columns zero): 4 rows' loads in flight per wave
  for (int row0 = wv; row0 < L.NR16; row0 += 4 * kTrWaves) {
    float v[4][kTrKV];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int row = row0 + u * kTrWaves;
      const float* src = row < NR ? A.ent.row(row_id(row)) : nullptr;
#pragma unroll
      for (int c4 = 0; c4 < kTrKV; ++c4) {
        const int c = lane + KGE_WAVE * c4;
        v[u][c4] = (src && c < d) ? src[c] : 0.f;
      }
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int row = row0 + u * kTrWaves;
      if (row >= L.NR16) break;
#pragma unroll
      for (int c4 = 0; c4 < kTrKV; ++c4) {
        const int c = lane + KGE_WAVE * c4;
        if (c < W) X[row * LX + c] = v[u][c4];
      }
    }
  }
  __syncthreads();
  KGE_PROF(33);
  // row statistics for the rel_proj slice norms: ||x||^2, x.h, x.t
  for (int row = wv; row < NR; row += kTrWaves) {
    float a = 0.f, b = 0.f, c2 = 0.f;
    for (int c = lane; c < d; c += KGE_WAVE) {
      const float x = X[row * LX + c];
      a += x * x;
      b += X[c] * x;
      c2 += X[LX + c] * x;
    }
    a = wsum(a);
    b = wsum(b);
    c2 = wsum(c2);
    if (lane == 0) { xx[row] = a; xh[row] = b; xt[row] = c2; }
  }

  // ---- GEMM1: P = X M_r  (wave = 16-column tile of P; row tiles in pairs)
  const float* Mr = T.proj.row(pr);
  {
    const int nct = (k + 15) / 16, nrt = L.NR16 / 16;
    // jobs = (column tile, row-tile pair), column-major, dealt to the waves in
    // equal contiguous ranges (13 column tiles over 8 waves left two SIMDs
    // with a third more work); B is reloaded only when the column tile changes
    const int npr = (nrt + 1) / 2, nj = nct * npr;
    const int jb = wv * nj / kTrWaves, je = (wv + 1) * nj / kTrWaves;
    int cur = -1;
    float bf[4 * NC];
    for (int jo = jb; jo < je; ++jo) {
      const int ct = jo / npr, rt = (jo - ct * npr) * 2;
      const int col = ct * 16 + (lane & 15);
      if (ct != cur) {
        cur = ct;
#pragma unroll
        for (int c = 0; c < NC; ++c)
#pragma unroll
          for (int u = 0; u < 4; ++u) {
            const int kk = 16 * c + g4 + u;
            bf[4 * c + u] = (kk < d && col < k) ? Mr[(int64_t)kk * k + col] : 0.f;
          }
      }
      {
        const int rt1 = rt + 1 < nrt ? rt + 1 : rt;   // odd count: the last tile alone
        f32x4 a0 = {0.f, 0.f, 0.f, 0.f}, a1 = {0.f, 0.f, 0.f, 0.f};
        const float* x0 = X + (rt * 16 + (lane & 15)) * LX + g4;
        const float* x1 = X + (rt1 * 16 + (lane & 15)) * LX + g4;
        if (rt1 != rt) mfma_pair_b128<NC>(a0, a1, x0, x1, bf);
        else mfma_one_b128<NC>(a0, x0, bf);
        if (col < W) {
#pragma unroll
          for (int g = 0; g < 4; ++g) {
            P[(rt * 16 + (lane >> 4) * 4 + g) * LP + col] = a0[g];
            if (rt1 != rt) P[(rt1 * 16 + (lane >> 4) * 4 + g) * LP + col] = a1[g];
          }
        }
      }
    }
  }
  __syncthreads();

  KGE_PROF(34);
  // ---- clip the projected rows (TransR.py:187-189, constraint.py:94-99)
  for (int row = wv; row < NR; row += kTrWaves) {
    float s2 = 0.f;
    for (int c = lane; c < k; c += KGE_WAVE) s2 += P[row * LP + c] * P[row * LP + c];
    const float n = sqrtf(wsum(s2));
    if (lane == 0) pn[row] = n;
    if (T.clip && !(n < 1.f)) {
      const float dv = fmaxf(n, 1e-9f);
      for (int c = lane; c < k; c += KGE_WAVE) P[row * LP + c] = P[row * LP + c] / dv;
    }
  }
  __syncthreads();

  // relation row r on the lanes (element c = lane + 64 v)
  float rr[kTrKV];
#pragma unroll
  for (int v = 0; v < kTrKV; ++v) {
    const int c = lane + KGE_WAVE * v;
    rr[v] = c < k ? A.rel.row(pr)[c] : 0.f;
  }
  // slot q (q < K: negative q; q == K: the positive) -> x / y rows of P
  auto xrow_of = [&](int q, int kind) { return kind == KIND_HC ? 2 + q : 0; };
  auto yrow_of = [&](int q, int kind) { return kind == KIND_TC ? 2 + q : 1; };
  auto kind_of = [&](int q) { return q == K ? KIND_POS : slot_kind(A.side_mode, q); };

  KGE_PROF(35);
  // ---- scores: s(x, y), x = P[xrow] + r, y = P[yrow]
  for (int m = 0; m < kTrQ; ++m) {
    const int q = wv + kTrWaves * m;
    if (q > K) break;
    const int kind = kind_of(q);
    const float* xp = P + xrow_of(q, kind) * LP;
    const float* yp = P + yrow_of(q, kind) * LP;
    float part = 0.f;
    float av[kTrKV];
#pragma unroll
    for (int v = 0; v < kTrKV; ++v) {
      const int c = lane + KGE_WAVE * v;
      av[v] = 0.f;
      if (c < k) {
        const float x = xp[c] + rr[v], y = yp[c];
        if (SK == SK_DOT) {
          part += x * y;
        } else {
          const float a = x - y, ma = fabsf(a);
          av[v] = a;
          part = SK == SK_P2 ? part + ma * ma : SK == SK_P1 ? part + ma
               : SK == SK_PGEN ? part + powf(ma, A.p) : fmaxf(part, ma);
        }
      }
    }
    const float R = SK == SK_PINF ? wmax(part) : wsum(part);
    float ties = 1.f;
    if (SK == SK_PINF) {
      float tq = 0.f;
#pragma unroll
      for (int v = 0; v < kTrKV; ++v)
        if (lane + KGE_WAVE * v < k && fabsf(av[v]) == R) tq += 1.f;
      ties = wsum(tq);
    }
    float lp;
    const float s = score_value<SK>(R, A.pw, &lp, A.p);
    if (lane == 0) { sS[q] = s; sR[q] = R; sT[q] = ties; }
  }
  __syncthreads();

  KGE_PROF(36);
  // ---- loss and dL/ds per triple (one wave, IEEE transcendentals; every
  // weight decided once -- the backward below reuses it)
  if (wv == 0) {
    const float sp = sS[K];
    const bool sans = A.loss_kind == KGE_LOSS_SANS;
    float Ms = -INFINITY;
    if (sans)
      for (int q = lane; q < K; q += KGE_WAVE) Ms = fmaxf(Ms, A.temperature * sS[q]);
    Ms = wmax(Ms);
    float Z = 0.f;
    if (sans)
      for (int q = lane; q < K; q += KGE_WAVE) Z += expf(A.temperature * sS[q] - Ms);
    Z = wsum(Z);
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
    lneg = wsum(lneg);
    csum = wsum(csum);
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
    for (int q = tid; q < K; q += kTrThreads) A.neg_score_out[i * K + q] = sS[q];
  __syncthreads();

  KGE_PROF(37);
  float n_ent = 0.f, n_rel = 0.f, n_proj = 0.f;
  if (A.train) {
    // ---- per-triple gradients wrt the projected rows, back through the clip;
    // kept in registers until every wave has finished reading P
    float G[kTrQ][2][kTrKV];   // [slot][0: positive side (h for pos), 1: entity side (t for pos)]
    float rsum[kTrKV];
#pragma unroll
    for (int v = 0; v < kTrKV; ++v) rsum[v] = 0.f;
    // Three passes over the wave's slots so the per-slot wave sums go through
    // two batched transposed reductions (multi_reduce: the same tree as wsum,
    // so the same bits) instead of five sequential reductions per slot.
    static_assert(3 * kTrQ <= 32, "batched slot reductions hold 32 values");
    float red[32];
#pragma unroll
    for (int t = 0; t < 32; ++t) red[t] = 0.f;
    // pass A: raw slice gradients (G[m][0] x side, G[m][1] y side), x . g_x, y . g_y
#pragma unroll
    for (int m = 0; m < kTrQ; ++m) {
      const int q = wv + kTrWaves * m;
#pragma unroll
      for (int v = 0; v < kTrKV; ++v) G[m][0][v] = G[m][1][v] = 0.f;
      if (q <= K) {
        const int kind = kind_of(q);
        const float* xp = P + xrow_of(q, kind) * LP;
        const float* yp = P + yrow_of(q, kind) * LP;
        const float alpha = sA[q], Mx = SK == SK_PGEN ? A.p : sR[q];
        float gxx = 0.f, dx = 0.f, dy = 0.f;
#pragma unroll
        for (int v = 0; v < kTrKV; ++v) {
          const int c = lane + KGE_WAVE * v;
          if (c < k) {
            const float x = xp[c] + rr[v], y = yp[c];
            float gx, gy;
            if (SK == SK_DOT) {
              gx = alpha * y;
              gy = alpha * x;
            } else {
              gx = lp_elem_grad<SK>(x - y, alpha, Mx);
              gy = -gx;
            }
            gxx += gx * gx;
            rsum[v] += gx;               // the r-lookup slice is d s / d x
            dx += gx * xp[c];
            dy += gy * yp[c];
            G[m][0][v] = gx;
            G[m][1][v] = gy;
          }
        }
        n_rel += gxx;
        red[2 * m] = dx;
        red[2 * m + 1] = dy;
      }
    }
    const float dxy = multi_reduce<32, false>(red);   // lane l: value l >> 1
    auto bcast = [](float v, int src) {
      return __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), src));
    };
    // pass B: back through clip_constraint (rows with norm >= 1 were divided by it)
#pragma unroll
    for (int t = 0; t < 32; ++t) red[t] = 0.f;
#pragma unroll
    for (int m = 0; m < kTrQ; ++m) {
      const int q = wv + kTrWaves * m;
      if (q <= K) {
        const int kind = kind_of(q);
        const int xr = xrow_of(q, kind), yr = yrow_of(q, kind);
        const float* xp = P + xr * LP;
        const float* yp = P + yr * LP;
        const float dx = bcast(dxy, (2 * m) << 1), dy = bcast(dxy, (2 * m + 1) << 1);
        const float nx = pn[xr], ny = pn[yr];
        const bool cx = T.clip && !(nx < 1.f), cy = T.clip && !(ny < 1.f);
        float a2 = 0.f, b2 = 0.f, ab = 0.f;
#pragma unroll
        for (int v = 0; v < kTrKV; ++v) {
          const int c = lane + KGE_WAVE * v;
          if (c < k) {
            if (cx) G[m][0][v] = (G[m][0][v] - dx * xp[c]) / nx;
            if (cy) G[m][1][v] = (G[m][1][v] - dy * yp[c]) / ny;
          }
          a2 += G[m][0][v] * G[m][0][v];
          b2 += G[m][1][v] * G[m][1][v];
          ab += G[m][0][v] * G[m][1][v];
        }
        red[3 * m] = a2;
        red[3 * m + 1] = b2;
        red[3 * m + 2] = ab;
      }
    }
    const float abr = multi_reduce<32, false>(red);
    // pass C: the rel_proj slice norms (x_h (x) g_h + x_t (x) g_t); the x side
    // is the head's projection, the y side the tail's
#pragma unroll
    for (int m = 0; m < kTrQ; ++m) {
      const int q = wv + kTrWaves * m;
      if (q <= K) {
        const int kind = kind_of(q);
        const int xr = xrow_of(q, kind), yr = yrow_of(q, kind);
        const float a2 = bcast(abr, (3 * m) << 1), b2 = bcast(abr, (3 * m + 1) << 1),
                    ab = bcast(abr, (3 * m + 2) << 1);
        const float hx = xx[xr], tx = xx[yr];
        const float htx = kind == KIND_POS ? xh[1] : (kind == KIND_TC ? xh[2 + q] : xt[2 + q]);
        n_proj += hx * a2 + tx * b2 + 2.f * htx * ab;
        if (kind == KIND_HC) {
#pragma unroll
          for (int v = 0; v < kTrKV; ++v) {
            const float t = G[m][0][v];
            G[m][0][v] = G[m][1][v];
            G[m][1][v] = t;
          }
        }
      }
    }
    __syncthreads();   // P is dead from here: S overwrites X and P
    KGE_PROF(38);
    // S rows: [0] sum of h-slices, [1] sum of t-slices, [2 + q] negative q's
    // entity slice, [K + 2] / [K + 3] the positive's h / t slices, [K + 4 + q]
    // negative q's positive-side slice; rows to SR16 zero
#pragma unroll
    for (int m = 0; m < kTrQ; ++m) {
      const int q = wv + kTrWaves * m;
      if (q > K) break;
      const int r0 = q == K ? K + 2 : K + 4 + q;   // positive-side slice
      const int r1 = q == K ? K + 3 : 2 + q;       // entity side (the positive's t)
#pragma unroll
      for (int v = 0; v < kTrKV; ++v) {
        const int c = lane + KGE_WAVE * v;
        if (c < W) {
          S[r0 * LP + c] = G[m][0][v];
          S[r1 * LP + c] = G[m][1][v];
        }
      }
    }
#pragma unroll
    for (int v = 0; v < kTrKV; ++v) {
      const int c = lane + KGE_WAVE * v;
      if (c < W) rp[wv * LP + c] = rsum[v];
    }
    for (int e = tid; e < (L.SR16 - NS) * LP; e += kTrThreads) S[NS * LP + e] = 0.f;
    __syncthreads();
    // summed positive rows, in slot order (deterministic): h = pos + tc slices,
    // t = pos + hc slices; r = the waves' partial sums in wave order
    float* gp = A.gpos + i * 3 * (int64_t)A.gcols;
    for (int c = tid; c < W; c += kTrThreads) {
      float h = S[(K + 2) * LP + c], t = S[(K + 3) * LP + c];
      for (int q = 0; q < K; ++q) {
        const float v = S[(K + 4 + q) * LP + c];
        if (slot_kind(A.side_mode, q) == KIND_TC) h += v; else t += v;
      }
      S[c] = h;
      S[LP + c] = t;
      float r = 0.f;
      for (int w = 0; w < kTrWaves; ++w) r += rp[w * LP + c];
      if (c < k) gp[A.gcols + c] = r;
    }
    __syncthreads();

    KGE_PROF(39);
    // ---- GEMM2: Y = S M_r^T -> entity-row gradients and slice norms
    {
      const int nct = (d + 15) / 16, nrt = (NS + 15) / 16;
      float* gp2 = gp;
      // (column tile, row-tile pair) jobs in equal contiguous ranges, as GEMM1
      const int npr = (nrt + 1) / 2, nj = nct * npr;
      const int jb = wv * nj / kTrWaves, je = (wv + 1) * nj / kTrWaves;
      // B = M_r^T: lane (column l & 15, group g) reads M_r row `col` at
      // 16c + 4g .. +3 -- one float4 per chunk when rows are 16-byte aligned
      const bool mv4 = (k & 3) == 0 && (T.proj.ld & 3) == 0 && ((uintptr_t)T.proj.p & 15) == 0;
      int cur = -1;
      float bf[4 * NC];
      for (int jo = jb; jo < je; ++jo) {
        const int ct = jo / npr, rt = (jo - ct * npr) * 2;
        const int col = ct * 16 + (lane & 15);
        if (ct != cur) {
          cur = ct;
          const float* mrow = Mr + (int64_t)col * k;
          if (mv4) {
#pragma unroll
            for (int c = 0; c < NC; ++c) {
              const int kk = 16 * c + g4;
              float4 m4 = make_float4(0.f, 0.f, 0.f, 0.f);
              if (kk < k && col < d) m4 = *reinterpret_cast<const float4*>(mrow + kk);
              bf[4 * c + 0] = m4.x;
              bf[4 * c + 1] = m4.y;
              bf[4 * c + 2] = m4.z;
              bf[4 * c + 3] = m4.w;
            }
          } else {
#pragma unroll
            for (int c = 0; c < NC; ++c)
#pragma unroll
              for (int u = 0; u < 4; ++u) {
                const int kk = 16 * c + g4 + u;
                bf[4 * c + u] = (kk < k && col < d) ? mrow[kk] : 0.f;
              }
          }
        }
        {
          const int rt1 = rt + 1 < nrt ? rt + 1 : rt;
          f32x4 acc[2] = {{0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}};
          const float* s0 = S + (rt * 16 + (lane & 15)) * LP + g4;
          const float* s1 = S + (rt1 * 16 + (lane & 15)) * LP + g4;
          if (rt1 != rt) mfma_pair_b128<NC>(acc[0], acc[1], s0, s1, bf);
          else mfma_one_b128<NC>(acc[0], s0, bf);
          if (col < d) {
#pragma unroll
            for (int h = 0; h < 2; ++h) {
              if (h == 1 && rt1 == rt) break;
              const int rtt = h ? rt1 : rt;
#pragma unroll
              for (int g = 0; g < 4; ++g) {
                const int row = rtt * 16 + (lane >> 4) * 4 + g;
                const float v = acc[h][g];
                if (row == 0) gp2[col] = v;
                else if (row == 1) gp2[2 * A.gcols + col] = v;
                else if (row < NS) {
                  n_ent += v * v;
                  if (row < NR) A.gneg[(int64_t)(((uint32_t)i << A.kshift) | (uint32_t)(row - 2)) * d + col] = v;
                }
              }
            }
          }
        }
      }
    }
    KGE_PROF(40);
    // ---- GEMM3: dM_i = X^T S[0 .. K+2) (X re-read from the table: L2); wave =
    // 16-row tile of dM with its A column in registers, column tiles in pairs
    {
      // N3: compile-time chunk count of the K + 2 slot rows (kTrKS3 / 4 at the
      // large K the kernel is sized for: straight-line, no per-chunk branch),
      // or 0: the runtime count
      auto gemm3 = [&](auto n3c) {
      constexpr int N3 = decltype(n3c)::value;
      const int nrt = (d + 15) / 16, nct = (k + 15) / 16, nkc = N3 ? N3 : (NR + 15) / 16;
      float* dm = T.dmpart + i * (int64_t)d * k;
      // (row tile, column-tile pair) jobs in equal contiguous ranges; the A
      // column is reloaded only when the row tile changes
      const int npc = (nct + 1) / 2, nj = nrt * npc;
      const int jb = wv * nj / kTrWaves, je = (wv + 1) * nj / kTrWaves;
      int cur = -1;
      float af[kTrKS3];
      for (int jo = jb; jo < je; ++jo) {
        const int rt = jo / npc, ct = (jo - rt * npc) * 2;
        const int ci = rt * 16 + (lane & 15);
        if (rt != cur) {
          cur = rt;
#pragma unroll
          for (int ks = 0; ks < kTrKS3; ++ks) {
            const int kk = ks * 4 + (lane >> 4);
            af[ks] = (kk < NR && ci < d) ? A.ent.row(row_id(kk))[ci] : 0.f;
          }
        }
        {
          const int ct1 = ct + 1 < nct ? ct + 1 : ct;
          f32x4 a0 = {0.f, 0.f, 0.f, 0.f}, a1 = {0.f, 0.f, 0.f, 0.f};
          const float* b0 = S + (lane >> 4) * LP + ct * 16 + (lane & 15);
          const float* b1 = S + (lane >> 4) * LP + ct1 * 16 + (lane & 15);
          if (ct1 != ct) {
#pragma unroll
            for (int c = 0; c < kTrKS3 / 4; ++c) {
              if (c < nkc) {
                float y0[4], y1[4];
#pragma unroll
                for (int u = 0; u < 4; ++u) {
                  y0[u] = b0[(c * 4 + u) * 4 * LP];
                  y1[u] = b1[(c * 4 + u) * 4 * LP];
                }
#pragma unroll
                for (int u = 0; u < 4; ++u) {
                  a0 = mfma16(af[c * 4 + u], y0[u], a0);
                  a1 = mfma16(af[c * 4 + u], y1[u], a1);
                }
              }
            }
          } else {   // the odd last column tile alone: two chains, added
#pragma unroll
            for (int c = 0; c < kTrKS3 / 4; ++c) {
              if (c < nkc) {
                float y0[4];
#pragma unroll
                for (int u = 0; u < 4; ++u) y0[u] = b0[(c * 4 + u) * 4 * LP];
                a0 = mfma16(af[c * 4 + 0], y0[0], a0);
                a1 = mfma16(af[c * 4 + 1], y0[1], a1);
                a0 = mfma16(af[c * 4 + 2], y0[2], a0);
                a1 = mfma16(af[c * 4 + 3], y0[3], a1);
              }
            }
            a0 += a1;
          }
#pragma unroll
          for (int h = 0; h < 2; ++h) {
            if (h == 1 && ct1 == ct) break;
            const int col = (h ? ct1 : ct) * 16 + (lane & 15);
            if (col >= k) continue;
#pragma unroll
            for (int g = 0; g < 4; ++g) {
              const int row = rt * 16 + (lane >> 4) * 4 + g;
              if (row < d) dm[(int64_t)row * k + col] = (h ? a1 : a0)[g];
            }
          }
        }
      }
      };
      if ((NR + 15) / 16 == kTrKS3 / 4) gemm3(std::integral_constant<int, kTrKS3 / 4>{});
      else gemm3(std::integral_constant<int, 0>{});
    }
    KGE_PROF(41);
    // ---- destination keys for the update pass
    for (int q = tid; q < K; q += kTrThreads) bin_key(A, ids[q], ((uint32_t)i << A.kshift) | (uint32_t)q);
    if (tid < 3) {
      const int64_t dest = tid == 0 ? ph : tid == 1 ? pt : A.ent.rows + pr;
      bin_key(A, dest, A.nkeyneg + ((uint32_t)i << 2) + (uint32_t)tid);
    }
  }
  if (err) set_status(A.status, err);
  KGE_PROF(42);

  // ---- partials: loss, ||g||^2 per variable (0 ent, 1 rel_emb, 2 rel_proj);
  // the last workgroup reduces them in a fixed order
  n_ent = wsum(n_ent);
  n_rel = wsum(n_rel);
  if (lane == 0) { s_w[wv][0] = n_ent; s_w[wv][1] = n_rel; s_w[wv][2] = n_proj; }
  __syncthreads();
  if (tid == 0) {
    float acc[5] = {misc[0], 0.f, 0.f, 0.f, 0.f};
    for (int w = 0; w < kTrWaves; ++w) {
      acc[1] += s_w[w][0];
      acc[2] += s_w[w][1];
      acc[3] += s_w[w][2];
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
    for (int c = 0; c < 5; ++c) acc[c] = wsum(acc[c]);
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

// rel_proj update: per relation, the positives' dM partials summed in
// sorted (positive) order, clip scale, SGD -- or the dense gradient in
// KGE_OPT_GRAD mode. 1024 elements of M_r per workgroup.
__global__ __launch_bounds__(256) void transr_proj_apply(StepArgs A, TrArgs T) {
  if (ws_refused(A.ctl, A.sig, A.status, A.loss_out)) return;
  const int64_t dk = (int64_t)T.d * T.k;
  const int64_t chunks = (dk + 1023) / 1024;
  const int64_t r = blockIdx.x / chunks, ch = blockIdx.x % chunks;
  const int64_t beg = T.rel_beg[r], end = beg + T.rel_cnt[r];
  if (beg == end) return;
  const float sc = A.ctl->scale[2];
  const int64_t e1 = min(dk, (ch + 1) * 1024);
  const bool v4 = dk % 4 == 0 && T.proj.ld % 4 == 0 && ((uintptr_t)T.proj.p % 16) == 0 &&
                  ((uintptr_t)T.dmpart % 16) == 0 && (!T.gproj_out || ((uintptr_t)T.gproj_out % 16) == 0);
  if (v4) {
    // a float4 of M_r per thread; the relation's partials four positives at
    // a time, every load issued before the adds (same ascending order)
    const int64_t e = ch * 1024 + 4 * (int64_t)threadIdx.x;
    if (e >= e1) return;
    float4 g = make_float4(0.f, 0.f, 0.f, 0.f);
    auto add = [&](const float4& x) { g.x += x.x; g.y += x.y; g.z += x.z; g.w += x.w; };
    const float* base = T.dmpart + e;
    int64_t p = beg;
    for (; p + 4 <= end; p += 4) {
      float4 x[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) x[u] = *reinterpret_cast<const float4*>(base + (int64_t)T.sorted[p + u] * dk);
#pragma unroll
      for (int u = 0; u < 4; ++u) add(x[u]);
    }
    for (; p < end; ++p) add(*reinterpret_cast<const float4*>(base + (int64_t)T.sorted[p] * dk));
    if (T.gproj_out) *reinterpret_cast<float4*>(T.gproj_out + r * dk + e) = g;
    else {
      float4* w = reinterpret_cast<float4*>(T.proj.p + r * T.proj.ld + e);
      float4 m = *w;
      m.x = m.x + g.x * sc; m.y = m.y + g.y * sc; m.z = m.z + g.z * sc; m.w = m.w + g.w * sc;
      *w = m;
    }
    return;
  }
  for (int64_t e = ch * 1024 + threadIdx.x; e < e1; e += 256) {
    float g = 0.f;
    for (int64_t p = beg; p < end; ++p) g += T.dmpart[(int64_t)T.sorted[p] * dk + e];
    if (T.gproj_out) T.gproj_out[r * dk + e] = g;
    else {
      float* w = T.proj.p + r * T.proj.ld + e;
      *w = *w + g * sc;
    }
  }
}

static void launch_update_mat(const StepArgs& A, const StepGeom& G, hipStream_t st) {
#define KGE_UPD(V, N)                                                                                            \
  do {                                                                                                           \
    if (A.compact)                                                                                               \
      hipLaunchKernelGGL((update_kernel<Materialised, V, N, SK_DOT, 1, true>), dim3(G.gridU), dim3(kUpdThreads), 0, \
                         st, A);                                                                                 \
    else                                                                                                         \
      hipLaunchKernelGGL((update_kernel<Materialised, V, N, SK_DOT>), dim3(G.gridU), dim3(kUpdThreads), 0, st, A); \
  } while (0)
  if (G.vec == 4) {
    if (G.nc == 1) KGE_UPD(4, 1); else if (G.nc == 2) KGE_UPD(4, 2); else KGE_UPD(4, 4);
  } else {
    if (G.nc == 1) KGE_UPD(1, 1); else if (G.nc == 2) KGE_UPD(1, 2); else KGE_UPD(1, 4);
  }
#undef KGE_UPD
}

template <int SK>
static void launch_tr(const StepArgs& A, const StepGeom& G, const TrArgs& T, const RelArgs& P, hipStream_t st,
                      hipEvent_t const* ev) {
  if (A.train) launch_rel_rank(P, st);
  const dim3 grid((unsigned)A.B), blk(kTrThreads);
  static const bool v1 = getenv("KGE_TRANSR_V1") != nullptr;   // (A/B timing of the one-per-CU kernel)
  if (v1) {
    const TrLds L = tr_lds(T.d, T.k, A.Keff);
    const size_t lds = (size_t)L.total_floats * 4;
    switch (L.NC) {
      case 4: hipLaunchKernelGGL((transr_kernel<SK, 4>), grid, blk, lds, st, A, T); break;
      case 8: hipLaunchKernelGGL((transr_kernel<SK, 8>), grid, blk, lds, st, A, T); break;
      case 13: hipLaunchKernelGGL((transr_kernel<SK, 13>), grid, blk, lds, st, A, T); break;
      default: hipLaunchKernelGGL((transr_kernel<SK, 16>), grid, blk, lds, st, A, T); break;
    }
  } else {
#ifndef KGE_ONLY_ONE
    launch_transr2<SK>(A, T, st);
#endif   // (single-instance tuning builds, tools/variants.py: no two-per-CU units linked)
  }
  if (ev) (void)hipEventRecord(ev[2], st);
  if (A.train) {
    launch_update_mat(A, G, st);
    const int64_t chunks = ((int64_t)T.d * T.k + 1023) / 1024;
    hipLaunchKernelGGL(transr_proj_apply, dim3((unsigned)(T.proj.rows * chunks)), dim3(256), 0, st, A, T);
  }
}

kge_status launch_step_transr(const StepArgs& A, const StepGeom& G, const TrArgs& T, const RelArgs& P, int sk,
                              hipStream_t st, hipEvent_t const* ev) {
  switch (sk) {
    case SK_P1: launch_tr<SK_P1>(A, G, T, P, st, ev); break;
    case SK_P2: launch_tr<SK_P2>(A, G, T, P, st, ev); break;
    case SK_PINF: launch_tr<SK_PINF>(A, G, T, P, st, ev); break;
    case SK_PGEN: launch_tr<SK_PGEN>(A, G, T, P, st, ev); break;
    default: launch_tr<SK_DOT>(A, G, T, P, st, ev); break;
  }
  return KGE_OK;
}

}  // namespace kge

#ifdef KGE_PHASE_PROF
// profiling builds (tools/transr_prof.py): read / reset this TU's phase counters
extern "C" int kge_trprof_read(unsigned long long* out, int n) {
  if (n > 64) n = 64;
  if (hipMemcpyFromSymbol(out, HIP_SYMBOL(kge::g_kge_prof), n * sizeof(unsigned long long)) != hipSuccess) return 1;
  unsigned long long z[64] = {0};
  return hipMemcpyToSymbol(HIP_SYMBOL(kge::g_kge_prof), z, sizeof(z)) != hipSuccess;
}
#endif
