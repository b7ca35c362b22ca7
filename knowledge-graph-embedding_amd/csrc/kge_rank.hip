// Batched filtered ranking for gfx950: KGEModel.evaluate / get_rank
// (BaseModel.py:578-654) for a whole evaluation set in three launches.
//
// The reference ranks ONE triple per Python iteration (batch_size=1,
// :598): it scores every entity on the corrupted side, overwrites the
// filtered positives with -inf (:650) and counts scores strictly above the
// true triple's (:654, int16). Here a query q is one evaluation triple; its
// candidates are all E entities:
//
//   rank_pos_kernel     thread per query: the true entity's score through
//                       the candidate scoring function (pos_score_out)
//   rank_count_kernel   workgroup = 256 candidates (one per lane) x 8
//                       queries; the queries' rows sit in LDS (broadcast
//                       reads), each candidate row is loaded once per 8
//                       queries and scored against all of them with no
//                       cross-lane reduction (a lane owns its candidate's
//                       whole sum); strict > pos per query -> ballot ->
//                       popcount -> one int64 atomic per wave and query
//   rank_filter_kernel  wave per query: rescores only its filtered entities
//                       and subtracts those above the true score, + 1
//
// With a filter bitmap (kge_rank_desc.filt_bits, ABI 8) rank_bits_kernel
// marks each query's filtered entities first, the count passes skip marked
// candidates and the pos pass starts every rank at 1: no rescoring pass. The
// comparisons are the same ones, so are the ranks.
//
// Every score is evaluated op by op (no contraction) in one fixed order, so
// the true entity scored as a candidate equals its pos score bit for bit and
// never counts itself, and the filter pass sees exactly the scores the count
// pass compared. Counts are integer atomics (order-free, deterministic).
//
// Query rows are prepared by the host (KGE/engine.py rank_queries) with the
// model's own op order: TransE t-side x = h + r; TransH x = P(h) + r with w_r;
// TransD r_p; TransR the group's pre-projected candidate table; DistMult
// h * r; RESCAL R^T h / R t; RotatE h o w / w, t.
#include <algorithm>

#include "kge_step.h"

namespace kge {

// Scores of candidate entity `e` against NQ queries whose rows sit at
// q0 + j * qs, q1 + j * qs, w + j * qs (any address space). The candidate's
// elements are loaded once and used by every query; each query's sum runs in
// the same element order for any NQ, so NQ = 1 (pos / filter passes) and
// NQ = 8 (count pass) give identical bits. MODE: KGE_RANK_*; PJ: KGE_RPROJ_*.
template <int MODE, int PJ, int SK, int NQ>
__device__ __forceinline__ void rank_scores(const RankArgs& A, int64_t e, const float* q0, const float* q1,
                                            const float* w, int qs, float (&out)[NQ]) {
#pragma clang fp contract(off)
  const float* x = A.cand + e * A.cand_ld;
  const int D = A.dim;
  float acc[NQ];
#pragma unroll
  for (int j = 0; j < NQ; ++j) acc[j] = 0.f;
  auto lp = [&](float& ac, float a) {
    const float m = fabsf(a);
    if (SK == SK_P2) ac = ac + m * m;
    else if (SK == SK_P1) ac = ac + m;
    else if (SK == SK_PGEN) ac = ac + powf(m, A.p);
    else ac = fmaxf(ac, m);
  };
  if (MODE == KGE_RANK_ROT) {
    // complex pairs; t-side a = q0 - e, h-side a = e o q0 - q1
    for (int c = 0; c < D; c += 2) {
      const float er = x[c], ei = x[c + 1];
#pragma unroll
      for (int j = 0; j < NQ; ++j) {
        const float* a0 = q0 + j * qs;
        float ar, ai;
        if (A.hside) {
          const float* a1 = q1 + j * qs;
          const float xr = er * a0[c] - ei * a0[c + 1];
          const float xi = er * a0[c + 1] + ei * a0[c];
          ar = xr - a1[c];
          ai = xi - a1[c + 1];
        } else {
          ar = a0[c] - er;
          ai = a0[c + 1] - ei;
        }
        if (SK == SK_P2) acc[j] = acc[j] + (ar * ar + ai * ai);
        else {
          const float m = sqrtf(ar * ar + ai * ai);
          acc[j] = SK == SK_P1 ? acc[j] + m : SK == SK_PGEN ? acc[j] + powf(m, A.p) : fmaxf(acc[j], m);
        }
      }
    }
  } else if (MODE == KGE_RANK_MUL || MODE == KGE_RANK_DOT) {
    // DistMult sum(h * r * t): t-side q0 = h * r, h-side (e * r) * t;
    // RESCAL: q0 = R^T h (t-side) or R t (h-side)
    for (int c = 0; c < D; ++c) {
      const float xe = x[c];
#pragma unroll
      for (int j = 0; j < NQ; ++j) {
        const float* a0 = q0 + j * qs;
        acc[j] = acc[j] + ((MODE == KGE_RANK_MUL && A.hside) ? (xe * a0[c]) * q1[j * qs + c] : a0[c] * xe);
      }
    }
  } else {
    // translating: P(e) then t-side a = q0 - P(e), h-side a = (P(e) + q0) - q1
    float dt[NQ], sc[NQ];
#pragma unroll
    for (int j = 0; j < NQ; ++j) { dt[j] = 0.f; sc[j] = 1.f; }
    if (PJ == KGE_RPROJ_HYPER) {
      for (int c = 0; c < D; ++c) {
        const float xe = x[c];
#pragma unroll
        for (int j = 0; j < NQ; ++j) dt[j] = dt[j] + w[j * qs + c] * xe;
      }
    } else if (PJ == KGE_RPROJ_RANK1) {
      // e_p . e is the candidate's own; the clip norm depends on the query's r_p
      const float* ep = A.caux + e * A.caux_ld;
      float de = 0.f;
      for (int c = 0; c < A.ecols; ++c) de = de + ep[c] * x[c];
#pragma unroll
      for (int j = 0; j < NQ; ++j) dt[j] = de;
      if (A.clip) {
        float n2[NQ];
#pragma unroll
        for (int j = 0; j < NQ; ++j) n2[j] = 0.f;
        for (int c = 0; c < D; ++c) {
          const float xe = c < A.kmin ? x[c] : 0.f;
#pragma unroll
          for (int j = 0; j < NQ; ++j) {
            const float p = w[j * qs + c] * de + xe;
            n2[j] = n2[j] + p * p;
          }
        }
#pragma unroll
        for (int j = 0; j < NQ; ++j) {
          const float n = sqrtf(n2[j]);
          if (!(n < 1.f)) sc[j] = fmaxf(n, 1e-9f);
        }
      }
    }
    for (int c = 0; c < D; ++c) {
      const float xe = (PJ != KGE_RPROJ_RANK1 || c < A.kmin) ? x[c] : 0.f;
#pragma unroll
      for (int j = 0; j < NQ; ++j) {
        const float* a0 = q0 + j * qs;
        float p;
        if (PJ == KGE_RPROJ_HYPER) p = xe - dt[j] * w[j * qs + c];
        else if (PJ == KGE_RPROJ_RANK1) p = (w[j * qs + c] * dt[j] + xe) / sc[j];
        else p = xe;
        if (SK == SK_DOT) acc[j] = acc[j] + (A.hside ? (p + a0[c]) * q1[j * qs + c] : a0[c] * p);
        else lp(acc[j], A.hside ? (p + a0[c]) - q1[j * qs + c] : a0[c] - p);
      }
    }
  }
#pragma unroll
  for (int j = 0; j < NQ; ++j) {
    if (SK == SK_DOT || MODE == KGE_RANK_MUL || MODE == KGE_RANK_DOT) {
      out[j] = acc[j];
    } else {
      float lpv;
      out[j] = score_value<SK>(acc[j], A.pw, &lpv, A.p);
    }
  }
}

__device__ __forceinline__ const float* qrow(const float* base, const RankArgs& A, int64_t q) {
  return base ? base + q * A.ldq : nullptr;
}

template <int MODE, int PJ, int SK>
__global__ __launch_bounds__(256) void rank_pos_kernel(RankArgs A) {
  const int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (q >= A.n) return;
  int64_t e = load_idx(A.true_ids, q, A.i64);
  if (e < 0 || e >= A.E) { set_status(A.status, KGE_ERANGE); e = 0; }
  float o[1];
  rank_scores<MODE, PJ, SK, 1>(A, e, qrow(A.q0, A, q), qrow(A.q1, A, q), qrow(A.qw, A, q), 0, o);
  A.pos[q] = o[0];
  if (A.fbits) A.rank[q] = 1ull;   // (bitmap filter: the +1 of the filter pass; counts are added after)
}

// The filter bitmap: workgroup per query, bit e of the query's words for each
// entity of its filter list (sorted, unique per query; an id outside [0, E)
// sets KGE_ERANGE). Up to kBitsLds words per query the bits are gathered in
// LDS and every word is written once (no clear needed); past that the caller
// (kge_rank) clears the words first and the bits go in with global atomics.
constexpr int kBitsLds = 8192;
template <bool LDS>
__global__ __launch_bounds__(256) void rank_bits_kernel(RankArgs A, uint32_t* bits) {
  __shared__ uint32_t sb[LDS ? kBitsLds : 1];
  const int64_t q = blockIdx.x;
  const int W = (int)A.fw;
  uint32_t* out = bits + q * A.fw;
  if (LDS) {
    for (int w = threadIdx.x; w < W; w += 256) sb[w] = 0u;
    __syncthreads();
  }
  for (int64_t j = A.fbeg[q] + threadIdx.x; j < A.fend[q]; j += 256) {
    const int64_t e = load_idx(A.fent, j, A.i64);
    if (e < 0 || e >= A.E) { set_status(A.status, KGE_ERANGE); continue; }
    const uint32_t m = 1u << (uint32_t)(e & 31);
    if (LDS) atomicOr(&sb[e >> 5], m);
    else atomicOr(&out[e >> 5], m);
  }
  if (LDS) {
    __syncthreads();
    for (int w = threadIdx.x; w < W; w += 256) out[w] = sb[w];
  }
}

template <int MODE, int PJ, int SK>
__global__ __launch_bounds__(kRankThreads) void rank_count_kernel(RankArgs A, int64_t g0, int64_t c0) {
  extern __shared__ __attribute__((aligned(16))) float qs[];
  // x: query group (consecutive workgroups share a candidate chunk, so its
  // rows are reused from L2 across groups), y: candidate chunk
  const int64_t g = g0 + blockIdx.x, ch = c0 + blockIdx.y;
  const int64_t q0i = g * kRankQ;
  const int nq = (int)min<int64_t>(kRankQ, A.n - q0i);
  const int LQ = (A.dim + 3) & ~3;
  float* s0 = qs;
  float* s1 = qs + kRankQ * LQ;
  float* sw = qs + 2 * kRankQ * LQ;
  // the group's query rows (rows past the set: zeros, results discarded)
  for (int t = threadIdx.x; t < kRankQ * A.dim; t += kRankThreads) {
    const int q = t / A.dim, c = t % A.dim;
    const bool v = q < nq;
    s0[q * LQ + c] = v ? A.q0[(q0i + q) * A.ldq + c] : 0.f;
    s1[q * LQ + c] = (v && A.q1) ? A.q1[(q0i + q) * A.ldq + c] : 0.f;
    sw[q * LQ + c] = (v && A.qw) ? A.qw[(q0i + q) * A.ldq + c] : 0.f;
  }
  float pos[kRankQ];
#pragma unroll
  for (int q = 0; q < kRankQ; ++q) pos[q] = q < nq ? A.pos[q0i + q] : INFINITY;
  __syncthreads();
  const int64_t e = ch * kRankThreads + threadIdx.x;
  const bool in = e < A.E;
  const int64_t ee = in ? e : 0;
  bool keep[kRankQ];   // (bitmap filter: the candidate is not a known positive of the query)
#pragma unroll
  for (int q = 0; q < kRankQ; ++q)
    keep[q] = !(A.fbits && q < nq && ((A.fbits[(q0i + q) * A.fw + (ee >> 5)] >> (uint32_t)(ee & 31)) & 1u));
  float s[kRankQ];
  rank_scores<MODE, PJ, SK, kRankQ>(A, ee, s0, s1, sw, LQ, s);
#pragma unroll
  for (int q = 0; q < kRankQ; ++q) {
    const unsigned long long m = __ballot(in && q < nq && keep[q] && s[q] > pos[q]);
    if (lane_id() == 0 && m) atomicAdd(&A.rank[q0i + q], (unsigned long long)__popcll(m));
  }
}

template <int MODE, int PJ, int SK>
__global__ __launch_bounds__(256) void rank_filter_kernel(RankArgs A) {
  const int64_t q = (int64_t)blockIdx.x * 4 + wave_id();
  if (q >= A.n) return;
  unsigned long long sub = 0;
  if (A.fbeg) {
    const float p = A.pos[q];
    const float* r0 = qrow(A.q0, A, q);
    const float* r1 = qrow(A.q1, A, q);
    const float* rw = qrow(A.qw, A, q);
    for (int64_t j = A.fbeg[q] + lane_id(); j < A.fend[q]; j += KGE_WAVE) {
      const int64_t e = load_idx(A.fent, j, A.i64);
      if (e < 0 || e >= A.E) { set_status(A.status, KGE_ERANGE); continue; }
      float o[1];
      rank_scores<MODE, PJ, SK, 1>(A, e, r0, r1, rw, 0, o);
      sub += o[0] > p ? 1ull : 0ull;
    }
  }
  for (int o = 32; o >= 1; o >>= 1) sub += __shfl_xor(sub, o, KGE_WAVE);
  if (lane_id() == 0) A.rank[q] = A.rank[q] - sub + 1ull;
}

// Register-tiled count pass for the element-wise scores (translating without
// a projection: TransE, TransR's pre-projected candidates; DistMult; RESCAL):
// a workgroup scores a 64-query x 64-candidate tile, each thread 4 x 4 pairs
// held in registers, over 16-element chunks staged transposed in LDS
// ([element][row]: a thread's four queries and four candidates are one
// ds_read_b128 each). Candidate rows are read once per 64 queries and with
// whole-row float4 loads (the lane-per-candidate pass reads 4 bytes of 64
// different rows per instruction). Every pair's sum runs over the elements in
// ascending order with the same ops as rank_scores, so the scores -- and the
// strict > comparisons -- are bit for bit those of the pos / filter passes.
constexpr int kRT = 64;    // queries / candidates per tile
constexpr int kRC = 16;    // elements per staged chunk

template <int MODE, int SK, bool HS>
__global__ __launch_bounds__(256) void rank_tile_kernel(RankArgs A, int64_t qt0) {
#pragma clang fp contract(off)
  using f2 = __attribute__((ext_vector_type(2))) float;
  __shared__ __attribute__((aligned(16))) float sq0[kRC][kRT];
  __shared__ __attribute__((aligned(16))) float sq1[kRC][kRT];
  __shared__ __attribute__((aligned(16))) float sx[kRC][kRT];
  const int tid = threadIdx.x, tq = tid >> 4, tc = tid & 15;
  const int64_t c0 = (int64_t)blockIdx.x * kRT, q0i = (qt0 + blockIdx.y) * kRT;
  constexpr bool two = (MODE == KGE_RANK_TRANS || MODE == KGE_RANK_MUL) && HS;   // h-side: q1 too
  const int D = A.dim;
  // pairs (i, 2jp) and (i, 2jp + 1) side by side: the element ops run as
  // packed f32 (v_pk_add / v_pk_mul), each lane of a pair in the scalar order
  f2 acc[4][2];
#pragma unroll
  for (int i = 0; i < 4; ++i) acc[i][0] = acc[i][1] = f2{0.f, 0.f};
  // staging: thread t loads row (t >> 2) elements 4 (t & 3) .. +3 of each tile
  const int sr = tid >> 2, se = (tid & 3) * 4;
  const int64_t qr = q0i + sr, er = c0 + sr;
  const bool qv = qr < A.n, ev = er < A.E;
  // bitmap filter: the word holding this thread's four candidates, per query
  // (c0 is a multiple of 64, so 4 tc .. 4 tc + 3 share one word)
  uint32_t fmask[4] = {0u, 0u, 0u, 0u};
  if (A.fbits && c0 + 4 * tc < A.E) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int64_t q = q0i + 4 * tq + i;
      if (q < A.n) fmask[i] = A.fbits[q * A.fw + ((c0 + 4 * tc) >> 5)] >> (uint32_t)((4 * tc) & 31);
    }
  }
  for (int e0 = 0; e0 < D; e0 += kRC) {
    const int ne = min(kRC, D - e0);
    float a[4], b[4], x[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int c = e0 + se + u;
      const bool in = se + u < ne;
      a[u] = (qv && in) ? A.q0[qr * A.ldq + c] : 0.f;
      b[u] = (two && qv && in) ? A.q1[qr * A.ldq + c] : 0.f;
      x[u] = (ev && in) ? A.cand[er * A.cand_ld + c] : 0.f;
    }
    __syncthreads();   // the previous chunk is consumed
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      sq0[se + u][sr] = a[u];
      if (two) sq1[se + u][sr] = b[u];
      sx[se + u][sr] = x[u];
    }
    __syncthreads();
    for (int c = 0; c < ne; ++c) {
      const float4 qa = *reinterpret_cast<const float4*>(&sq0[c][4 * tq]);
      const float4 xa = *reinterpret_cast<const float4*>(&sx[c][4 * tc]);
      float4 qb = make_float4(0.f, 0.f, 0.f, 0.f);
      if (two) qb = *reinterpret_cast<const float4*>(&sq1[c][4 * tq]);
      const float qv0[4] = {qa.x, qa.y, qa.z, qa.w}, qv1[4] = {qb.x, qb.y, qb.z, qb.w};
      const f2 xp[2] = {f2{xa.x, xa.y}, f2{xa.z, xa.w}};
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const f2 a0 = f2{qv0[i], qv0[i]}, a1 = f2{qv1[i], qv1[i]};
#pragma unroll
        for (int jp = 0; jp < 2; ++jp) {
          const f2 xe = xp[jp];
          f2& ac = acc[i][jp];
          if (MODE == KGE_RANK_MUL) {
            ac = ac + (HS ? (xe * a0) * a1 : a0 * xe);
          } else if (MODE == KGE_RANK_DOT) {
            ac = ac + a0 * xe;
          } else if (SK == SK_DOT) {
            ac = ac + (HS ? (xe + a0) * a1 : a0 * xe);
          } else {
            const f2 d = HS ? (xe + a0) - a1 : a0 - xe;
            if (SK == SK_P2) {
              ac = ac + d * d;   // |d| |d| == d d bit for bit
            } else {
#pragma unroll
              for (int h = 0; h < 2; ++h) {
                const float m = fabsf(d[h]);
                if (SK == SK_P1) ac[h] = ac[h] + m;
                else if (SK == SK_PGEN) ac[h] = ac[h] + powf(m, A.p);
                else ac[h] = fmaxf(ac[h], m);
              }
            }
          }
        }
      }
    }
  }
  // strict > the query's true score; counts summed over the 16 lanes of a row
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int64_t q = q0i + 4 * tq + i;
    const float pv = q < A.n ? A.pos[q] : INFINITY;
    unsigned cnt = 0;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const float av = acc[i][j >> 1][j & 1];
      float sc;
      if (SK == SK_DOT || MODE == KGE_RANK_MUL || MODE == KGE_RANK_DOT) {
        sc = av;
      } else {
        float lpv;
        sc = score_value<SK>(av, A.pw, &lpv, A.p);
      }
      cnt += (c0 + 4 * tc + j < A.E && sc > pv && !((fmask[i] >> j) & 1u)) ? 1u : 0u;
    }
#pragma unroll
    for (int o = 1; o < 16; o <<= 1) cnt += (unsigned)__shfl_xor((int)cnt, o, KGE_WAVE);
    if (tc == 0 && q < A.n && cnt) atomicAdd(&A.rank[q], (unsigned long long)cnt);
  }
}

// Filter pass for the tiled modes: workgroup per query, its four waves take
// turns at 64 filtered entities per round, one per lane (a long filter list
// -- thousands of known heads of one (r, t) -- is spread over four waves). Their rows are staged through the wave's LDS 16
// elements at a time (float4 loads along each row, written transposed) so a
// lane sums its entity's elements in ascending order from LDS -- the same ops
// and order as rank_scores, hence exactly the scores the count pass compared
// -- without 64 scattered row reads per element.
template <int MODE, int SK>
__global__ __launch_bounds__(256) void rank_filter_tile_kernel(RankArgs A) {
#pragma clang fp contract(off)
  __shared__ __attribute__((aligned(16))) float sx[4][kRC][KGE_WAVE];
  __shared__ unsigned long long s_sub[4];
  const int lane = lane_id(), wv = wave_id();
  const int64_t q = blockIdx.x;
  unsigned long long sub = 0;
  if (A.fbeg) {
    const float pv = A.pos[q];
    const float* r0 = A.q0 + q * A.ldq;
    const float* r1 = (A.q1 && A.hside) ? A.q1 + q * A.ldq : nullptr;
    const int D = A.dim;
    float (*T)[KGE_WAVE] = sx[wv];
    for (int64_t j0 = A.fbeg[q] + wv * KGE_WAVE; j0 < A.fend[q]; j0 += 4 * KGE_WAVE) {
      const int cnt = (int)min<int64_t>(KGE_WAVE, A.fend[q] - j0);
      int64_t e = 0;
      bool ok = lane < cnt;
      if (ok) {
        e = load_idx(A.fent, j0 + lane, A.i64);
        if (e < 0 || e >= A.E) { set_status(A.status, KGE_ERANGE); ok = false; e = 0; }
      }
      float acc = 0.f;
      for (int e0 = 0; e0 < D; e0 += kRC) {
        const int ne = min(kRC, D - e0);
        // staging: 64 rows x 16 elements, four (row, element quad) per lane
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const int idx = k * KGE_WAVE + lane, r = idx >> 2, u0 = (idx & 3) * 4;
          const int64_t er = __shfl(e, r, KGE_WAVE);
          const bool rv = r < cnt;
#pragma unroll
          for (int u = 0; u < 4; ++u)
            T[u0 + u][r] = (rv && u0 + u < ne) ? A.cand[er * A.cand_ld + e0 + u0 + u] : 0.f;
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        for (int c = 0; c < ne; ++c) {
          const float xe = T[c][lane], a0 = r0[e0 + c];
          if (MODE == KGE_RANK_MUL) {
            acc = acc + (A.hside ? (xe * a0) * r1[e0 + c] : a0 * xe);
          } else if (MODE == KGE_RANK_DOT) {
            acc = acc + a0 * xe;
          } else if (SK == SK_DOT) {
            acc = acc + (A.hside ? (xe + a0) * r1[e0 + c] : a0 * xe);
          } else {
            const float m = fabsf(A.hside ? (xe + a0) - r1[e0 + c] : a0 - xe);
            if (SK == SK_P2) acc = acc + m * m;
            else if (SK == SK_P1) acc = acc + m;
            else if (SK == SK_PGEN) acc = acc + powf(m, A.p);
            else acc = fmaxf(acc, m);
          }
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      }
      float sc;
      if (SK == SK_DOT || MODE == KGE_RANK_MUL || MODE == KGE_RANK_DOT) {
        sc = acc;
      } else {
        float lpv;
        sc = score_value<SK>(acc, A.pw, &lpv, A.p);
      }
      sub += (ok && sc > pv) ? 1ull : 0ull;
    }
  }
  for (int o = 32; o >= 1; o >>= 1) sub += __shfl_xor(sub, o, KGE_WAVE);
  if (lane == 0) s_sub[wv] = sub;
  __syncthreads();
  if (threadIdx.x == 0) A.rank[q] = A.rank[q] - (s_sub[0] + s_sub[1] + s_sub[2] + s_sub[3]) + 1ull;
}

template <int MODE, int PJ, int SK>
static void rank_launch(const RankArgs& A, hipStream_t st) {
  hipLaunchKernelGGL((rank_pos_kernel<MODE, PJ, SK>), dim3((unsigned)((A.n + 255) / 256)), dim3(256), 0, st, A);
  const bool bits = A.fbits != nullptr;   // (the bitmap was built by launch_rank; no filter pass)
  if constexpr ((MODE == KGE_RANK_TRANS && PJ == KGE_RPROJ_NONE) || MODE == KGE_RANK_MUL || MODE == KGE_RANK_DOT) {
    const int64_t nct = (A.E + kRT - 1) / kRT, nqt = (A.n + kRT - 1) / kRT;
    constexpr int64_t kMaxY = 65535;
    if (!A.lane_pass && nct <= ((int64_t)1 << 31) - 1) {
      for (int64_t t0 = 0; t0 < nqt; t0 += kMaxY) {
        const dim3 grid((unsigned)nct, (unsigned)std::min(nqt - t0, kMaxY));
        if (A.hside) hipLaunchKernelGGL((rank_tile_kernel<MODE, SK, true>), grid, dim3(256), 0, st, A, t0);
        else hipLaunchKernelGGL((rank_tile_kernel<MODE, SK, false>), grid, dim3(256), 0, st, A, t0);
      }
      if (!bits) hipLaunchKernelGGL((rank_filter_tile_kernel<MODE, SK>), dim3((unsigned)A.n), dim3(256), 0, st, A);
      return;
    }
  }
  const int64_t nchunk = (A.E + kRankThreads - 1) / kRankThreads;
  const int64_t ng = (A.n + kRankQ - 1) / kRankQ;
  const size_t lds = (size_t)3 * kRankQ * ((A.dim + 3) & ~3) * 4;
  // grid limits: y <= 65535 chunks, x * 256 work-items < 2^32 per launch
  constexpr int64_t kMaxY = 65535, kMaxX = (int64_t)1 << 22;
  for (int64_t c0 = 0; c0 < nchunk; c0 += kMaxY)
    for (int64_t g0 = 0; g0 < ng; g0 += kMaxX)
      hipLaunchKernelGGL((rank_count_kernel<MODE, PJ, SK>),
                         dim3((unsigned)std::min(ng - g0, kMaxX), (unsigned)std::min(nchunk - c0, kMaxY)),
                         dim3(kRankThreads), lds, st, A, g0, c0);
  if (!bits) hipLaunchKernelGGL((rank_filter_kernel<MODE, PJ, SK>), dim3((unsigned)((A.n + 3) / 4)), dim3(256), 0, st, A);
}

template <int MODE, int PJ>
static void rank_by_sk(const RankArgs& A, int sk, hipStream_t st) {
  switch (sk) {
    case SK_P1: rank_launch<MODE, PJ, SK_P1>(A, st); break;
    case SK_P2: rank_launch<MODE, PJ, SK_P2>(A, st); break;
    case SK_PINF: rank_launch<MODE, PJ, SK_PINF>(A, st); break;
    case SK_PGEN: rank_launch<MODE, PJ, SK_PGEN>(A, st); break;
    default: rank_launch<MODE, PJ, SK_DOT>(A, st); break;
  }
}

kge_status launch_rank(const RankArgs& A, int mode, int proj, int sk, hipStream_t st) {
  if (A.fbits) {   // the filter bitmap, before the passes that read it
    uint32_t* bits = const_cast<uint32_t*>(A.fbits);
    if (A.fw <= kBitsLds) {
      hipLaunchKernelGGL(rank_bits_kernel<true>, dim3((unsigned)A.n), dim3(256), 0, st, A, bits);
    } else {
      (void)hipMemsetAsync(bits, 0, (size_t)(A.n * A.fw) * sizeof(uint32_t), st);
      hipLaunchKernelGGL(rank_bits_kernel<false>, dim3((unsigned)A.n), dim3(256), 0, st, A, bits);
    }
  }
  switch (mode) {
    case KGE_RANK_TRANS:
      if (proj == KGE_RPROJ_HYPER) rank_by_sk<KGE_RANK_TRANS, KGE_RPROJ_HYPER>(A, sk, st);
      else if (proj == KGE_RPROJ_RANK1) rank_by_sk<KGE_RANK_TRANS, KGE_RPROJ_RANK1>(A, sk, st);
      else rank_by_sk<KGE_RANK_TRANS, KGE_RPROJ_NONE>(A, sk, st);
      return KGE_OK;
    case KGE_RANK_ROT:
      if (sk == SK_DOT) return KGE_EUNSUPPORTED;
      rank_by_sk<KGE_RANK_ROT, KGE_RPROJ_NONE>(A, sk, st);
      return KGE_OK;
    case KGE_RANK_MUL: rank_launch<KGE_RANK_MUL, KGE_RPROJ_NONE, SK_DOT>(A, st); return KGE_OK;
    case KGE_RANK_DOT: rank_launch<KGE_RANK_DOT, KGE_RPROJ_NONE, SK_DOT>(A, st); return KGE_OK;
    default: return KGE_EUNSUPPORTED;
  }
}

}  // namespace kge
