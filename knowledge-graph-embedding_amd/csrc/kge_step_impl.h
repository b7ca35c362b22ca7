// Fused KGE training step for gfx950 -- kernel templates (score / update).
// Instantiated per model family in kge_step_<family>.hip (parallel builds);
// kge_step.hip holds the non-template kernels and the dispatch.
//
// One reference batch step (KGEModel.__run_single_batch, BaseModel.py:293-330)
// runs as stream-ordered kernels:
//
//   K0  constrain   full-table row renormalisation of ent_emb when the model's
//                   _constraint_loss assigns it (TransE.py:171-172,
//                   DistMult.py:162-163).
//   KS  score       8-wave workgroups, `wpp` waves per positive. In-register
//                   Philox negative draws (ns_strategy.py:39-64 in the layout
//                   of BaseModel.py:332-408); each wave streams its slots'
//                   rows in register batches (gather -> forward -> ONE
//                   transposed multi-reduction per batch -> loss weight ->
//                   backward), with SANS's softmax folded in online (loss.py
//                   :174-182), so every sampled row is read exactly once. The
//                   positive's own rows are reduced on chip; every negative
//                   leaves one (alpha, value) coefficient and its destination
//                   key, filed straight into that destination's list (one
//                   int atomic per key). The last workgroup reduces the
//                   loss and the per-variable gradient norms (clip_by_norm,
//                   BaseModel.py:327) in a fixed order.
//   KU  update      destination-major, one wave per entity / relation row:
//                   its keys in ascending code order (bit-reproducible sums,
//                   no float atomics), each negative's row gradient re-derived
//                   from ONE frozen context row + its coefficient, the
//                   positives' own row gradients added, clip scale and SGD
//                   (BaseModel.py:328, keras SGD ResourceScatterAdd) applied
//                   with ONE read-modify-write per touched row.
#pragma once
#include <utility>

#include "kge_step.h"

#ifndef KGE_SCORE_PREFETCH
#define KGE_SCORE_PREFETCH 0   // score kernel: software-pipelined row batches (tuning knob)
#endif
#ifndef KGE_STREAM_ROWS
#define KGE_STREAM_ROWS 8   // sampled rows per stream batch at NC = 1 (tuning knob)
#endif
#ifndef KGE_UPD_COMPACT_WPE
#define KGE_UPD_COMPACT_WPE 8   // compact update launch: amdgpu_waves_per_eu (tuning knob)
#endif
#ifndef KGE_UPD_COMPACT_U
#define KGE_UPD_COMPACT_U 4     // compact update launch (8 waves / SIMD): entries in flight (tuning knob)
#endif
#ifndef KGE_UPD_WIDE_WPE
#define KGE_UPD_WIDE_WPE 1      // update launches of wide rows (NC >= 2 or WIDE): amdgpu_waves_per_eu (tuning knob)
#endif
#ifndef KGE_COMPACT_LIST0
#define KGE_COMPACT_LIST0 1 // compact launches: list position 0 lives only in the leader table (A-B knob)
#endif
#ifndef KGE_GUARD_KU
#define KGE_GUARD_KU 1      // update kernel: workspace plan guard at entry (tuning / A-B knob)
#endif
#ifndef KGE_FILE_EARLY
// score kernel: when the negatives' keys are filed. 2 (default): each lane's
// slot claims its destination (counter add / hash-slot CAS) right after the
// row stream and stores the code after the merge barrier, so the claim's
// round trip hides under the barrier wait and the merge (C2 KS 53.7 -> 48.7
// us, profiles/r06e); 1: claims after the first batch's loads (slower: 55.4);
// 0: claim and store in the finalise pass (A-B knob)
#define KGE_FILE_EARLY 2
#endif
#ifndef KGE_CTX_LATE
#define KGE_CTX_LATE 1      // score kernel: the positive's context rows finished after the first row batch's
                            // loads are issued (one dependent round trip fewer per wave) (A-B knob)
#endif
#ifndef KGE_UPDATE_U
#define KGE_UPDATE_U 8      // update kernel: list entries in flight per wave at NC = 1 (tuning knob)
#endif

namespace kge {

#ifdef KGE_PHASE_PROF
// one counter array per translation unit (no relocatable device code): each
// profiled TU exports its own reader (kge_prof_read, kge_trprof_read)
static __device__ unsigned long long g_kge_prof[64];
#endif

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

__device__ __forceinline__ float bcast(float v, int lane) {
  return __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), lane));
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

// dL/ds of one negative (loss.py); SANS with its positive's final softmax
// reference max Ms and 1/Z
__device__ __forceinline__ float neg_coef(const StepArgs& A, float s, float sp, float Ms, float invZ) {
  switch (A.loss_kind) {
    case KGE_LOSS_HINGE: return (A.margin + s - sp >= 0.f) ? A.inv_bk : 0.f;
    case KGE_LOSS_LOGISTIC: { const float ex = expf(s - sp); return ex / (1.f + ex); }
    case KGE_LOSS_BCE: return sigmoid(s) * A.inv_b;
    case KGE_LOSS_SANS: return expf(A.temperature * s - Ms) * invZ * sigmoid(s + A.margin) * A.inv_b;
    default: return s * A.inv_b;
  }
}

// one destination key: append its code to the destination's list (arrival
// order), or to the overflow list once that list is full. Compact launches:
// the list is the destination's hash slot's (one 64-bit CAS claims an empty
// slot -- the common case on a large table -- else one atomic add on the
// slot that holds the destination), and the key's position in the leader
// table records (destination, code if it took list position 0, slot);
// positives' keys first (they hold the longest lists -- relation rows,
// skewed entities -- which then start early instead of forming the update
// launch's tail), then the negatives'
struct KeyClaim {
  uint32_t r;               // list position the key took (compact: resolved by bin_commit)
  uint32_t h;               // compact launches: its hash slot
  unsigned long long cur;   // compact launches: what the first CAS found
};
// The returning half of bin_key, issued: the destination's counter (one
// atomic add) or, compact launches, the first compare-and-swap on the
// destination's hash slot. Nothing here waits for the result, so the
// score kernel can issue its keys' claims and go on (early filing):
// bin_commit uses the results.
__device__ __forceinline__ KeyClaim bin_claim(const StepArgs& A, int64_t dest) {
  KeyClaim c;
  if (A.compact) {
    const unsigned long long key = (unsigned long long)((uint32_t)dest + 1u) << 32;
    c.h = ((uint32_t)dest * 2654435761u) >> A.hshift;
    c.cur = atomicCAS(&A.htab[c.h], 0ull, key | 1ull);
    c.r = 0u;
  } else {
    c.r = atomicAdd(&A.cnt[dest], 1u);
    c.h = 0u;
    c.cur = 0ull;
  }
  return c;
}
// The storing half: compact launches first finish the claim (an empty slot
// taken -- the common case on a large table -- or one atomic add on the
// slot that holds the destination, else probe on: the table has >= 2x as
// many slots as keys), then the code goes into the destination's list at
// the claimed position (the overflow list past capacity) and compact
// launches record the key's leader-table entry
__device__ __forceinline__ void bin_commit(const StepArgs& A, int64_t dest, uint32_t code, KeyClaim c,
                                           uint32_t kpos_own = ~0u) {
  int64_t li = dest;   // list index
  if (A.compact) {
    const unsigned long long key = (unsigned long long)((uint32_t)dest + 1u) << 32;
    for (;;) {
      if (c.cur == 0ull) { c.r = 0u; break; }
      if ((c.cur & 0xFFFFFFFF00000000ull) == key) { c.r = (uint32_t)atomicAdd(&A.htab[c.h], 1ull); break; }
      c.h = (c.h + 1u) & A.hmask;
      c.cur = atomicCAS(&A.htab[c.h], 0ull, key | 1ull);
    }
    li = c.h;
    // (the owner pass hands each key its position in the workgroup's block)
    const uint32_t kpos = kpos_own != ~0u ? kpos_own
        : code < A.nkeyneg
        ? A.npos3 + (code >> A.kshift) * (uint32_t)A.Keff + (code & ((1u << A.kshift) - 1u))
        : 3u * ((code - A.nkeyneg) >> 2) + ((code - A.nkeyneg) & 3u);
    A.leaders[kpos] = make_uint4((uint32_t)dest, c.r == 0u ? code : 0xFFFFFFFFu, c.h, 0u);
    // position 0's code is the leader table's (a 50M-row table's destinations
    // mostly hold one key: no scattered list store for them at all)
    if (KGE_COMPACT_LIST0 && c.r == 0u) return;
  }
  if (c.r < (uint32_t)A.cap) {
    A.list[li * A.cap + c.r] = code;
  } else {
    const uint32_t o = atomicAdd(&A.ctl->ovf_count, 1u);
    A.ovf[o] = ((uint64_t)dest << 32) | code;
  }
}
__device__ __forceinline__ void bin_key(const StepArgs& A, int64_t dest, uint32_t code, uint32_t kpos_own = ~0u) {
  bin_commit(A, dest, code, bin_claim(A, dest), kpos_own);
}

// global entity id -> its row of the step's entity table, range-checked:
// the identity, or (multi-GPU, KGE/sharded.py) the row of id e in the
// all-gathered shards, (e mod G) * shard_rows + e div G
__device__ __forceinline__ int64_t ent_row(const StepArgs& A, int64_t e, int* err) {
  if (e < 0 || e >= A.n_ent) { *err = KGE_ERANGE; return 0; }
  return A.rG > 1 ? (e % A.rG) * A.rEs + e / A.rG : e;
}

// slot j of positive i: its entity id (drawn, or read from the caller's
// negatives), bounds-checked; a drawn id is handed back when asked
__device__ __forceinline__ int32_t slot_entity(const StepArgs& A, int64_t i, int j, int* err) {
  int kind; uint64_t n, poff;
  slot_layout(A.side_mode, A.Kside, i, j, &kind, &n, &poff);
  int64_t e;
  if (A.given) {
    e = load_idx(A.neg_user, i * A.Keff + j, A.i64);
  } else {
    const int64_t x = load_idx(A.pos, i * 3 + (kind == KIND_HC ? 0 : 2), A.i64);
    if (A.smp.kind == KGE_SAMPLER_TYPED && (x < 0 || x >= A.n_ent)) { e = 0; *err = KGE_ERANGE; }
    else {
      e = sample_entity(A.smp, A.smp.offset + poff, n, x, err);   // plane offset (+1 for the t side)
      if (e < 0) e = 0;
    }
    if (A.neg_user) store_idx(A.neg_user, i * A.Keff + j, e, A.i64);
  }
  return (int32_t)ent_row(A, e, err);
}

// owner pass: slot j of virtual positive v = q * own_Bq + i (rank q's
// positive i), drawn as rank q's own step draws it -- its planes start at
// offset + q * own_planes (KGE/sharded.py's rank-disjoint planes) -- or read
// from the all-gathered given negatives; the local row if this rank owns the
// entity (e mod own_G == own_g: row e div own_G), else -1
__device__ __forceinline__ int32_t owner_slot(const StepArgs& A, int64_t v, int j, int* err) {
  const int64_t q = v / A.own_Bq, i = v - q * A.own_Bq;
  int kind; uint64_t n, poff;
  slot_layout(A.side_mode, A.Kside, i, j, &kind, &n, &poff);
  int64_t e;
  if (A.given) {
    e = load_idx(A.neg_user, v * A.Keff + j, A.i64);
  } else {
    const int64_t x = load_idx(A.pos, v * 3 + (kind == KIND_HC ? 0 : 2), A.i64);
    if (A.smp.kind == KGE_SAMPLER_TYPED && (x < 0 || x >= A.n_ent)) { *err = KGE_ERANGE; return -1; }
    e = sample_entity(A.smp, A.smp.offset + (uint64_t)q * (uint64_t)A.own_planes + poff, n, x, err);
    if (e < 0) return -1;   // (the sampler reported it)
  }
  if (e < 0 || e >= A.n_ent) { *err = KGE_ERANGE; return -1; }
  return (e % A.own_G) == A.own_g ? (int32_t)(e / A.own_G) : -1;
}

// compile-time loop over u = 0 .. N-1 (fn gets std::integral_constant<int, u>)
template <class Fn, int... Is>
__device__ __forceinline__ void static_for_impl(Fn& fn, std::integer_sequence<int, Is...>) {
  (fn(std::integral_constant<int, Is>{}), ...);
}
template <int N, class Fn>
__device__ __forceinline__ void static_for(Fn&& fn) {
  static_for_impl(fn, std::make_integer_sequence<int, N>{});
}

// models whose context load comes in two halves (load_ctx_raw, ctx_finish)
template <class M, class = void> struct ctx_split { static constexpr bool v = false; };
template <class M>
struct ctx_split<M, std::void_t<decltype(&M::ctx_finish)>> { static constexpr bool v = true; };

// corruption kind of row u of a stream batch (batches start on an even slot:
// 'h+t' slots alternate h-corrupt / t-corrupt, BaseModel.py:353-356)
template <int SIDE>
__host__ __device__ constexpr int kind_at(int u) {
  return SIDE == KGE_SIDE_HT ? ((u & 1) ? KIND_TC : KIND_HC) : SIDE == KGE_SIDE_H ? KIND_HC : KIND_TC;
}

// element i of a row fragment, as a wave-uniform scalar (i wave-uniform)
template <int VEC, int NC>
__device__ __forceinline__ float frag_elem_bcast(const Frag<VEC, NC>& f, int i) {
  const int c = i / (KGE_WAVE * VEC), rem = i - c * KGE_WAVE * VEC;
  const int q = c * VEC + rem % VEC;
  float v = 0.f;
#pragma unroll
  for (int k = 0; k < VEC * NC; ++k) v = k == q ? f.v[k] : v;
  return bcast(v, rem / VEC);
}

// RESCAL context products of one positive (RESCAL.py:166-171), shared by its
// waves: this wave takes rows [rb, re) of R (row i at Rm + i d) in batches
// of 16 (every row's load issued before use) and accumulates
//   u-like  up += x_i R_i            (u = R^T x: the wave's partial)
//   v-like  vl[i] = R_i . y          (v = R y: one transposed 8-row reduction)
// The callers sum the waves' partials of u in wave order (LDS).
template <int VEC, int NC>
__device__ void rel_gemv_pair(const float* __restrict__ Rm, int d, int rb, int re, const Frag<VEC, NC>& x,
                              const Frag<VEC, NC>& y, Frag<VEC, NC>& up, float* vl) {
  using F = Frag<VEC, NC>;
  constexpr int NB = 16, SH = 2;   // lane l holds row (l >> SH) of the batch after multi_reduce
  up.zero();
  for (int i0 = rb; i0 < re; i0 += NB) {
    F Rr[NB];   // rows past re repeat the last one (weight 0, result dropped)
#pragma unroll
    for (int u = 0; u < NB; ++u) load_row(Rr[u], Rm + (int64_t)min(i0 + u, re - 1) * d, d);
    float part[NB];
#pragma unroll
    for (int u = 0; u < NB; ++u) {
      const float xi = i0 + u < re ? frag_elem_bcast(x, i0 + u) : 0.f;
      float p = 0.f;
#pragma unroll
      for (int q = 0; q < VEC * NC; ++q) {
        up.v[q] += xi * Rr[u].v[q];
        p += Rr[u].v[q] * y.v[q];
      }
      part[u] = p;
    }
    const float vr = multi_reduce<NB, false>(part);
    const int u = lane_id() >> SH;
    if ((lane_id() & ((1 << SH) - 1)) == 0 && i0 + u < re) vl[i0 + u] = vr;
  }
}

// per-positive merge slots (LDS)
enum { MG_F = 0, MG_AP = kMaxWpp, MG_LOSS = kMaxWpp + 1, MG_N = kMaxWpp + 2, MG_UN = kMaxWpp + 8,
       MG_RP = kMaxWpp + 12, MG_TP = kMaxWpp + 13, MG_SP = kMaxWpp + 14, MG_LPP = kMaxWpp + 15,
       MG_RSQ = kMaxWpp + 16, MG_MS = kMaxWpp + 17, MG_IZ = kMaxWpp + 18,
       MG_NH = kMaxWpp + 19, MG_KC = kMaxWpp + 20, MG_KB = kMaxWpp + 21,   // owner pass: h slots, slots, key base
       MG_STRIDE = kMergeStride };
static_assert(MG_KB < MG_STRIDE, "merge slots exceed the LDS stride");

// ------------------------------------------------------------ KS score
// One workgroup = kStepWaves waves = nP positives x wpp waves. A wave owns
// SW consecutive negative slots of its positive and streams them in batches
// of ROWS rows held in registers: gather (one global_load_dwordx4 per row
// per lane), forward, ONE transposed multi-reduction for the whole batch,
// per-row loss weight computed by the lanes that hold that row's score,
// analytic backward into the positive's h / r / t accumulators. SANS's
// softmax is folded in online (running max; accumulators rescaled when it
// grows), so no row outlives its batch and no row is read twice. The
// positive's waves merge their states through LDS; then every wave
// finalises its slots' coefficients and files every destination key into
// that destination's list for the update kernel.
//
// OWN (KGE_FLAG_OWNER, the multi-GPU owner-side scoring pass): the batch is
// the virtual batch of every rank's positives; each positive's waves draw its
// slots from its rank's counter planes, keep the slots whose entity this rank
// owns, compact them per corruption side (h-corrupt slots, then t-corrupt),
// stream those, and leave a record (partial softmax state, loss / norm
// partials, the h / r / t accumulators) instead of finishing the positive;
// its keys go to per-workgroup blocks of key positions (own_codes).
template <template <int, int, int> class Model, int VEC, int NC, int SK, int SIDE, bool OWN = false>
__global__ __launch_bounds__(kStepThreads) __attribute__((amdgpu_waves_per_eu((NC >= 2 || Model<VEC, NC, SK>::WIDE) ? KGE_SCORE_WPE_WIDE : KGE_SCORE_WPE))) void score_kernel(StepArgs A) {
  using M = Model<VEC, NC, SK>;
  using F = Frag<VEC, NC>;
  constexpr int W = kStepWaves;
  constexpr int FL = KGE_WAVE * VEC * NC;   // floats per fragment image
  constexpr int ROWS = KGE_STREAM_ROWS / NC > 1 ? KGE_STREAM_ROWS / NC : 2;   // rows per batch (in registers)
  constexpr int SH = ROWS == 16 ? 2 : ROWS == 8 ? 3 : ROWS == 4 ? 4 : 5;   // lane l holds row l >> SH after multi_reduce
  constexpr int LPR = 1 << SH;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];

  const int Keff = A.Keff, nP = A.nP, wpp = A.wpp;
  const ScoreLds L = score_lds(FL, nP, Keff, OWN);
  int64_t* s_pos = reinterpret_cast<int64_t*>(smem + L.pos);
  int32_t* s_ids = reinterpret_cast<int32_t*>(smem + L.ids);
  float* s_R = reinterpret_cast<float*>(smem + L.sR);
  float* s_T = reinterpret_cast<float*>(smem + L.sT);
  float* s_st = reinterpret_cast<float*>(smem + L.st);
  float* s_mrg = reinterpret_cast<float*>(smem + L.mrg);
  float* red = reinterpret_cast<float*>(smem + L.red);
  float* posg = reinterpret_cast<float*>(smem + L.posg);
  float* s_misc = reinterpret_cast<float*>(smem + L.misc);
  __shared__ int s_last;

  if (ws_refused(A.ctl, A.sig, A.status, A.loss_out)) return;
  KGE_PROF_INIT();
  const int tid = threadIdx.x, lane = lane_id(), wv = wave_id();
  const int grp = wv / wpp, gw = wv % wpp;
  int err = 0;

  const int64_t i0 = (int64_t)blockIdx.x * nP;
  const int nValid = (int)min<int64_t>((int64_t)nP, A.B - i0);

  const bool active = grp < nValid;
  const int64_t i = i0 + grp;
  const MP mp{A.limit, A.fuse_norm, A.snap + (active ? i : 0) * (M::NSNAP * (int64_t)A.snap_cols)};
  const int jbeg = min(Keff, gw * A.SW);
  const int jend = min(Keff, jbeg + A.SW);
  int32_t* ids = s_ids + grp * Keff;
  float* gR = s_R + grp * Keff;
  float* gT = s_T + grp * Keff;

  // every wave fetches its positive's ids and draws its own slots (no
  // workgroup barrier: the slots' ids are read back by this wave only)
  int64_t ph = 0, pr = 0, pt = 0;
  if (active) {
    if constexpr (OWN) {
      // the caller's gathered copies of the positive's rows; its global ids
      // stay in pos (typed draws, the all-gathered triples)
      ph = A.own_rows_from + 2 * i;
      pt = ph + 1;
      pr = load_idx(A.pos, i * 3 + 1, A.i64);
    } else {
      ph = load_idx(A.pos, i * 3 + 0, A.i64);
      pr = load_idx(A.pos, i * 3 + 1, A.i64);
      pt = load_idx(A.pos, i * 3 + 2, A.i64);
      ph = ent_row(A, ph, &err);
      pt = ent_row(A, pt, &err);
    }
    if (pr < 0 || pr >= A.rel.rows) { err = KGE_ERANGE; pr = 0; }
    if (gw == 0 && lane < 3) s_pos[grp * 3 + lane] = lane == 0 ? ph : lane == 1 ? pr : pt;
    if constexpr (OWN) {
      for (int j = jbeg + lane; j < jend; j += KGE_WAVE) ids[j] = owner_slot(A, i, j, &err);
    } else {
      for (int j = jbeg + lane; j < jend; j += KGE_WAVE) ids[j] = slot_entity(A, i, j, &err);
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  }
  // owner pass: the positive's owned slots compacted by its first wave --
  // rows into crow, slot numbers into jmap: h-corrupt slots [0, nh), then
  // t-corrupt [nh, Kc) -- and each wave's ranges of both; the workgroup's
  // key positions taken in one block (one atomic per workgroup)
  int hb = 0, he = 0, tb = 0, te = 0;
  int32_t* jmap = nullptr;
  if constexpr (OWN) {
    int32_t* crow = reinterpret_cast<int32_t*>(smem + L.jmap) + nP * Keff + grp * Keff;
    jmap = reinterpret_cast<int32_t*>(smem + L.jmap) + grp * Keff;
    float* mgo = s_mrg + grp * MG_STRIDE;
    __syncthreads();
    if (active && gw == 0) {
      int base = 0, nh = 0;
      for (int pass = 0; pass < (SIDE == KGE_SIDE_HT ? 2 : 1); ++pass) {
        const int kind = SIDE == KGE_SIDE_HT ? (pass ? KIND_TC : KIND_HC) : kind_at<SIDE>(0);
        for (int c0 = 0; c0 < Keff; c0 += KGE_WAVE) {
          const int j = c0 + lane;
          const int32_t rw = j < Keff ? ids[j] : -1;
          const bool own = j < Keff && rw >= 0 && slot_kind(A.side_mode, j) == kind;
          const uint64_t m = __ballot(own);
          if (own) {
            const int c = base + __popcll(m & ((1ull << lane) - 1ull));
            crow[c] = rw;
            jmap[c] = j;
          }
          base += __popcll(m);
        }
        if (pass == 0) nh = base;
      }
      if (lane == 0) { mgo[MG_NH] = (float)nh; mgo[MG_KC] = (float)base; }
    }
    __syncthreads();
    if (tid == 0) {   // this workgroup's block of key positions
      int tot = 0;
      for (int p = 0; p < nValid; ++p) tot += (int)s_mrg[p * MG_STRIDE + MG_KC];
      const uint32_t b0 = tot ? atomicAdd(&A.ctl->own_count, (uint32_t)tot) : 0u;
      int o = 0;
      for (int p = 0; p < nValid; ++p) {
        s_mrg[p * MG_STRIDE + MG_KB] = __builtin_bit_cast(float, b0 + (uint32_t)o);
        o += (int)s_mrg[p * MG_STRIDE + MG_KC];
      }
    }
    __syncthreads();
    ids = crow;
    if (active) {
      const int nh = (int)mgo[MG_NH], kc = (int)mgo[MG_KC], nt = kc - nh;
      const int swh = (nh + wpp - 1) / wpp, swt = (nt + wpp - 1) / wpp;
      hb = min(nh, gw * swh); he = min(nh, hb + swh);
      tb = nh + min(nt, gw * swt); te = nh + min(nt, gw * swt + swt);
    }
  }
  KGE_PROF(0);

  // early filing (KGE_FILE_EARLY): this lane's slot jbeg + lane, its claim
  // (not for the wide instances -- rows of two chunks, RotatE, DistMult: their
  // 2-waves-per-SIMD budget is nearly full and the claims' registers spilled)
  constexpr bool NARROW = !(NC >= 2 || M::WIDE);
  const bool early = KGE_FILE_EARLY != 0 && NARROW && !OWN && A.train && A.SW <= KGE_WAVE;
  const int jfile = jbeg + lane;
  int64_t kdest = 0;
  KeyClaim kc{0u, 0u};
  auto claim_early = [&]() {
    __builtin_amdgcn_sched_barrier(0);   // (after the batch's row loads, not before them)
    if (jfile < jend) { kdest = ids[jfile]; kc = bin_claim(A, kdest); }
    __builtin_amdgcn_sched_barrier(0);
  };
  auto commit_early = [&]() {
    if (jfile < jend) bin_commit(A, kdest, ((uint32_t)i << A.kshift) | (uint32_t)jfile, kc);
  };
  // the owner pass's early filing: its two ranges' claims (h-corrupt, t-corrupt)
  bool early_own = false;
  KeyClaim kco[2] = {{0u, 0u, 0ull}, {0u, 0u, 0ull}};
  typename M::Ctx ctx;
  float Mrun = -INFINITY, Zs = 0.f, csum = 0.f;
  float nrm[4] = {0.f, 0.f, 0.f, 0.f};
  F accH, accR, accT;
  accH.zero(); accR.zero(); accT.zero();
  float Rp = 0.f, tp = 1.f, sp = 0.f, lpp = 0.f;
  if constexpr (M::SELF_CTX) {
    // the positive's waves compute its context rows together (Rescal):
    // u = R^T h (waves' partials summed in wave order), v = R t (each entry
    // from the wave owning its row) -- through the wave's slices of `red`
    const int d = A.ent.cols;
    const int rpw = ((d + wpp - 1) / wpp + 7) & ~7;
    const int rb = min(d, gw * rpw), re = min(d, rb + rpw);
    float* myred = red + wv * 3 * FL;
    for (int e = lane; e < FL; e += KGE_WAVE) myred[FL + e] = 0.f;
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    F up;
    up.zero();
    if (active) {
      load_row(ctx.H, A.ent.row(ph), d);
      load_row(ctx.T, A.ent.row(pt), d);
      rel_gemv_pair<VEC, NC>(A.rel.row(pr), d, rb, re, ctx.H, ctx.T, up, myred + FL);
    }
#pragma unroll
    for (int q = 0; q < VEC * NC; ++q) myred[(q / VEC * KGE_WAVE + lane) * VEC + q % VEC] = up.v[q];
    __syncthreads();
    if (active) {
      ctx.U.zero();
      ctx.V.zero();
      for (int g = 0; g < wpp; ++g) {
        const float* gr = red + (grp * wpp + g) * 3 * FL;
#pragma unroll
        for (int q = 0; q < VEC * NC; ++q) {
          const int e = (q / VEC * KGE_WAVE + lane) * VEC + q % VEC;
          ctx.U.v[q] += gr[e];
          ctx.V.v[q] += gr[FL + e];
        }
      }
      if (gw == 0 && A.train) {   // the update kernel's context rows (snap)
        float* sn = A.snap + i * (M::NSNAP * (int64_t)A.snap_cols);
        store_row(ctx.U, sn, d);
        store_row(ctx.V, sn + A.snap_cols, d);
      }
    }
    __syncthreads();   // `red` is reused for the wave states below
  }
  // KGE_CTX_LATE: the context rows' loads go out now, their combination (and
  // the positive's score) after the first row batch's loads are issued
  constexpr bool LATE = KGE_CTX_LATE && NARROW && !OWN && ctx_split<M>::v;   // (wide instances: it spilled, C3)
  bool ctx_done = !LATE;
  if constexpr (!M::SELF_CTX) {
    if (active) {
      if constexpr (LATE) M::load_ctx_raw(ctx, A.ent, A.rel, ph, pr, pt);
      else M::load_ctx(ctx, A.ent, A.rel, ph, pr, pt, mp);
    }
  }
  // the positive's score, in every wave (hinge / logistic weights need it)
  auto pos_score = [&]() {
    if constexpr (LATE) M::ctx_finish(ctx, mp);
    F a, b, E0;
    E0.zero();
    M::fwd(ctx, KIND_POS, E0, a, b);
    const float part = score_partial<SK, M::CPLX>(a, b, A.p);
    Rp = lane_reduce<5, SK == SK_PINF>(part);
    if (SK == SK_PINF) tp = lane_reduce<5, false>(tie_partial<M::CPLX>(a, Rp));
    sp = score_value<SK>(Rp, A.pw, &lpp, A.p);
    ctx_done = true;
  };
  if (active) {
    if (!LATE) pos_score();
    const int lrow = lane >> SH;
    const bool lead = (lane & (LPR - 1)) == 0;
    // RAW: unmasked row loads, only the score partial masked (NRM_FROM_R
    // models keep no per-element norm, single-chunk rows)
    constexpr bool RAW = M::NRM_FROM_R && NC == 1;
    const bool lane_in = lane * VEC < A.ent.cols;
    int idv = 0;   // the wave's next 64 slot ids, one per lane
    // every row's load is issued before any is used; rows past the slot
    // range repeat the last valid row (finite values, weight 0)
    // (NRM_FROM_R models: lanes past the row's end keep whatever they
    // loaded and only their score partial is masked -- their accumulator
    // lanes are never read back)
    // (the stream's range [sb, se) comes in by value: one range per call)
    auto issue = [&](F (&dst)[ROWS], int jb, const int sb, const int se) {
      if (((jb - sb) & (KGE_WAVE - 1)) == 0) idv = (jb + lane < se) ? ids[jb + lane] : 0;
      const int jo = (jb - sb) & (KGE_WAVE - 1);
      const int nr = min(ROWS, se - jb);
#pragma unroll
      for (int u = 0; u < ROWS; ++u) {
        const float* row = A.ent.row(__builtin_amdgcn_readlane(idv, jo + min(u, nr - 1)));
        if (RAW) load_row_raw(dst[u], row, A.ent.cols);
        else load_row(dst[u], row, A.ent.cols);
      }
    };
    // KGE_SCORE_PREFETCH: the next batch's rows are in flight while this
    // batch is reduced and differentiated (one more batch of registers)
    // one range [sb, se) of slots whose corruption kinds follow the
    // pattern S2 (the launch's side; the owner pass: one side per range).
    // LK: the loss kind when known at compile time (SANS, the configs' loss:
    // its loop carries no branch of the other kinds), else -1 (A.loss_kind)
    auto stream = [&](auto sidec, auto lkc, const int sb, const int se) {
    constexpr int S2 = decltype(sidec)::value;
    constexpr int LK = decltype(lkc)::value;
    const int lk = LK >= 0 ? LK : A.loss_kind;
    F En[KGE_SCORE_PREFETCH ? ROWS : 1];
    if constexpr (KGE_SCORE_PREFETCH) issue(En, sb, sb, se);
    for (int j0 = sb; j0 < se; j0 += ROWS) {
      const int nrow = min(ROWS, se - j0);   // wave-uniform, >= 1
      F E[ROWS];
      if constexpr (KGE_SCORE_PREFETCH) {
#pragma unroll
        for (int u = 0; u < ROWS; ++u) E[u] = En[u];
        if (j0 + ROWS < se) issue(En, j0 + ROWS, sb, se);
      } else {
        issue(E, j0, sb, se);
      }
      if constexpr (KGE_FILE_EARLY == 1 && !OWN) {
        if (early && j0 == sb) claim_early();
      }
      if constexpr (LATE) {
        if (!ctx_done) pos_score();
      }
      if (A.fuse_norm) {
        // fused _constraint_loss: each sampled row normalised in registers
        // (one transposed reduction for the batch; same tree as lane_reduce)
        float sq[ROWS];
#pragma unroll
        for (int u = 0; u < ROWS; ++u) sq[u] = (!RAW || lane_in) ? norm_partial(E[u]) : 0.f;
        const float inv = inv_norm(multi_reduce<ROWS, false>(sq));
#pragma unroll
        for (int u = 0; u < ROWS; ++u) scale_row(E[u], bcast(inv, u << SH));
      }
      F a[ROWS], b[ROWS];
      float part[ROWS];
      static_for<ROWS>([&](auto uc) {
        constexpr int u = decltype(uc)::value;
        M::template fwdk<kind_at<S2>(u)>(ctx, E[u], a[u], b[u]);
        float pu;
        if constexpr (M::FAST_STREAM) pu = M::template fast_partial<SK>(a[u], b[u]);
        else pu = score_partial<SK, M::CPLX>(a[u], b[u], A.p);
        part[u] = (u < nrow && (!RAW || lane_in)) ? pu : 0.f;
      });
      const float Rl = multi_reduce<ROWS, SK == SK_PINF>(part);
      float tl = 1.f;
      if constexpr (SK == SK_PINF) {
        float tq[ROWS];
#pragma unroll
        for (int u = 0; u < ROWS; ++u) tq[u] = u < nrow ? tie_partial<M::CPLX>(a[u], bcast(Rl, u << SH)) : 0.f;
        tl = multi_reduce<ROWS, false>(tq);
      }
      const int j = j0 + lrow;
      const bool valid = lrow < nrow;
      // this lane's row weight dL/ds (loss.py; the loss VALUE is summed in
      // the finalise pass), hardware-rate transcendentals
      float lp;
      const float s = score_value_fast<SK>(Rl, A.pw, &lp, A.p);
      float c = 0.f;
      switch (lk) {
        case KGE_LOSS_HINGE: {
          // the hinge's on/off decision is the finalise pass's (IEEE score), so
          // a negative on the margin is active for its own row and for its
          // positive's rows alike (the weight itself is constant)
          float lpi;
          const float si = score_value<SK>(Rl, A.pw, &lpi, A.p);
          c = (A.margin + si - sp >= 0.f) ? A.inv_bk : 0.f;
          if (valid && lead) csum += c;
        } break;
        case KGE_LOSS_LOGISTIC: {
          const float ex = fast_exp(s - sp);
          c = ex * __builtin_amdgcn_rcpf(1.f + ex);
          if (valid && lead) csum += c;
        } break;
        case KGE_LOSS_BCE:
          c = fast_sigmoid(s) * A.inv_b;
          break;
        case KGE_LOSS_SANS: {
          const float z = valid ? A.temperature * s : -INFINITY;
          const float Mn = fmaxf(Mrun, lane_reduce<5, true>(z));
          if (Mn > Mrun) {   // wave-uniform: rescale everything accumulated so far
            const float sc = (Mrun == -INFINITY) ? 0.f : fast_exp(Mrun - Mn);
            const float sc2 = sc * sc;
#pragma unroll
            for (int q = 0; q < VEC * NC; ++q) { accH.v[q] *= sc; accR.v[q] *= sc; accT.v[q] *= sc; }
#pragma unroll
            for (int v = 0; v < 4; ++v) nrm[v] *= sc2;
            Zs *= sc;
            Mrun = Mn;
          }
          const float e = valid ? fast_exp(z - Mrun) : 0.f;
          c = e * fast_sigmoid(s + A.margin) * A.inv_b;
          if (valid && lead) Zs += e;
        } break;
        default:  // SQERR
          c = s * A.inv_b;
          break;
      }
      const float al = valid ? score_alpha_fast<SK>(c, Rl, lp, tl, A.pw, A.p) : 0.f;
      if (valid && lead) {
        gR[j] = Rl;
        gT[j] = tl;
        if (M::NRM_FROM_R) {   // ||alpha a||^2 = alpha^2 R: h- and t-lookup slices, r-lookup slice
          const float n2 = al * al * Rl;
          nrm[0] += 2.f * n2;
          nrm[1] += n2;
        }
      }
      // backward: rows past the range carry alpha = 0
      static_for<ROWS>([&](auto uc) {
        constexpr int u = decltype(uc)::value;
        const float alu = bcast(al, u << SH);
        const float Mu = SK == SK_PINF ? bcast(Rl, u << SH) : SK == SK_PGEN ? A.p : 0.f;
        M::template bwdk<kind_at<S2>(u)>(ctx, E[u], a[u], b[u], alu, Mu, accH, accR, accT, nrm, mp);
      });
      if constexpr (KGE_FILE_EARLY == 1 && !OWN) {
        if (early && j0 == sb) commit_early();
      }
    }
    };
    auto stream_lk = [&](auto sidec, const int sb, const int se) {
      if (A.loss_kind == KGE_LOSS_SANS) stream(sidec, std::integral_constant<int, KGE_LOSS_SANS>{}, sb, se);
      else stream(sidec, std::integral_constant<int, -1>{}, sb, se);
    };
    if constexpr (OWN) {
      stream_lk(std::integral_constant<int, SIDE == KGE_SIDE_HT ? KGE_SIDE_H : SIDE>{}, hb, he);
      if constexpr (SIDE == KGE_SIDE_HT) stream_lk(std::integral_constant<int, KGE_SIDE_T>{}, tb, te);
      if constexpr (KGE_FILE_EARLY == 2) {
        // the owned slots' claims (lane l: slot hb + l, slot tb + l), stored
        // by the finalise pass after the merge
        const uint32_t kb = __builtin_bit_cast(uint32_t, s_mrg[grp * MG_STRIDE + MG_KB]);
        early_own = A.train && he - hb <= KGE_WAVE && te - tb <= KGE_WAVE;
        if (early_own) {
          __builtin_amdgcn_sched_barrier(0);
#pragma unroll
          for (int r = 0; r < 2; ++r) {
            const int c = (r ? tb : hb) + lane;
            if (c < (r ? te : he) && kb + (uint32_t)c < A.own_cap) kco[r] = bin_claim(A, ids[c]);
          }
          __builtin_amdgcn_sched_barrier(0);
        }
      }
    } else {
      stream_lk(std::integral_constant<int, SIDE>{}, jbeg, jend);
      if constexpr (LATE) {
        if (!ctx_done) pos_score();   // (a wave with no slots)
      }
      if constexpr (KGE_FILE_EARLY == 2) {
        if (early) claim_early();
      }
    }
    M::finish(accH, accR, accT);
  }
  KGE_PROF(1);

  // ---- wave state -> LDS
  {
    const float Zw = wave_sum(Zs), cw = wave_sum(csum);
    float nw[4];
#pragma unroll
    for (int v = 0; v < 4; ++v) nw[v] = wave_sum(nrm[v]);
    if (lane == 0) {
      float* st = s_st + wv * 8;
      st[0] = Mrun; st[1] = Zw; st[2] = 0.f; st[3] = cw;
      st[4] = nw[0]; st[5] = nw[1]; st[6] = nw[2]; st[7] = nw[3];
    }
    if (A.train) {
      float* my = red + wv * 3 * FL;
#pragma unroll
      for (int q = 0; q < VEC * NC; ++q) {
        const int c = q / VEC, k = q % VEC;
        const int e = (c * KGE_WAVE + lane) * VEC + k;
        my[e] = accH.v[q];
        my[FL + e] = accR.v[q];
        my[2 * FL + e] = accT.v[q];
      }
    }
  }
  // the positive's own gradient at unit alpha (wave 0 of each positive)
  if constexpr (OWN) {
    // the owner keeps only the context rows its update pass re-derives the
    // negatives' gradients from, and the positive's score (hinge / logistic)
    if (active && gw == 0) {
      if (A.train) M::write_snap(ctx, A.snap + i * (M::NSNAP * (int64_t)A.snap_cols), A.snap_cols);
      if (lane == 0) s_mrg[grp * MG_STRIDE + MG_SP] = sp;
    }
  } else if (active && gw == 0) {
    float* mg = s_mrg + grp * MG_STRIDE;
    float pn[4] = {0.f, 0.f, 0.f, 0.f};
    if (A.train) {
      F pH, pR, pT, a, b, E0;
      pH.zero(); pR.zero(); pT.zero(); E0.zero();
      M::fwd(ctx, KIND_POS, E0, a, b);
      M::bwd(ctx, KIND_POS, E0, a, b, 1.f, SK == SK_PGEN ? A.p : Rp, pH, pR, pT, pn, mp);
      float* pg = posg + grp * 3 * FL;
#pragma unroll
      for (int q = 0; q < VEC * NC; ++q) {
        const int c = q / VEC, k = q % VEC;
        const int e = (c * KGE_WAVE + lane) * VEC + k;
        pg[e] = pH.v[q];
        pg[FL + e] = pR.v[q];
        pg[2 * FL + e] = pT.v[q];
      }
      M::write_snap(ctx, A.snap + i * (M::NSNAP * (int64_t)A.snap_cols), A.snap_cols);
    }
#pragma unroll
    for (int v = 0; v < 4; ++v) pn[v] = wave_sum(pn[v]);
    float rsq = 0.f;
    if (A.rel_reg != 0.f) {   // DistMult: lambda * mean_i ||r_i||^2 (DistMult.py:164-165)
      F Rr;
      load_row(Rr, A.rel.row(pr), A.rel.cols);
      rsq = wave_sum(sq_partial(Rr));
    }
    if (lane == 0) {
#pragma unroll
      for (int v = 0; v < 4; ++v) mg[MG_UN + v] = pn[v];
      mg[MG_RP] = Rp; mg[MG_TP] = tp; mg[MG_SP] = sp; mg[MG_LPP] = lpp; mg[MG_RSQ] = rsq;
    }
  }
  __syncthreads();
  KGE_PROF(2);
  if constexpr (KGE_FILE_EARLY == 2 && !OWN) {
    if (active && early) commit_early();
  }

  // ---- merge the positive's waves (one thread per positive)
  if constexpr (OWN) {
    // the owner's record header: its waves merged at its own reference
    // maximum (no 1/Z: the positive's rank normalises over every owner)
    if (tid < nValid) {
      const int p = tid;
      float* mg = s_mrg + p * MG_STRIDE;
      const float* st = s_st + p * wpp * 8;
      const bool sans = A.loss_kind == KGE_LOSS_SANS;
      float Ms = -INFINITY;
      for (int g = 0; g < wpp; ++g) Ms = fmaxf(Ms, st[g * 8]);
      float Z = 0.f, cw = 0.f, n[4] = {0.f, 0.f, 0.f, 0.f};
      for (int g = 0; g < wpp; ++g) {
        const float sc = !sans ? 1.f : (st[g * 8] == -INFINITY ? 0.f : expf(st[g * 8] - Ms));
        mg[MG_F + g] = sc;
        Z += st[g * 8 + 1] * sc;
        cw += st[g * 8 + 3];
#pragma unroll
        for (int v = 0; v < 4; ++v) n[v] += sc * sc * st[g * 8 + 4 + v];
      }
      mg[MG_MS] = Ms;
      mg[MG_IZ] = 1.f;
      float* rec = A.own_rec + (i0 + p) * (int64_t)A.rec_cols;
      rec[0] = Ms;
      rec[1] = Z;
      rec[3] = cw;
#pragma unroll
      for (int v = 0; v < 4; ++v) rec[4 + v] = n[v];
    }
  } else if (tid < nValid) {
    const int p = tid;
    float* mg = s_mrg + p * MG_STRIDE;
    const float* st = s_st + p * wpp * 8;
    const bool sans = A.loss_kind == KGE_LOSS_SANS;
    float Ms = -INFINITY;
    for (int g = 0; g < wpp; ++g) Ms = fmaxf(Ms, st[g * 8]);
    float f[kMaxWpp];
    float Z = 0.f, cw = 0.f;
    for (int g = 0; g < wpp; ++g) {
      const float sc = !sans ? 1.f : (st[g * 8] == -INFINITY ? 0.f : expf(st[g * 8] - Ms));
      f[g] = sc;
      Z += st[g * 8 + 1] * sc;
      cw += st[g * 8 + 3];
    }
    const float invZ = sans ? (Z > 0.f ? 1.f / Z : 0.f) : 1.f;
    // the positive's own loss terms; the negatives' sums come from the finalise pass
    const float lw = 0.f;
    const float Rpv = mg[MG_RP], tpv = mg[MG_TP], spv = mg[MG_SP], lppv = mg[MG_LPP];
    float lossp, cp;
    switch (A.loss_kind) {
      case KGE_LOSS_HINGE:
        lossp = lw * A.inv_bk;
        cp = -cw;
        if (Keff == 0) lossp = NAN;   // sum([]) / 0 (loss.py:81-82)
        break;
      case KGE_LOSS_LOGISTIC: lossp = lw; cp = -cw; break;
      case KGE_LOSS_BCE:
        lossp = -(log_sigmoid(spv) + lw) * A.inv_b;
        cp = -sigmoid(-spv) * A.inv_b;
        break;
      case KGE_LOSS_SANS:
        lossp = -(log_sigmoid(spv + A.margin) + lw) * A.inv_b;
        cp = -sigmoid(-(spv + A.margin)) * A.inv_b;
        break;
      default:
        lossp = ((spv - 1.f) * (spv - 1.f) + lw) * 0.5f * A.inv_b;
        cp = (spv - 1.f) * A.inv_b;
        break;
    }
    const float ap = score_alpha<SK>(cp, Rpv, lppv, tpv, A.pw, A.p);
    float n[4];
#pragma unroll
    for (int v = 0; v < 4; ++v) n[v] = ap * ap * mg[MG_UN + v];
    for (int g = 0; g < wpp; ++g) {
      const float fg = f[g] * invZ;
      mg[MG_F + g] = fg;
#pragma unroll
      for (int v = 0; v < 4; ++v) n[v] += fg * fg * st[g * 8 + 4 + v];
    }
    if (A.rel_reg != 0.f) {
      // its own IndexedSlices block: (lambda / B) * 2 r  (pow-2 gradient)
      const float gsc = A.rel_reg * A.inv_b;
      lossp += mg[MG_RSQ] * gsc;
      n[1] += 4.f * gsc * gsc * mg[MG_RSQ];
    }
    mg[MG_AP] = ap;
    mg[MG_LOSS] = lossp;
#pragma unroll
    for (int v = 0; v < 4; ++v) mg[MG_N + v] = n[v];
    mg[MG_MS] = Ms;
    mg[MG_IZ] = invZ;
    if (A.pos_score_out) A.pos_score_out[(i0 + p)] = spv;
  }
  __syncthreads();
  KGE_PROF(3);

  // ---- the positives' row gradients: sum of the waves' scaled accumulators
  if constexpr (OWN) {
    if (A.train) {   // the record's accumulator images (merged at the owner's maximum)
      constexpr int NI = rec_img<M>::n;   // 2: h and t (image v -> accumulator 2v), 3: h, r, t
      for (int e = tid; e < nValid * NI * FL; e += blockDim.x) {
        const int p = e / (NI * FL), rem = e % (NI * FL);
        const int v = rem / FL, k = rem % FL;
        const int src = NI == 2 ? 2 * v : v;
        const float* mg = s_mrg + p * MG_STRIDE;
        float sum = 0.f;
        for (int g = 0; g < wpp; ++g) sum += mg[MG_F + g] * red[((p * wpp + g) * 3 + src) * FL + k];
        A.own_rec[(i0 + p) * (int64_t)A.rec_cols + kRecHead + v * FL + k] = sum;
      }
    }
  } else if (A.train) {
    for (int e = tid; e < nValid * 3 * FL; e += blockDim.x) {
      const int p = e / (3 * FL), rem = e % (3 * FL);
      const int v = rem / FL, k = rem % FL;
      const int cols = v == 1 ? A.rel_gcols : A.ent.cols;
      if (k >= cols) continue;
      // RotatE keeps the phase gradient of complex element k in float 2k
      const int src = (v == 1 && A.rel_half) ? 2 * k : k;
      const float* mg = s_mrg + p * MG_STRIDE;
      float s = mg[MG_AP] * posg[(p * 3 + v) * FL + src];
      for (int g = 0; g < wpp; ++g) s += mg[MG_F + g] * red[((p * wpp + g) * 3 + v) * FL + src];
      if (v == 1 && A.rel_reg != 0.f) s += (A.rel_reg * A.inv_b) * (2.f * A.rel.row(s_pos[p * 3 + 1])[k]);
      A.gpos[(i0 + p) * 3 * (int64_t)A.gcols + v * (int64_t)A.gcols + k] = s;
      if constexpr (M::SELF_CTX) posg[(p * 3 + v) * FL + k] = s;   // (read just above by this thread only)
    }
  }
  if constexpr (M::SELF_CTX) {
    if (A.train) {
      // the positive's own entity-row gradients g_h = R A, g_t = R^T B
      // (A = row 0, B = row 2 of its gradient sums), the same split of R's
      // rows over its waves; written where the update kernel reads them (gpe)
      __syncthreads();
      const int d = A.ent.cols;
      const int rpw = ((d + wpp - 1) / wpp + 7) & ~7;
      const int rb = min(d, gw * rpw), re = min(d, rb + rpw);
      float* myred = red + wv * 3 * FL;
      for (int e = lane; e < FL; e += KGE_WAVE) myred[FL + e] = 0.f;
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      F up;
      up.zero();
      if (active) {
        F Ar, Br;
        const float* pa = posg + (grp * 3 + 0) * FL;
        const float* pb = posg + (grp * 3 + 2) * FL;
#pragma unroll
        for (int q = 0; q < VEC * NC; ++q) {
          const int e = (q / VEC * KGE_WAVE + lane) * VEC + q % VEC;
          Ar.v[q] = e < d ? pa[e] : 0.f;
          Br.v[q] = e < d ? pb[e] : 0.f;
        }
        rel_gemv_pair<VEC, NC>(A.rel.row(pr), d, rb, re, Br, Ar, up, myred + FL);
      }
#pragma unroll
      for (int q = 0; q < VEC * NC; ++q) myred[(q / VEC * KGE_WAVE + lane) * VEC + q % VEC] = up.v[q];
      __syncthreads();
      if (active && gw == 0) {
        F gh, gt;
        gh.zero();
        gt.zero();
        for (int g = 0; g < wpp; ++g) {
          const float* gr = red + (grp * wpp + g) * 3 * FL;
#pragma unroll
          for (int q = 0; q < VEC * NC; ++q) {
            const int e = (q / VEC * KGE_WAVE + lane) * VEC + q % VEC;
            gt.v[q] += gr[e];
            gh.v[q] += gr[FL + e];
          }
        }
        float* go = A.gpe + i * (int64_t)A.gpe_stride;
        store_row(gh, go, d);
        store_row(gt, go + A.gpe_toff, d);
      }
    }
  }

  // ---- each wave finalises its slots: loss terms, coefficient, score,
  // destination key (one lane per slot, IEEE transcendentals)
  float lfin = 0.f;
  if constexpr (OWN) {
    // the owner's loss partial (SANS: at its own maximum, no 1/Z), each owned
    // slot's (R, ties) for the coefficient pass and its destination key in
    // the workgroup's block of key positions
    if (active) {
      const float* mg = s_mrg + grp * MG_STRIDE;
      const float Ms = mg[MG_MS], spv = mg[MG_SP];
      const uint32_t kb = __builtin_bit_cast(uint32_t, mg[MG_KB]);
      auto fin = [&](int cb, int ce, int rng) {
        for (int c = cb + lane; c < ce; c += KGE_WAVE) {
          const float R = gR[c];
          float lp;
          const float s = score_value<SK>(R, A.pw, &lp, A.p);
          switch (A.loss_kind) {
            case KGE_LOSS_HINGE: lfin += fmaxf(A.margin + s - spv, 0.f); break;
            case KGE_LOSS_LOGISTIC: lfin += logf(1.f + expf(s - spv)); break;
            case KGE_LOSS_BCE: lfin += log_sigmoid(-s); break;
            case KGE_LOSS_SANS: lfin += expf(A.temperature * s - Ms) * log_sigmoid(-s - A.margin); break;
            default: lfin += s * s; break;
          }
          if (A.train) {
            const uint32_t code = ((uint32_t)i << A.kshift) | (uint32_t)jmap[c];
            A.coef[code] = make_float2(R, gT[c]);
            const uint32_t kpos = kb + (uint32_t)c;
            if (kpos < A.own_cap) {
              A.own_codes[kpos] = code;
              if (early_own) bin_commit(A, ids[c], code, kco[rng], kpos);   // (one slot per lane and range)
              else bin_key(A, ids[c], code, kpos);
            } else if (A.own_err) {
              *A.own_err = 2.f;   // (2: told apart from the exchange plan's block overflow, 1)
            }
          }
        }
      };
      fin(hb, he, 0);
      fin(tb, te, 1);
    }
  } else if (active) {
    const float* mg = s_mrg + grp * MG_STRIDE;
    const float Ms = mg[MG_MS], invZ = mg[MG_IZ], spv = mg[MG_SP];
    for (int j = jbeg + lane; j < jend; j += KGE_WAVE) {
      const float R = gR[j];
      float lp;
      const float s = score_value<SK>(R, A.pw, &lp, A.p);
      const int64_t q = i * Keff + j;
      switch (A.loss_kind) {
        case KGE_LOSS_HINGE: lfin += fmaxf(A.margin + s - spv, 0.f); break;
        case KGE_LOSS_LOGISTIC: lfin += logf(1.f + expf(s - spv)); break;
        case KGE_LOSS_BCE: lfin += log_sigmoid(-s); break;
        case KGE_LOSS_SANS: lfin += expf(A.temperature * s - Ms) * invZ * log_sigmoid(-s - A.margin); break;
        default: lfin += s * s; break;
      }
      if (A.neg_score_out) A.neg_score_out[q] = s;
      if (A.train) {
        const float c = neg_coef(A, s, spv, Ms, invZ);
        // .y: what the update kernel's gradient needs besides alpha (p = inf: the
        // row maximum; general p: p itself)
        A.coef[((uint32_t)i << A.kshift) | (uint32_t)j] =
            make_float2(score_alpha<SK>(c, R, lp, gT[j], A.pw, A.p), SK == SK_PGEN ? A.p : R);
        if (!early) bin_key(A, ids[j], ((uint32_t)i << A.kshift) | (uint32_t)j);
      }
    }
  }
  lfin = wave_sum(lfin);
  if (lane == 0) s_st[wv * 8 + 2] = lfin;   // (merge state already consumed)
  if constexpr (OWN) {
    if (err) set_status(A.status, err);
    __syncthreads();
    if (tid < nValid) {
      float l = 0.f;
      for (int g = 0; g < wpp; ++g) l += s_st[(tid * wpp + g) * 8 + 2];
      A.own_rec[(i0 + tid) * (int64_t)A.rec_cols + 2] = l;
    }
    if (tid == 0) {
      __builtin_amdgcn_s_waitcnt(0);
      const uint32_t prev = __hip_atomic_fetch_add(&A.ctl->score_ticket, 1u, __ATOMIC_RELAXED,
                                                    __HIP_MEMORY_SCOPE_AGENT);
      if (prev == (uint32_t)(gridDim.x - 1)) {   // every workgroup's keys are filed
        A.ctl->score_ticket = 0u;
        A.ctl->ovf_len = __hip_atomic_exchange(&A.ctl->ovf_count, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        A.ctl->own_len = __hip_atomic_exchange(&A.ctl->own_count, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        A.ctl->score_pending = A.sig;   // (the owner pass is always a PHASE_SCORE call)
      }
    }
    return;
  }
  if (A.train && tid < nValid * 3 && (A.rel_dests || tid % 3 != 2)) {
    const int p = tid / 3, c = tid % 3;
    const int64_t dest = c == 0 ? s_pos[p * 3] : c == 1 ? s_pos[p * 3 + 2] : A.ent.rows + s_pos[p * 3 + 1];
    bin_key(A, dest, A.nkeyneg + (((uint32_t)(i0 + p)) << 2) + (uint32_t)c);
  }
  if (err) set_status(A.status, err);
  KGE_PROF(4);
  __syncthreads();

  // ---- workgroup partials; the last workgroup to finish reduces them in a
  // fixed order and publishes the clip scales and the loss
  if (tid == 0) {
    float wl;   // weight of a wave's summed negative loss terms (loss.py)
    switch (A.loss_kind) {
      case KGE_LOSS_HINGE: wl = A.inv_bk; break;
      case KGE_LOSS_LOGISTIC: wl = 1.f; break;
      case KGE_LOSS_SANS: case KGE_LOSS_BCE: wl = -A.inv_b; break;
      default: wl = 0.5f * A.inv_b; break;
    }
    float acc[5] = {0.f, 0.f, 0.f, 0.f, 0.f};
    for (int p = 0; p < nValid; ++p) {
      const float* mg = s_mrg + p * MG_STRIDE;
      float lneg = 0.f;
      for (int g = 0; g < wpp; ++g) lneg += s_st[(p * wpp + g) * 8 + 2];
      acc[0] += mg[MG_LOSS] + wl * lneg;
#pragma unroll
      for (int v = 0; v < 4; ++v) acc[1 + v] += mg[MG_N + v];
    }
    // publish: write-through (agent-scope) stores, drained before the ticket
    // add -- no L2 write-back fence (MI355X: one per workgroup is costly)
#pragma unroll
    for (int k = 0; k < 5; ++k)
      __hip_atomic_store(&A.part[(int64_t)blockIdx.x * 8 + k], acc[k], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __builtin_amdgcn_s_waitcnt(0);   // vmcnt / lgkmcnt / expcnt drained
    const uint32_t prev = __hip_atomic_fetch_add(&A.ctl->score_ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    s_last = prev == (uint32_t)(gridDim.x - 1);
  }
  __syncthreads();
  if (s_last) {
    float acc[5] = {0.f, 0.f, 0.f, 0.f, 0.f};
    for (int w = tid; w < (int)gridDim.x; w += blockDim.x) {
#pragma unroll
      for (int k = 0; k < 5; ++k)
        acc[k] += __hip_atomic_load(&A.part[(int64_t)w * 8 + k], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
#pragma unroll
    for (int k = 0; k < 5; ++k) acc[k] = wave_sum(acc[k]);
    if (lane == 0) {
#pragma unroll
      for (int k = 0; k < 5; ++k) s_misc[wv * 8 + k] = acc[k];
    }
    __syncthreads();
    if (tid < 5) {
      float s = 0.f;
      for (int w = 0; w < W; ++w) s += s_misc[w * 8 + tid];
      if (tid == 0) {
        A.loss_out[0] = s;
        if (A.loss_accum) A.loss_accum[0] += s;
        A.ctl->loss = s;
        A.ctl->score_ticket = 0u;
        // every workgroup's keys are filed: hand the overflow length to the
        // update kernel and restart the overflow list for the next step
        A.ctl->ovf_len = __hip_atomic_exchange(&A.ctl->ovf_count, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        // the phase gate's token (kge_abi.hip): set by a PHASE_SCORE pass,
        // cleared by any other score pass of the plan (a full step consumes
        // the lists a pending update pass would have read)
        __hip_atomic_store(&A.ctl->score_pending, A.mark_pending ? A.sig : 0u, __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
      } else {
        A.ctl->scale[tid - 1] = -A.lr * (A.clip_norm / fmaxf(sqrtf(s), A.clip_norm));
        if (A.norm2_out) A.norm2_out[tid - 1] = s;
      }
    }
  }
  KGE_PROF(5);
}

// ------------------------------------------------------------ KU update
// Destination-major: one wave per destination row (entities [0, E), then
// relations [E, E + R)). The wave reads its list of codes (filed in arrival
// order by the score kernel) and visits them in ascending code order -- so
// every row is summed in the same order on every run (bit-reproducible, no
// float atomics). It re-derives each negative's row gradient from ONE
// frozen context row + its coefficient, adds the positives' own row
// gradients, and applies clip_by_norm(5) per variable (BaseModel.py:327;
// TF-2.5 IndexedSlices: norm over un-deduplicated slices, reduced by the
// score kernel) and the SGD update (BaseModel.py:328, keras SGD
// ResourceScatterAdd) with ONE read-modify-write per touched row. The
// destination's counter is cleared for the next step as it is read.
// UW: amdgpu_waves_per_eu. The compact launch (one short wave per key over a
// table far larger than L2) runs an 8-waves-per-SIMD instance: its latency
// chain wants occupancy more than it minds 16 spilled registers in the
// long-list paths (C2-50M KU 189 -> 172 us); the full launch keeps the
// allocator's choice (71 registers, 7 waves), 2 % faster at C2.
template <template <int, int, int> class Model, int VEC, int NC, int SK, int UW = 1, bool CMP = false>
__global__ __launch_bounds__(kUpdThreads) __attribute__((amdgpu_waves_per_eu(UW)))
void update_kernel(StepArgs A) {
  using M = Model<VEC, NC, SK>;
  using F = Frag<VEC, NC>;
  // entries in flight per wave; the compact instance (8 waves / SIMD: 64
  // VGPRs) takes 4 -- 8 spilled 28 bytes per lane (C2-50M KU 170 -> 160 us).
  // Rows of two or more fragment chunks (RotatE d = 256, TransE d = 512) keep
  // two: four made C3's KU 79 -> 100.5 us (register-bound occupancy,
  // profiles/r06z), eight 138 us
  constexpr int UU = UW >= 8 ? KGE_UPD_COMPACT_U : KGE_UPDATE_U;
  constexpr int U = NC >= 2 ? 2 : (UU > 1 ? UU : 2);
  constexpr int RV = RelV<M::CPLX, VEC>::n;
  constexpr int CHMAX = 4;                            // in-register ordering up to 256 codes
  __shared__ uint32_t s_scr[kUpdWaves][CHMAX * KGE_WAVE];
  __shared__ uint32_t s_sort[kUpdWaves][kSortMax];    // longer lists: gathered + bitonic-sorted here

  KGE_PROF_INIT();
  const int lane = lane_id(), wv = wave_id();
  const int64_t E_ = A.ent.rows;
  // relation rows first: few rows with the longest lists (every positive
  // files one), so they start early instead of forming the kernel's tail
  const int64_t R_ = A.rel_dests ? A.rel.rows : 0;
  const int64_t ndest = E_ + R_;
  const int64_t dd = (int64_t)blockIdx.x * kUpdWaves + wv;
  // workspace guard (ws_refused): the step's first kernel claimed the
  // workspace for this plan or refused it (and reported); here a refused
  // workspace just leaves every wave idle -- one scalar compare, no branch
  // of its own (an early return cost the compact instance registers)
  const bool ws_ok = !KGE_GUARD_KU || *reinterpret_cast<const uint32_t*>(&A.ctl->plan_sig) == A.sig;
  // split step, a rank's exchange failed: no table, gradient or relation
  // write at all, but every destination's counter / hash slot still goes
  // back to zero -- the workspace is ready for the next step's score pass
  const bool abort_ = A.abort_flag && *A.abort_flag != 0.f;
  const uint32_t nneg = A.nkeyneg;
  const uint32_t kmask = (1u << A.kshift) - 1u;
  const uint32_t snap_stride = (uint32_t)(M::NSNAP * A.snap_cols);   // B * stride < 2^32 (plan check)
  float sc_ent = A.ctl->scale[A.sc_ent_idx], sc_rel = A.ctl->scale[A.sc_rel_idx];   // issued up front
  if (A.scale_from_norm2) {   // split step: the caller's (all-reduced) norms
    sc_ent = -A.lr * (A.clip_norm / fmaxf(sqrtf(A.norm2_out[A.sc_ent_idx]), A.clip_norm));
    sc_rel = -A.lr * (A.clip_norm / fmaxf(sqrtf(A.norm2_out[A.sc_rel_idx]), A.clip_norm));
  }

  // one code -> its positive i and slot j (negative, c = -1) or row part c (0 h, 1 t, 2 r)
  auto decode = [&](uint32_t code, int64_t* i, int* j, int* c) {
    if (code < nneg) {
      *i = code >> A.kshift;
      *j = (int)(code & ((1u << A.kshift) - 1u));
      *c = -1;
    } else {
      *i = (code - nneg) >> 2;
      *j = 0;
      *c = (int)((code - nneg) & 3u);
    }
  };
  // entity destination: add the gradient rows of `cntv` (<= U) entries
  float accE = 0.f;   // LINEAR_E models: summed coefficient of the destination row itself
  auto entity_add = [&](const uint32_t* codes, int cntv, const F& E, F& acc) {
    int64_t ii[U];
    int jj[U], cc[U];
    typename M::ECtx ec[U];   // a positive's own row gradient goes into ec[u].c0
    float2 cf[U];
    // compile-time entry indices (static_for): the per-entry context rows stay
    // in registers (a runtime-indexed loop too large to unroll put them in scratch)
    static_for<U>([&](auto uc) {
      constexpr int u = decltype(uc)::value;
      if (u < cntv) {
        decode(codes[u], &ii[u], &jj[u], &cc[u]);
        if (cc[u] < 0) {
          if constexpr (M::MAT) {
            load_row(ec[u].c0, A.gneg + (int64_t)codes[u] * A.ent.cols, A.ent.cols);
            cf[u] = make_float2(0.f, 0.f);
          } else {
            cf[u] = A.coef[codes[u]];
            M::load_ectx(A.snap + ii[u] * (M::NSNAP * (int64_t)A.snap_cols), A.snap_cols,
                         slot_kind(A.side_mode, jj[u]), ec[u]);
          }
        } else {
          load_row(ec[u].c0, A.gpe + ii[u] * (int64_t)A.gpe_stride + (cc[u] == 0 ? 0 : A.gpe_toff), A.ent.cols);
        }
      }
    });
    static_for<U>([&](auto uc) {
      constexpr int u = decltype(uc)::value;
      if (u < cntv) {
        if (cc[u] < 0) {
          if constexpr (M::LINEAR_E) {
            // g = alpha_E * E + alpha_C * c0: wave-uniform scalars, one FMA per element
            float aE, aC;
            M::lin_coefs(slot_kind(A.side_mode, jj[u]), cf[u].x, aE, aC);
            accE += aE;
#pragma unroll
            for (int q = 0; q < VEC * NC; ++q) acc.v[q] += aC * ec[u].c0.v[q];
          } else {
            F g;
            M::grad_entity(ec[u], slot_kind(A.side_mode, jj[u]), E, cf[u].x, cf[u].y, g);
            add_to(acc, g);
          }
        } else {
          add_to(acc, ec[u].c0);
        }
      }
    });
  };
  auto rel_add = [&](const uint32_t* codes, int cntv, float (&acc)[RV * NC]) {
    float g[U][RV * NC];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if (u < cntv) {
        int64_t ii;
        int jj, cc;
        decode(codes[u], &ii, &jj, &cc);
        load_rel_row<M::CPLX, VEC, NC>(g[u], A.gpos + ii * 3 * (int64_t)A.gcols + A.gcols, A.rel_gcols);
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u)
      if (u < cntv) {
#pragma unroll
        for (int q = 0; q < RV * NC; ++q) acc[q] += g[u][q];
      }
  };

  float dn2 = 0.f;   // dense mode: this wave's ||summed row gradient||^2
  float en2 = 0.f;   // dense mode: this wave's ||entity row||^2 (the regulariser loss, RESCAL.py:190-198)
  // one destination row d (list index li; compact: code1 = its first filed code)
  auto run_dest = [&](const int64_t d, const int64_t li, const uint32_t code1, const bool active) {
  accE = 0.f;
  if (active) {
    const bool is_ent = d < E_;
    const uint32_t* lst = A.list + li * (int64_t)A.cap;
    // issued together: the counter, the list's first 64 entries (speculative;
    // lanes past the count are ignored) and the entity row
    const uint32_t n = CMP ? (uint32_t)A.htab[li] : A.cnt[d];
    if constexpr (CMP) {
      // merge update, a long list: long_rows_kernel takes it (all threads of a
      // workgroup, kLongU rows in flight) if there is room in lng[]
      if (A.pos_only && is_ent && n > (uint32_t)kLongN && n <= (uint32_t)kLongMax) {
        uint32_t slot = 0u;
        if (lane == 0) slot = atomicAdd(&A.ctl->lng_count, 1u);
        slot = (uint32_t)__builtin_amdgcn_readfirstlane((int)slot);
        if (slot < A.lng_cap) {
          if (lane == 0) A.lng[slot] = make_uint4((uint32_t)d, (uint32_t)((uint64_t)d >> 32), (uint32_t)li, code1);
          return;
        }
      }
    }
    // list entry q (compact launches: position 0 is the leader's code1, and
    // the list is read only once the count says there is more than one key)
    const bool l0 = KGE_COMPACT_LIST0 && CMP;
    auto lst_at = [&](uint32_t q) -> uint32_t { return (l0 && q == 0u) ? code1 : lst[q]; };
    uint32_t code0 = 0xFFFFFFFFu;
    if (!CMP) code0 = lst[min(lane, A.cap - 1)];   // speculative: issued with the counter
    F E, acc;
    acc.zero();
    E.zero();
    // compact launches over large tables: most destinations hold exactly one
    // key, whose code came with the destination -- its coefficient and context
    // row are requested together with the counter (used when n == 1)
    const bool pre = CMP && is_ent && code1 < nneg;
    typename M::ECtx ec1;
    float2 cf1 = make_float2(0.f, 0.f);
    int kd1 = 0;
    if (pre) {
      kd1 = slot_kind(A.side_mode, (int)(code1 & kmask));
      if constexpr (M::MAT) {
        load_row(ec1.c0, A.gneg + (int64_t)code1 * A.ent.cols, A.ent.cols);
      } else {
        cf1 = A.coef[code1];
        M::load_ectx(A.snap + (code1 >> A.kshift) * snap_stride, A.snap_cols, kd1, ec1);
      }
    }
    // an untouched row is read only when the step rewrites it anyway (fused
    // constraint) or it carries a dense term; a compact launch visits only
    // touched rows (issued without waiting for the counter)
    if (is_ent && (CMP || n != 0u || A.fuse_norm || A.dense)) {
      load_row(E, A.ent.row(d), A.ent.cols);
      if (A.fuse_norm) {
        normalize_row(E);   // the step's constraint assign, then this step's update
        // (grad mode: every row goes back normalised; the caller's apply follows)
        if (n == 0u || A.grad_mode) store_row(E, A.ent.row_w(d), A.ent.cols);
      }
    }
    if (n != 0u || (A.dense && is_ent)) {
      if (lane == 0 && n != 0u && !A.keep_cnt) {   // ready for the next step
        if (CMP) A.htab[li] = 0ull;
        else A.cnt[d] = 0u;
      }
      float racc[RV * NC];
#pragma unroll
      for (int q = 0; q < RV * NC; ++q) racc[q] = 0.f;
      auto consume_sorted = [&](auto code_at) {
        int p0 = 0;
        if constexpr (M::LINEAR_E) {
          if (is_ent) {
            // the negatives come first in code order: U-wide batches with no
            // per-entry branches (padding entries repeat a code with weight 0)
            int nn = 0;   // negatives among the n codes (binary search on the sorted codes)
            {
              int lo = 0, hi = (int)n;
              while (lo < hi) {
                const int mid = (lo + hi) >> 1;
                if (code_at(mid) < nneg) lo = mid + 1; else hi = mid;
              }
              nn = lo;
            }
            for (; p0 < nn; p0 += U) {
              typename M::ECtx ec[U];
              float2 cf[U];
              int kd[U];
              static_for<U>([&](auto uc) {
                constexpr int u = decltype(uc)::value;
                const uint32_t code = code_at(min(p0 + u, nn - 1));
                const uint32_t i = code >> A.kshift;
                kd[u] = slot_kind(A.side_mode, (int)(code & kmask));
                cf[u] = A.coef[code];
                M::load_ectx(A.snap + i * snap_stride, A.snap_cols, kd[u], ec[u]);
              });
              static_for<U>([&](auto uc) {
                constexpr int u = decltype(uc)::value;
                float aE, aC;
                M::lin_coefs(kd[u], p0 + u < nn ? cf[u].x : 0.f, aE, aC);
                accE += aE;
#pragma unroll
                for (int q = 0; q < VEC * NC; ++q) acc.v[q] += aC * ec[u].c0.v[q];
              });
            }
            p0 = nn;
          }
        }
        for (; p0 < (int)n; p0 += U) {
          uint32_t cs[U];
#pragma unroll
          for (int u = 0; u < U; ++u) cs[u] = code_at(min(p0 + u, (int)n - 1));
          if (is_ent) entity_add(cs, min(U, (int)n - p0), E, acc);
          else rel_add(cs, min(U, (int)n - p0), racc);
        }
      };
      if (n == 0u) {
        // dense mode, untouched row: the regulariser term only
      } else if (pre && n == 1u) {
        // the single (negative) key, context already in registers
        if constexpr (M::LINEAR_E) {
          float aE, aC;
          M::lin_coefs(kd1, cf1.x, aE, aC);
          accE += aE;
#pragma unroll
          for (int q = 0; q < VEC * NC; ++q) acc.v[q] += aC * ec1.c0.v[q];
        } else {
          F g;
          M::grad_entity(ec1, kd1, E, cf1.x, cf1.y, g);
          add_to(acc, g);
        }
      } else if (n <= (uint32_t)A.cap && n <= (uint32_t)KGE_WAVE) {
        // ascending code order: each code's rank among the n (codes are
        // unique), then a forward permute puts code of rank r in lane r
        if (CMP) code0 = lane < (int)n ? lst_at((uint32_t)lane) : 0xFFFFFFFFu;
        const uint32_t code = lane < (int)n ? code0 : 0xFFFFFFFFu;
        uint32_t rank = 0u;
        for (int q = 0; q < (int)n; ++q) rank += ((uint32_t)__builtin_amdgcn_readlane((int)code, q) < code) ? 1u : 0u;
        const int sorted = __builtin_amdgcn_ds_permute((int)(min(rank, 63u) << 2), (int)code);
        consume_sorted([&](int p) { return (uint32_t)__builtin_amdgcn_readlane(sorted, p); });
      } else if (n <= (uint32_t)A.cap && n <= (uint32_t)(CHMAX * KGE_WAVE)) {
        const int nch = (int)((n + KGE_WAVE - 1) / KGE_WAVE);
        uint32_t code[CHMAX];
#pragma unroll
        for (int c = 0; c < CHMAX; ++c) {
          const uint32_t q = (uint32_t)(c * KGE_WAVE + lane);
          code[c] = (c < nch && q < n) ? lst_at(q) : 0xFFFFFFFFu;
        }
        uint32_t rank[CHMAX] = {0u, 0u, 0u, 0u};
#pragma unroll
        for (int c2 = 0; c2 < CHMAX; ++c2) {
          if (c2 < nch) {
            const int lim = min(KGE_WAVE, (int)n - c2 * KGE_WAVE);
            for (int q = 0; q < lim; ++q) {
              const uint32_t o = (uint32_t)__builtin_amdgcn_readlane((int)code[c2], q);
#pragma unroll
              for (int c = 0; c < CHMAX; ++c) rank[c] += (o < code[c]) ? 1u : 0u;
            }
          }
        }
        uint32_t* scr = s_scr[wv];
#pragma unroll
        for (int c = 0; c < CHMAX; ++c)
          if (c < nch && (uint32_t)(c * KGE_WAVE + lane) < n) scr[rank[c]] = code[c];
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        consume_sorted([&](int p) { return (uint32_t)__builtin_amdgcn_readfirstlane((int)scr[p]); });
      } else if (n <= (uint32_t)kSortMax) {
        // a long list (past its capacity or past 256 codes; skewed graphs):
        // the list part and this destination's overflow entries (one pass
        // over the overflow array, ballot-compacted) gathered into LDS, then
        // a wave-local bitonic sort -- linear gather, n log^2 n compares
        uint32_t* buf = s_sort[wv];
        const uint32_t nl = min(n, (uint32_t)A.cap);
        for (uint32_t q = lane; q < nl; q += KGE_WAVE) buf[q] = lst_at(q);
        if (n > nl) {
          const uint32_t novf = A.ctl->ovf_len;
          uint32_t fill = nl;
          for (uint32_t q0 = 0; q0 < novf && fill < n; q0 += KGE_WAVE) {
            const uint32_t q = q0 + lane;
            uint64_t y = 0;
            const bool hit = q < novf && (int64_t)((y = A.ovf[q]) >> 32) == d;
            const uint64_t m = __ballot(hit);
            if (hit) buf[fill + __popcll(m & ((1ull << lane) - 1ull))] = (uint32_t)y;
            fill += (uint32_t)__popcll(m);
          }
        }
        uint32_t P = 1;
        while (P < n) P <<= 1;
        for (uint32_t q = n + lane; q < P; q += KGE_WAVE) buf[q] = 0xFFFFFFFFu;
        auto wave_sync = [] {
          __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
          __builtin_amdgcn_wave_barrier();
          __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        };
        wave_sync();
        for (uint32_t k = 2; k <= P; k <<= 1) {
          for (uint32_t j = k >> 1; j > 0; j >>= 1) {
            for (uint32_t i = lane; i < P; i += KGE_WAVE) {
              const uint32_t l = i ^ j;
              if (l > i) {
                const uint32_t a = buf[i], b = buf[l];
                if ((a > b) == ((i & k) == 0)) { buf[i] = b; buf[l] = a; }
              }
            }
            wave_sync();
          }
        }
        consume_sorted([&](int p) { return (uint32_t)__builtin_amdgcn_readfirstlane((int)buf[p]); });
      } else {
        // past kSortMax codes: repeated selection of the next code from the
        // list and the overflow entries (correct for any skew, not fast)
        const uint32_t nl = min(n, (uint32_t)A.cap);
        const uint32_t novf = A.ctl->ovf_len;
        uint32_t last = 0u;
        for (uint32_t p = 0; p < n; ++p) {
          uint32_t best = 0xFFFFFFFFu;
          for (uint32_t q = lane; q < nl; q += KGE_WAVE) {
            const uint32_t x = lst_at(q);
            if ((p == 0u || x > last) && x < best) best = x;
          }
          for (uint32_t q = lane; q < novf; q += KGE_WAVE) {
            const uint64_t y = A.ovf[q];
            const uint32_t x = (uint32_t)y;
            if ((int64_t)(y >> 32) == d && (p == 0u || x > last) && x < best) best = x;
          }
#pragma unroll
          for (int o = 32; o >= 1; o >>= 1) best = min(best, (uint32_t)__shfl_xor((int)best, o, KGE_WAVE));
          last = best;
          uint32_t cs[U];
#pragma unroll
          for (int u = 0; u < U; ++u) cs[u] = best;
          if (is_ent) entity_add(cs, 1, E, acc);
          else rel_add(cs, 1, racc);
        }
      }
      if (is_ent) {
        if constexpr (M::LINEAR_E) {
#pragma unroll
          for (int q = 0; q < VEC * NC; ++q) acc.v[q] += accE * E.v[q];
        }
        if (A.dense) {
          en2 = sq_partial(E);
#pragma unroll
          for (int q = 0; q < VEC * NC; ++q) acc.v[q] += A.dense_ent * E.v[q];
          dn2 = sq_partial(acc);
        }
        if (A.grad_mode || A.dense) {
          store_row(acc, A.gent + d * (int64_t)A.ent.cols, A.ent.cols);
        } else if (d >= A.remote_from) {
          // a row fetched from its owner (split step): its raw summed
          // gradient replaces it, and travels back to the owner
          store_row(acc, A.ent.row_w(d), A.ent.cols);
        } else {
#pragma unroll
          for (int q = 0; q < VEC * NC; ++q) E.v[q] = E.v[q] + acc.v[q] * sc_ent;
          store_row(E, A.ent.row_w(d), A.ent.cols);
        }
      } else {
        const int64_t r = d - E_;
        if (A.grad_mode || A.rel_grad) {
          store_rel_row<M::CPLX, VEC, NC>(racc, A.grel + r * (int64_t)A.rel_gcols, A.rel.cols);
        } else {
          float row[RV * NC];
          load_rel_row<M::CPLX, VEC, NC>(row, A.rel.row(r), A.rel.cols);
#pragma unroll
          for (int q = 0; q < RV * NC; ++q) row[q] = row[q] + racc[q] * sc_rel;
          store_rel_row<M::CPLX, VEC, NC>(row, A.rel.row_w(r), A.rel.cols);
        }
      }
    } else if (A.zero_untouched) {
      if (is_ent) {
        store_row(acc, A.gent + d * (int64_t)A.ent.cols, A.ent.cols);
      } else {
        float z[RV * NC];
#pragma unroll
        for (int q = 0; q < RV * NC; ++q) z[q] = 0.f;
        store_rel_row<M::CPLX, VEC, NC>(z, A.grel + (d - E_) * (int64_t)A.rel_gcols, A.rel.cols);
      }
    }
  }
  };

  if constexpr (CMP) {
    // KR key positions per wave: the destinations' first keys lead. Every
    // position's leader entry, then for the common case at large tables -- an
    // entity row holding exactly one (negative) key, whose code came with the
    // destination -- the counter, coefficient, context row and entity row of
    // all KR are requested together (KR times the bytes in flight of one
    // destination per wave: the launch is latency-bound). Those rows are
    // finished here with the arithmetic of run_dest's single-key case; every
    // other destination goes through run_dest. (Leaders are read
    // unconditionally: the array is padded to the grid.)
    constexpr int KR = kUpdKeysPerWave;
    const bool one_ok = !A.dense && !A.grad_mode;
    // (owner pass: the key positions its score pass took)
    const int64_t nkeys = A.own_keys ? (int64_t)min(A.nkeys, A.ctl->own_len) : (int64_t)A.nkeys;
    uint4 t[KR];
    bool act[KR], one[KR];
    uint32_t n1[KR];
    F E1[KR];
    typename M::ECtx c1[KR];
    float2 f1[KR];
    static_for<KR>([&](auto rc) {
      constexpr int r = decltype(rc)::value;
      t[r] = A.leaders[dd * KR + r];
    });
    static_for<KR>([&](auto rc) {
      constexpr int r = decltype(rc)::value;
      act[r] = ws_ok && dd * KR + r < nkeys && t[r].y != 0xFFFFFFFFu &&
               !(A.rel_only && (int64_t)t[r].x < E_);
      if (abort_ || (A.rel_seg && (int64_t)t[r].x >= E_)) {   // (the leader's slot: one per destination)
        if (act[r] && lane == 0 && !A.keep_cnt) A.htab[t[r].z] = 0ull;
        act[r] = false;
      }
      one[r] = one_ok && act[r] && (int64_t)t[r].x < E_ && t[r].y < nneg;
      n1[r] = 0u;
      f1[r] = make_float2(0.f, 0.f);
      E1[r].zero();
      if (one[r]) {
        n1[r] = (uint32_t)A.htab[t[r].z];
        if constexpr (M::MAT) {
          load_row(c1[r].c0, A.gneg + (int64_t)t[r].y * A.ent.cols, A.ent.cols);
        } else {
          f1[r] = A.coef[t[r].y];
          M::load_ectx(A.snap + (t[r].y >> A.kshift) * snap_stride, A.snap_cols,
                       slot_kind(A.side_mode, (int)(t[r].y & kmask)), c1[r]);
        }
        load_row(E1[r], A.ent.row(t[r].x), A.ent.cols);
      }
    });
    static_for<KR>([&](auto rc) {
      constexpr int r = decltype(rc)::value;
      if (one[r] && n1[r] == 1u) {
        const int64_t d = (int64_t)t[r].x;
        F E = E1[r], acc;
        acc.zero();
        if (A.fuse_norm) normalize_row(E);
        if (lane == 0 && !A.keep_cnt) A.htab[t[r].z] = 0ull;
        const int kd = slot_kind(A.side_mode, (int)(t[r].y & kmask));
        if constexpr (M::LINEAR_E) {
          float aE, aC;
          M::lin_coefs(kd, f1[r].x, aE, aC);
          const float sE = 0.f + aE;
#pragma unroll
          for (int q = 0; q < VEC * NC; ++q) acc.v[q] += aC * c1[r].c0.v[q];
#pragma unroll
          for (int q = 0; q < VEC * NC; ++q) acc.v[q] += sE * E.v[q];
        } else {
          F g;
          M::grad_entity(c1[r], kd, E, f1[r].x, f1[r].y, g);
          add_to(acc, g);
        }
        if (d >= A.remote_from) {
          store_row(acc, A.ent.row_w(d), A.ent.cols);
        } else {
#pragma unroll
          for (int q = 0; q < VEC * NC; ++q) E.v[q] = E.v[q] + acc.v[q] * sc_ent;
          store_row(E, A.ent.row_w(d), A.ent.cols);
        }
        act[r] = false;
      }
    });
#pragma unroll
    for (int r = 0; r < KR; ++r)
      if (act[r]) run_dest((int64_t)t[r].x, (int64_t)t[r].z, t[r].y, true);
  } else {
    const bool active = ws_ok && dd < (A.rel_only ? R_ : ndest);
    const int64_t d = dd < R_ ? E_ + dd : dd - R_;
    const bool skip = abort_ || (A.rel_seg && d >= E_);
    if (skip && active && lane == 0 && !A.keep_cnt) A.cnt[d] = 0u;
    run_dest(d, d, 0xFFFFFFFFu, active && !skip);
  }
  if (A.dense) {
    // ||dense gradient||^2: workgroup partial; partials_norm_kernel (the next
    // launch) sums them in a fixed order (clip_by_norm of the dense tensor) --
    // no ticket on one counter from every workgroup
    // (in the sort scratch: 20 bytes of their own would cost a workgroup of
    // occupancy -- 7 instead of 8 per CU at 20,480 bytes of LDS each)
    float* s_n2 = reinterpret_cast<float*>(&s_scr[0][0]);
    __syncthreads();   // every wave is done with its scratch
    dn2 = wave_sum(dn2);
    en2 = wave_sum(en2);
    if (lane == 0) { s_n2[wv] = dn2; s_n2[kUpdWaves + wv] = en2; }
    __syncthreads();
    if (threadIdx.x < 2) {   // [gridU] gradient norm^2 | [gridU] entity norm^2
      float w = 0.f;
      for (int k = 0; k < kUpdWaves; ++k) w += s_n2[threadIdx.x * kUpdWaves + k];
      A.upart[threadIdx.x * gridDim.x + blockIdx.x] = w;
    }
  }
  KGE_PROF(16);
}

// ------------------------------------------------------------ long lists
// (A.pos_only, the owner merge's update pass) One destination row per
// workgroup iteration: its codes -- list position 0 from the leader, the
// list, then its overflow entries -- gathered into LDS and bitonic-sorted.
// The 1024 threads are four row groups of 256: group g sums the positives'
// row gradients (gpe) of the g-th quarter of the sorted codes, kLongU rows in
// flight per thread (up to kLongCPT columns each); the four partial rows are
// added in group order (deterministic). Then the update kernel's write (raw
// gradient for a fetched row, else the clip-scaled SGD step) and the hash
// slot emptied. (One wave summing a Zipf-hot row two codes at a time was a
// 60 us chain; one 256-thread group, 41 us.)
template <int UNUSED>
__global__ __launch_bounds__(1024) void long_rows_kernel(StepArgs A) {
  __shared__ uint32_t s_codes[kLongMax];
  __shared__ float s_part[3][256 * kLongCPT];
  __shared__ uint32_t s_fill;
  if (ws_refused(A.ctl, A.sig, A.status, nullptr)) return;
  const int tid = threadIdx.x, grp = tid >> 8, t = tid & 255;
  const uint32_t nitems = min(A.ctl->lng_count, A.lng_cap);
  float sc = A.ctl->scale[A.sc_ent_idx];
  if (A.scale_from_norm2) sc = -A.lr * (A.clip_norm / fmaxf(sqrtf(A.norm2_out[A.sc_ent_idx]), A.clip_norm));
  const uint32_t nneg = A.nkeyneg;
  for (uint32_t it = blockIdx.x; it < nitems; it += gridDim.x) {
    const uint4 w = A.lng[it];
    const int64_t d = (int64_t)((uint64_t)w.x | ((uint64_t)w.y << 32));
    const int64_t li = w.z;
    const uint32_t n = (uint32_t)A.htab[li];
    const uint32_t nl = min(n, (uint32_t)A.cap);
    const uint32_t* lst = A.list + li * (int64_t)A.cap;
    for (uint32_t q = tid; q < nl; q += 1024) s_codes[q] = (KGE_COMPACT_LIST0 && q == 0u) ? w.w : lst[q];
    if (tid == 0) s_fill = nl;
    __syncthreads();
    if (n > nl) {
      const uint32_t novf = A.ctl->ovf_len;
      for (uint32_t q = tid; q < novf; q += 1024) {
        const uint64_t y = A.ovf[q];
        if ((int64_t)(y >> 32) == d) s_codes[atomicAdd(&s_fill, 1u)] = (uint32_t)y;
      }
    }
    uint32_t P = 1;
    while (P < n) P <<= 1;
    for (uint32_t q = n + tid; q < P; q += 1024) s_codes[q] = 0xFFFFFFFFu;
    __syncthreads();
    for (uint32_t k = 2; k <= P; k <<= 1) {
      for (uint32_t j = k >> 1; j > 0; j >>= 1) {
        for (uint32_t i = tid; i < P; i += 1024) {
          const uint32_t l = i ^ j;
          if (l > i) {
            const uint32_t a = s_codes[i], b = s_codes[l];
            if ((a > b) == ((i & k) == 0)) { s_codes[i] = b; s_codes[l] = a; }
          }
        }
        __syncthreads();
      }
    }
    // this group's quarter of the sorted codes
    const uint32_t q0 = (uint32_t)((uint64_t)n * grp / 4), q1 = (uint32_t)((uint64_t)n * (grp + 1) / 4);
    float acc[kLongCPT];
#pragma unroll
    for (int j = 0; j < kLongCPT; ++j) acc[j] = 0.f;
    for (uint32_t p0 = q0; p0 < q1; p0 += kLongU) {
      float x[kLongU][kLongCPT];
#pragma unroll
      for (int u = 0; u < kLongU; ++u) {
        const uint32_t code = s_codes[min(p0 + (uint32_t)u, q1 - 1u)] - nneg;   // (positive codes only)
        const float* g = A.gpe + (int64_t)(code >> 2) * A.gpe_stride + ((code & 3u) == 0u ? 0 : A.gpe_toff);
#pragma unroll
        for (int j = 0; j < kLongCPT; ++j) {
          const int c = t + 256 * j;
          x[u][j] = c < A.ent.cols ? g[c] : 0.f;
        }
      }
#pragma unroll
      for (int u = 0; u < kLongU; ++u)
        if (p0 + (uint32_t)u < q1) {
#pragma unroll
          for (int j = 0; j < kLongCPT; ++j) acc[j] += x[u][j];
        }
    }
    if (grp > 0) {
#pragma unroll
      for (int j = 0; j < kLongCPT; ++j) s_part[grp - 1][t + 256 * j] = acc[j];
    }
    __syncthreads();
    if (grp == 0) {
      float* row = A.ent.row_w(d);
#pragma unroll
      for (int j = 0; j < kLongCPT; ++j) {
        const int c = t + 256 * j;
        if (c >= A.ent.cols) continue;
        const float v = ((acc[j] + s_part[0][c]) + s_part[1][c]) + s_part[2][c];
        if (d >= A.remote_from) row[c] = v;
        else row[c] = row[c] + v * sc;
      }
      if (t == 0 && !A.keep_cnt) A.htab[li] = 0ull;
    }
    __syncthreads();   // s_codes / s_part are rewritten by the next destination
  }
}

// ------------------------------------------------------------ relation rows
// (A.rel_seg, the owner merge's update pass) launch_rel_rank puts the batch's
// positives in relation order (stable: ascending positive index within a
// relation), then one workgroup per (relation r, 256-column strip), 1024
// threads: a relation without positives returns after one load; otherwise its
// positions are staged in LDS kRsChunk at a time and the threads, four row
// groups of 256, each sum their column of one quarter of them (the positives'
// relation-row gradients, gpos), kRsU rows in flight; the partials add in
// group order (deterministic). Then the update kernel's relation write: the
// raw gradient (grad / split update modes) or the clip-scaled SGD step;
// relations with no positive get a zero gradient row (grad / relation-gradient
// modes) or are left alone (SGD). Flat rows: both fragment layouts (load_row, load_row_half) keep
// element e at float e.
constexpr int kRsThreads = 1024, kRsChunk = 4096, kRsU = 32;

template <int UNUSED>
__global__ __launch_bounds__(kRsThreads) void rel_seg_kernel(StepArgs A) {
  __shared__ int32_t s_list[kRsChunk];
  __shared__ float s_part[3][256];
  if (ws_refused(A.ctl, A.sig, A.status, nullptr)) return;
  const int tid = threadIdx.x, grp = tid >> 8, t = tid & 255;
  const int64_t r = blockIdx.x;
  const int cols = A.rel.cols;
  const int c = (int)blockIdx.y * 256 + t;
  const bool cv = c < cols;
  if (A.abort_flag && *A.abort_flag != 0.f) {
    // an aborted step: no table written, but every relation gradient row is
    // still this kernel's to write (the caller skipped the zero-fill) -- zeros,
    // never the previous step's values
    if ((A.grad_mode || A.rel_grad) && grp == 0 && cv) A.grel[r * (int64_t)A.rel_gcols + c] = 0.f;
    return;
  }
  const int64_t cnt = A.rs_beg[A.rel.rows + r];   // (rel_cnt follows rel_beg)
  if (cnt == 0) {
    // (every relation row of grel is written here: the caller skips its zero-fill)
    if ((A.grad_mode || A.rel_grad) && grp == 0 && cv) A.grel[r * (int64_t)A.rel_gcols + c] = 0.f;
    return;
  }
  const int64_t beg = A.rs_beg[r];
  const float* g = A.gpos + A.gcols + (cv ? c : 0);
  const int64_t gstride = 3 * (int64_t)A.gcols;
  float acc = 0.f;
  for (int64_t base = 0; base < cnt; base += kRsChunk) {
    const int n = (int)min<int64_t>(kRsChunk, cnt - base);
    for (int q = tid; q < n; q += kRsThreads) s_list[q] = A.rs_sorted[beg + base + q];
    __syncthreads();
    const int q0 = n * grp / 4, q1 = n * (grp + 1) / 4;
    for (int p0 = q0; p0 < q1; p0 += kRsU) {
      float x[kRsU];
#pragma unroll
      for (int u = 0; u < kRsU; ++u) x[u] = cv ? g[(int64_t)s_list[min(p0 + u, q1 - 1)] * gstride] : 0.f;
#pragma unroll
      for (int u = 0; u < kRsU; ++u)
        if (p0 + u < q1) acc += x[u];
    }
    __syncthreads();   // s_list is rewritten by the next chunk
  }
  if (grp > 0) s_part[grp - 1][t] = acc;
  __syncthreads();
  if (grp != 0 || !cv) return;
  acc = ((acc + s_part[0][t]) + s_part[1][t]) + s_part[2][t];
  if (A.grad_mode || A.rel_grad) {
    A.grel[r * (int64_t)A.rel_gcols + c] = acc;
  } else {
    float sc = A.ctl->scale[A.sc_rel_idx];
    if (A.scale_from_norm2) sc = -A.lr * (A.clip_norm / fmaxf(sqrtf(A.norm2_out[A.sc_rel_idx]), A.clip_norm));
    float* w = A.rel.row_w(r) + c;
    *w = *w + acc * sc;
  }
}

static inline void launch_rel_seg(const StepArgs& A, hipStream_t st) {
  RelArgs R{};
  R.ent = A.ent;
  R.rel = A.rel;
  R.pos = A.pos;
  R.i64 = A.i64;
  R.B = A.B;
  R.sorted = A.rs_sorted;
  R.srel = A.rs_srel;
  R.rel_beg = A.rs_beg;
  R.rel_cnt = A.rs_beg + A.rel.rows;
  R.status = A.status;
  launch_rel_rank(R, st);
  const dim3 grid((unsigned)A.rel.rows, (unsigned)((A.rel.cols + 255) / 256));
  hipLaunchKernelGGL(rel_seg_kernel<0>, grid, dim3(kRsThreads), 0, st, A);
}

// ------------------------------------------------------------ dispatch
template <template <int, int, int> class Model, int VEC, int NC, int SK>
static void launch_score(const StepArgs& A, const StepGeom& G, hipStream_t st) {
#ifdef KGE_ONLY_ONE
  hipLaunchKernelGGL((score_kernel<Model, VEC, NC, SK, KGE_SIDE_HT>), dim3(G.nWG), dim3(kStepThreads), G.lds_score,
                     st, A);
#else
  if (A.side_mode == KGE_SIDE_HT)
    hipLaunchKernelGGL((score_kernel<Model, VEC, NC, SK, KGE_SIDE_HT>), dim3(G.nWG), dim3(kStepThreads), G.lds_score,
                       st, A);
  else if (A.side_mode == KGE_SIDE_H)
    hipLaunchKernelGGL((score_kernel<Model, VEC, NC, SK, KGE_SIDE_H>), dim3(G.nWG), dim3(kStepThreads), G.lds_score,
                       st, A);
  else
    hipLaunchKernelGGL((score_kernel<Model, VEC, NC, SK, KGE_SIDE_T>), dim3(G.nWG), dim3(kStepThreads), G.lds_score,
                       st, A);
#endif
}

template <template <int, int, int> class Model, int VEC, int NC, int SK>
static kge_status launch_family(const StepArgs& A, const StepGeom& G, hipStream_t st, hipEvent_t const* ev) {
  if (A.run_score) launch_score<Model, VEC, NC, SK>(A, G, st);
  if (ev) (void)hipEventRecord(ev[2], st);
  if (A.train && A.run_update) {
    if (A.compact) {
      if constexpr (NC == 1 && !Model<VEC, NC, SK>::WIDE)
        hipLaunchKernelGGL((update_kernel<Model, VEC, NC, SK, KGE_UPD_COMPACT_WPE, true>), dim3(G.gridU),
                           dim3(kUpdThreads), 0, st, A);
      else
        hipLaunchKernelGGL((update_kernel<Model, VEC, NC, SK, KGE_UPD_WIDE_WPE, true>), dim3(G.gridU),
                           dim3(kUpdThreads), 0, st, A);
    } else if constexpr (NC >= 2 || Model<VEC, NC, SK>::WIDE) {
      hipLaunchKernelGGL((update_kernel<Model, VEC, NC, SK, KGE_UPD_WIDE_WPE>), dim3(G.gridU), dim3(kUpdThreads), 0,
                         st, A);
    } else {
      hipLaunchKernelGGL((update_kernel<Model, VEC, NC, SK>), dim3(G.gridU), dim3(kUpdThreads), 0, st, A);
    }
    if (A.rel_seg) launch_rel_seg(A, st);
    if (A.pos_only) hipLaunchKernelGGL(long_rows_kernel<0>, dim3(kLongWGs), dim3(1024), 0, st, A);
  }
  return KGE_OK;
}

#ifndef KGE_ONLY_ONE
template <template <int, int, int> class Model, int VEC, int NC>
static kge_status by_sk(const StepArgs& A, const StepGeom& G, int sk, hipStream_t st, hipEvent_t const* ev) {
  switch (sk) {
    case SK_P1: return launch_family<Model, VEC, NC, SK_P1>(A, G, st, ev);
    case SK_P2: return launch_family<Model, VEC, NC, SK_P2>(A, G, st, ev);
    case SK_PINF: return launch_family<Model, VEC, NC, SK_PINF>(A, G, st, ev);
    case SK_PGEN: return launch_family<Model, VEC, NC, SK_PGEN>(A, G, st, ev);
    default: return launch_family<Model, VEC, NC, SK_DOT>(A, G, st, ev);
  }
}

template <template <int, int, int> class Model, int VEC, int NC>
static kge_status by_sk_lp(const StepArgs& A, const StepGeom& G, int sk, hipStream_t st, hipEvent_t const* ev) {
  switch (sk) {
    case SK_P1: return launch_family<Model, VEC, NC, SK_P1>(A, G, st, ev);
    case SK_P2: return launch_family<Model, VEC, NC, SK_P2>(A, G, st, ev);
    case SK_PINF: return launch_family<Model, VEC, NC, SK_PINF>(A, G, st, ev);
    case SK_PGEN: return launch_family<Model, VEC, NC, SK_PGEN>(A, G, st, ev);
    default: return KGE_EUNSUPPORTED;
  }
}

#endif  // KGE_ONLY_ONE

}  // namespace kge
