// C-ABI layer of libkge_hip.so: descriptor validation, launch geometry,
// workspace layout and the standalone sampler / constraint kernels.
// Never throws across the ABI; errors -> kge_status + kge_last_error().
#include <algorithm>
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <string>

#include "kge_owner.h"
#include "kge_proj.h"

using namespace kge;

namespace {

thread_local std::string g_err;

kge_status fail(kge_status s, const char* fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof(buf), fmt, ap);
  va_end(ap);
  g_err = buf;
  return s;
}

kge_status hip_check(const char* what) {
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) return fail(KGE_EHIP, "%s: %s", what, hipGetErrorString(e));
  return KGE_OK;
}

inline int64_t ceil_div(int64_t a, int64_t b) { return (a + b - 1) / b; }
inline int64_t round_up(int64_t a, int64_t b) { return ceil_div(a, b) * b; }
inline int next_pow2(int64_t x) { int p = 1; while (p < x) p <<= 1; return p; }
inline bool aligned(const void* p, size_t a) { return ((uintptr_t)p % a) == 0; }

constexpr int kWaves = 4;      // constrain / sample / apply kernels: waves per workgroup


struct Plan {
  StepArgs A;
  StepGeom G;
  int sk;
  uint64_t ws_bytes;
  // workspace offsets
  uint64_t o_ctl, o_cnt, o_coef, o_snap, o_gpos, o_part, o_list, o_ovf;
  // dense-gradient / relation-matrix models (RESCAL)
  uint64_t o_upart, o_sorted, o_srel, o_gproj, o_rpart, o_regpart, o_gent, o_grel;
  uint64_t o_gneg, o_dm;   // TransR
  uint64_t o_leaders, o_htab, o_relseg, o_lng, o_rsorted, o_rsrel, o_rsbeg;
  int hbits;
  uint64_t o_gnegp, o_gpos2, o_gdense[3], o_dpart;   // TransH / TransD
  uint64_t o_owncodes;                               // owner-side scoring
  uint64_t o_segraw, o_segkeys, o_segpart;           // owner merge update: segmented sum
  bool rescal, transr, proj, td, pj_dense, own, omerge, pos_only, seg;
  uint32_t lng_cap;
  uint32_t sig;   // workspace plan signature
};

int score_sk(int kind, float p) {
  if (kind == KGE_SCORE_DOT) return SK_DOT;
  if (std::isinf(p)) return SK_PINF;
  return p == 1.f ? SK_P1 : p == 2.f ? SK_P2 : SK_PGEN;
}

kge_status check_table(const kge_table& t, const char* name, int64_t cols) {
  if (!t.data) return fail(KGE_EINVAL, "%s: null data pointer", name);
  if (t.rows <= 0) return fail(KGE_EINVAL, "%s: rows must be > 0 (got %lld)", name, (long long)t.rows);
  if (t.cols != cols)
    return fail(KGE_EINVAL, "%s: expected %lld columns, got %lld", name, (long long)cols, (long long)t.cols);
  if (t.ld < t.cols) return fail(KGE_EINVAL, "%s: ld (%lld) < cols", name, (long long)t.ld);
  return KGE_OK;
}

kge_status make_plan(const kge_step_desc* d, Plan* pl) {
  if (!d) return fail(KGE_EINVAL, "null descriptor");
  if (d->abi_version != KGE_ABI_VERSION)
    return fail(KGE_EINVAL, "abi_version %d != library %d", d->abi_version, KGE_ABI_VERSION);
  const int model = d->model;
  if (model < KGE_MODEL_TRANSE || model > KGE_MODEL_RESCAL)
    return fail(KGE_EUNSUPPORTED, "model %d has no fused kernel in this build", model);
  if (d->dim <= 0) return fail(KGE_EINVAL, "dim must be > 0");
  const bool rescal = model == KGE_MODEL_RESCAL, transr = model == KGE_MODEL_TRANSR;
  const bool td = model == KGE_MODEL_TRANSD, proj = td || model == KGE_MODEL_TRANSH;
  const int64_t entc = model == KGE_MODEL_ROTATE ? 2 * (int64_t)d->dim : d->dim;
  // RESCAL: [R, d, d] matrices; TransR: rel_emb [R, k] (+ rel_proj [R, d, k] in rel_aux);
  // TransD: rel_emb / rel_proj [R, k]
  const int64_t relc = rescal ? (int64_t)d->dim * d->dim : (transr || td) ? d->dim_rel : d->dim;
  if ((transr || td) && d->dim_rel <= 0) return fail(KGE_EINVAL, "dim_rel must be > 0");
  kge_status s;
  if ((s = check_table(d->ent, "ent_emb", entc))) return s;
  if ((s = check_table(d->rel, (model == KGE_MODEL_DISTMULT || rescal) ? "rel_inter" : "rel_emb", relc))) return s;
  if (rescal) {
    // the regulariser makes both gradients dense (RESCAL.py:190-198); without
    // it TF clips by per-lookup slice norms, which need every negative's
    // projection R e -- that case stays on the plugin path
    if (!d->constraint)
      return fail(KGE_EUNSUPPORTED, "RESCAL with constraint=False (slice-norm clipping) has no fused kernel");
    if (d->dim > 256) return fail(KGE_EUNSUPPORTED, "RESCAL fused step supports d <= 256 (got %d)", d->dim);
  }
  if (proj) {
    // TransH rel_hyper [R, d]; TransD rel_proj [R, k] + ent_proj [E, d]
    if ((s = check_table(d->rel_aux, td ? "rel_proj" : "rel_hyper", relc))) return s;
    if (d->rel_aux.rows != d->rel.rows) return fail(KGE_EINVAL, "rel_aux rows != rel_emb rows");
    if (td) {
      if ((s = check_table(d->ent_aux, "ent_proj", entc))) return s;
      if (d->ent_aux.rows != d->ent.rows) return fail(KGE_EINVAL, "ent_proj rows != ent_emb rows");
    }
  }
  if (transr) {
    if ((s = check_table(d->rel_aux, "rel_proj", (int64_t)d->dim * d->dim_rel))) return s;
    if (d->rel_aux.rows != d->rel.rows) return fail(KGE_EINVAL, "rel_proj rows != rel_emb rows");
    if (d->dim > kTrMaxDim || d->dim_rel > kTrMaxDim)
      return fail(KGE_EUNSUPPORTED, "TransR fused step supports embedding sizes <= %d", kTrMaxDim);
  }
  if (d->shard_count > 1) {
    if (rescal || (model == KGE_MODEL_TRANSH && d->constraint))
      return fail(KGE_EUNSUPPORTED, "sharded tables: full-table regulariser models are not sharded");
    if (d->shard_rows <= 0 || d->global_entities <= 0 ||
        d->global_entities > (int64_t)d->shard_count * d->shard_rows ||
        d->ent.rows < (int64_t)d->shard_count * d->shard_rows)
      return fail(KGE_EINVAL, "sharded tables: need shard_count * shard_rows >= global_entities rows");
  }
  if (d->batch < 0) return fail(KGE_EINVAL, "batch must be >= 0");
  if (d->negative_ratio < 0) return fail(KGE_EINVAL, "negative_ratio must be >= 0");
  if (d->corrupt_side < KGE_SIDE_H || d->corrupt_side > KGE_SIDE_HT)
    return fail(KGE_EINVAL, "Invalid corrupt_side, valid options: 'h+t', 'h', 't'");
  if (d->idx_dtype != KGE_IDX_I32 && d->idx_dtype != KGE_IDX_I64)
    return fail(KGE_EINVAL, "idx_dtype must be KGE_IDX_I32 or KGE_IDX_I64");
  if (d->batch > 0 && !d->pos) return fail(KGE_EINVAL, "null positive triples");
  if (d->loss_kind < KGE_LOSS_HINGE || d->loss_kind > KGE_LOSS_SQERR)
    return fail(KGE_EINVAL, "unknown loss kind %d", d->loss_kind);
  if (d->score_kind < KGE_SCORE_LP || d->score_kind > KGE_SCORE_DOT)
    return fail(KGE_EINVAL, "unknown score kind %d", d->score_kind);
  const float p = d->score_p;
  if (d->score_kind != KGE_SCORE_DOT && !(p > 0.f))
    return fail(KGE_EINVAL, "Lp score needs p > 0 (got %g)", (double)p);
  if (model == KGE_MODEL_ROTATE && d->score_kind == KGE_SCORE_DOT)
    return fail(KGE_EUNSUPPORTED, "RotatE with Dot() yields a complex score");
  if (model == KGE_MODEL_ROTATE && !(d->rotate_limit > 0.f))
    return fail(KGE_EINVAL, "RotatE rotate_limit must be > 0");
  if (d->optimizer != KGE_OPT_NONE && d->optimizer != KGE_OPT_SGD && d->optimizer != KGE_OPT_GRAD)
    return fail(KGE_EINVAL, "kge_step optimizer must be NONE, SGD or GRAD (got %d)", d->optimizer);
  if (d->optimizer == KGE_OPT_SGD && !(d->clip_norm > 0.f)) return fail(KGE_EINVAL, "clip_norm must be > 0");
  if (d->optimizer == KGE_OPT_GRAD && (!d->grad_out[0] || !d->grad_out[1]))
    return fail(KGE_EINVAL, "KGE_OPT_GRAD needs grad_out[0] (ent) and grad_out[1] (rel)");
  if (d->optimizer == KGE_OPT_GRAD && (transr || proj) && !d->grad_out[2])
    return fail(KGE_EINVAL, "KGE_OPT_GRAD needs grad_out[2] (rel_proj / rel_hyper)");
  if (d->optimizer == KGE_OPT_GRAD && td && !d->grad_out[3])
    return fail(KGE_EINVAL, "KGE_OPT_GRAD needs grad_out[3] (ent_proj) for TransD");
  if (d->optimizer == KGE_OPT_GRAD && !d->norm2_out) return fail(KGE_EINVAL, "KGE_OPT_GRAD needs norm2_out");
  if (!d->loss_out) return fail(KGE_EINVAL, "null loss_out");
  const kge_sampler_desc& sm = d->sampler;
  if (sm.kind == KGE_SAMPLER_GIVEN) {
    if (d->batch > 0 && d->negative_ratio > 0 && !d->neg_ids) return fail(KGE_EINVAL, "GIVEN sampler needs neg_ids");
  } else if (sm.kind == KGE_SAMPLER_UNIFORM) {
    if (sm.n_entities <= 0) return fail(KGE_EINVAL, "uniform sampler: empty pool");
  } else if (sm.kind == KGE_SAMPLER_TYPED) {
    if (!sm.ent_type || !sm.type_offsets || !sm.type_members || !sm.pos_in_type || sm.n_types <= 0)
      return fail(KGE_EINVAL, "typed sampler: missing type tables");
  } else {
    return fail(KGE_EINVAL, "unknown sampler kind %d", sm.kind);
  }
  if (sm.idx_dtype != d->idx_dtype && sm.kind != KGE_SAMPLER_GIVEN)
    return fail(KGE_EINVAL, "sampler idx_dtype must match triples");

  const bool own = d->flags & KGE_FLAG_OWNER, omerge = d->flags & KGE_FLAG_OWNER_MERGE;
  const bool ph_s = d->flags & KGE_FLAG_PHASE_SCORE, ph_u = d->flags & KGE_FLAG_PHASE_UPDATE;
  if (own || omerge) {
    if (own && omerge) return fail(KGE_EINVAL, "KGE_FLAG_OWNER and KGE_FLAG_OWNER_MERGE are exclusive");
    if (model != KGE_MODEL_TRANSE && model != KGE_MODEL_DISTMULT && model != KGE_MODEL_ROTATE)
      return fail(KGE_EUNSUPPORTED, "owner-side scoring covers the element-wise family (TransE, DistMult, RotatE)");
    if (!ph_s && !ph_u) return fail(KGE_EINVAL, "owner-side passes run with KGE_FLAG_PHASE_SCORE or _UPDATE");
    if (d->owner_world < 1 || d->owner_rank < 0 || d->owner_rank >= d->owner_world || d->owner_batch < 0)
      return fail(KGE_EINVAL, "owner_world / owner_rank / owner_batch out of range");
    if (own && d->batch != (int64_t)d->owner_world * d->owner_batch)
      return fail(KGE_EINVAL, "KGE_FLAG_OWNER: batch must be owner_world * owner_batch");
    if (omerge && d->batch != d->owner_batch) return fail(KGE_EINVAL, "KGE_FLAG_OWNER_MERGE: batch must be owner_batch");
    if (d->shard_count > 1) return fail(KGE_EINVAL, "owner-side scoring takes local rows (shard_count <= 1)");
    if (own && (d->global_entities <= 0 || d->global_entities >= (int64_t)0x7FFFFFFF * d->owner_world))
      return fail(KGE_EINVAL, "KGE_FLAG_OWNER needs global_entities (the ids' range)");
    if (own && d->owner_rows_from < 0) return fail(KGE_EINVAL, "owner_rows_from must be >= 0");
    if (ph_s && d->batch > 0 && !d->owner_records) return fail(KGE_EINVAL, "owner-side passes need owner_records");
    if (own && ph_u && !d->owner_stats) return fail(KGE_EINVAL, "KGE_FLAG_OWNER | PHASE_UPDATE needs owner_stats");
    if (omerge && ph_s && !d->owner_stats_out) return fail(KGE_EINVAL, "KGE_FLAG_OWNER_MERGE needs owner_stats_out");
    if (d->constraint && (model == KGE_MODEL_TRANSE || model == KGE_MODEL_DISTMULT) &&
        !(d->flags & KGE_FLAG_NO_TABLE_CONSTRAINT))
      return fail(KGE_EINVAL, "owner-side scoring needs KGE_FLAG_NO_TABLE_CONSTRAINT (the caller renormalises its shard)");
  }

  Plan& P = *pl;
  P = Plan{};   // every offset defined (the signature hashes them)
  StepArgs& A = P.A;
  const int K = d->negative_ratio;
  const int Kside = d->corrupt_side == KGE_SIDE_HT ? K / 2 : K;
  const int Keff = d->corrupt_side == KGE_SIDE_HT ? 2 * Kside : K;
  const int64_t B = d->batch;

  // fragment geometry
  int vec;
  const bool a16 = aligned(d->ent.data, 16) && aligned(d->rel.data, 16);
  if (model == KGE_MODEL_ROTATE) {
    vec = (entc % 4 == 0 && d->ent.ld % 4 == 0 && relc % 2 == 0 && d->rel.ld % 2 == 0 && a16) ? 4 : 2;
    if (vec == 2 && !(d->ent.ld % 2 == 0 && aligned(d->ent.data, 8)))
      return fail(KGE_EINVAL, "RotatE ent_emb must be 8-byte aligned with even row stride");
  } else if (proj) {
    // every table of the projection family shares the fragment layout
    const kge_table* tb[4] = {&d->ent, &d->rel, &d->rel_aux, &d->ent_aux};
    auto all = [&](int m) {
      for (int q = 0; q < (td ? 4 : 3); ++q)
        if (tb[q]->cols % m != 0 || tb[q]->ld % m != 0 || !aligned(tb[q]->data, 4 * m)) return false;
      return true;
    };
    vec = all(4) ? 4 : all(2) ? 2 : 1;
  } else {
    vec = (entc % 4 == 0 && relc % 4 == 0 && d->ent.ld % 4 == 0 && d->rel.ld % 4 == 0 && a16) ? 4 : 1;
  }
  const int64_t rowlen = rescal ? entc : std::max(entc, relc);   // fragment row length
  if (transr) {
    const int Keff_ = d->corrupt_side == KGE_SIDE_HT ? 2 * (d->negative_ratio / 2) : d->negative_ratio;
    if (Keff_ + 1 > kTrMaxSlots)
      return fail(KGE_EUNSUPPORTED, "TransR fused step supports negative_ratio <= %d", kTrMaxSlots - 1);
    const TrLds TL = tr_lds(d->dim, d->dim_rel, Keff_);
    if ((size_t)TL.total_floats * 4 + 256 > 160 * 1024)
      return fail(KGE_EUNSUPPORTED, "TransR LDS budget exceeded (%d bytes)", TL.total_floats * 4);
  }
  const int nc = (int)ceil_div(rowlen, 64 * vec);
  if (nc > 4)
    return fail(KGE_EUNSUPPORTED, "row of %lld floats exceeds the fused kernel's %d", (long long)rowlen, 256 * vec);
  const int ncp = nc <= 1 ? 1 : nc <= 2 ? 2 : 4;
  if (proj && ncp > 2)
    return fail(KGE_EUNSUPPORTED, "row of %lld floats exceeds the projection kernel's %d", (long long)rowlen, 128 * vec);

  // score kernel: wpp waves per positive -- the smallest divisor of the
  // workgroup's waves that keeps a wave's share within KGE_SLOTS_PER_WAVE
  // slots, else the whole workgroup -- and kStepWaves / wpp positives per
  // workgroup
  // (owner pass: a positive streams the ~K_eff / owner_world slots it owns)
  const int Kw = own ? (int)ceil_div(Keff, d->owner_world) : Keff;
  int wpp = 1;
  while (wpp < kStepWaves && ((int64_t)wpp * KGE_SLOTS_PER_WAVE < Kw || kStepWaves % wpp != 0)) ++wpp;
  // small grids (C4: 512 positives x 64 negatives gave 64 workgroups for 256
  // CUs): spread each positive's slots over more waves while the grid has
  // fewer than two workgroups per CU and every wave keeps >= 8 slots
  while (wpp < kStepWaves && ceil_div(B, kStepWaves / wpp) < 512 && Kw >= 16 * wpp) wpp *= 2;
  const int nP = kStepWaves / wpp;
  // 'h+t': even slot ranges, so every stream batch starts on an h-corrupt slot
  int SW = std::max<int>(1, (int)ceil_div(Keff, wpp));
  if (d->corrupt_side == KGE_SIDE_HT) SW = (int)round_up(SW, 2);
  const int64_t nWG = std::max<int64_t>(1, ceil_div(B, nP));
  if (nWG > 0x7fffffff) return fail(KGE_EUNSUPPORTED, "batch %lld too large", (long long)B);
  // destination keys: codes i*Keff + j (negatives), B*Keff + 3i + c (positive rows)
  const int64_t E = d->ent.rows, R = d->rel.rows;
  const int64_t ndest = rescal ? E : E + R;   // RESCAL's relation gradient comes from the dR pass
  // key positions: the owner pass's owned negatives (a block per workgroup),
  // the merge pass's positive rows, else every negative + 3 rows per positive
  int64_t T = B * (Keff + 3);
  if (own) {
    T = d->owner_key_capacity > 0 ? d->owner_key_capacity
                                  : std::min<int64_t>(B * Keff, ceil_div(5 * d->owner_batch * Keff, 4) + 4096);
    if (T >= (int64_t)0xFFFFFFFF) return fail(KGE_EUNSUPPORTED, "owner key capacity exceeds 32 bits");
  } else if (omerge) {
    T = 3 * B;
  }
  // destination codes: (i << kshift) | j for slot j of positive i, then
  // (B << kshift) + 4 i + c for the positive's own rows (shift-decoded)
  int kshift = 0;
  while ((1LL << kshift) < Keff) ++kshift;
  if ((B << kshift) + 4 * B >= (int64_t)0xFFFFFFFF)
    return fail(KGE_EUNSUPPORTED, "batch x negative_ratio too large for 32-bit destination codes");
  if (B * 3 * rowlen >= (int64_t)0xFFFFFFFF)
    return fail(KGE_EUNSUPPORTED, "batch x embedding size too large for 32-bit context offsets");
  // per-destination list capacity: ~4x the mean load, 64..256 entries (the
  // update kernel orders up to 256 in registers; longer lists overflow)
  int64_t cap = 64;
  while (cap < 256 && cap < 4 * ceil_div(T, ndest)) cap <<= 1;
  while (cap > 16 && ndest * cap * 4 > ((int64_t)1 << 30)) cap >>= 1;
  if (d->flags & KGE_FLAG_DEBUG_LIST_CAP) cap = 4;   // test hook: exercise the overflow path

  const int FL = 64 * vec * ncp;
  const ScoreLds SL = score_lds(FL, nP, Keff, own);
  P.G.vec = vec;
  P.G.nc = ncp;
  P.G.nWG = (int)nWG;
  // compact update launch: when the tables have far more rows than the step
  // has keys, visit only the touched destinations (not with a fused full-table
  // constraint or a dense gradient, which rewrite every row)
  const bool fuse_norm_plan = (d->optimizer == KGE_OPT_SGD ||
                               (d->optimizer == KGE_OPT_GRAD && (d->flags & KGE_FLAG_GRAD_RENORM))) &&
                              d->constraint &&
                              !(d->flags & KGE_FLAG_NO_TABLE_CONSTRAINT) &&
                              (model == KGE_MODEL_TRANSE || model == KGE_MODEL_DISTMULT) &&
                              !(d->flags & KGE_FLAG_DEBUG_UNFUSED_CONSTRAINT);
  const bool compact = !rescal && !fuse_norm_plan && ndest > 2 * T;
  // compact: hash slots for the destination lists, >= 2 per key
  int hbits = 1;
  while ((1LL << hbits) < 2 * T) ++hbits;
  if (compact) {
    if (hbits > 31) return fail(KGE_EUNSUPPORTED, "batch x negative_ratio too large for the hashed lists");
    if (ndest >= (int64_t)0xFFFFFFFF) return fail(KGE_EUNSUPPORTED, "more than 2^32 - 1 destination rows");
    cap = 64;
    if (d->flags & KGE_FLAG_DEBUG_LIST_CAP) cap = 4;
  }
  const int64_t nlists = compact ? (1LL << hbits) : ndest;
  const int64_t nupd = compact ? ceil_div(T, kUpdKeysPerWave) : ndest;   // compact: waves of kUpdKeysPerWave keys
  P.G.gridU = (int)ceil_div(nupd, kUpdWaves);
  P.rescal = rescal;
  P.transr = transr;
  P.proj = proj;
  P.td = td;
  // TransH + constraint: the soft / orthogonality terms make every gradient dense
  // (a validation step still adds their loss, BaseModel.py:319-323)
  P.pj_dense = proj && !td && d->constraint;
  P.G.lds_score = (size_t)SL.total;
  if (proj) P.G.lds_score = (size_t)pj_lds(Keff, FL, td).total * 4;
  if (P.G.lds_score > 160 * 1024)
    return fail(KGE_EUNSUPPORTED, "LDS budget exceeded (score kernel %zu bytes)", P.G.lds_score);
  P.sk = score_sk(d->score_kind, p);

  A.ent = TabView{d->ent.data, d->ent.ld, (int32_t)entc, E};
  A.n_ent = d->shard_count > 1 ? d->global_entities : E;
  A.rG = d->shard_count > 1 ? d->shard_count : 1;
  A.rEs = d->shard_count > 1 ? d->shard_rows : 0;
  A.rel = TabView{d->rel.data, d->rel.ld, (int32_t)relc, R};
  A.pos = d->pos;
  A.i64 = d->idx_dtype == KGE_IDX_I64;
  A.train = d->optimizer != KGE_OPT_NONE;
  A.grad_mode = d->optimizer == KGE_OPT_GRAD;
  // every entity row is renormalised by the step itself: rows on the stream
  // as they are loaded, every row again (bit-identically) by the update
  // kernel, which writes the normalised row plus this step's SGD delta
  A.fuse_norm = fuse_norm_plan;
  A.compact = compact;
  A.zero_untouched = A.grad_mode && !compact && !rescal && !transr && !proj &&
                     !(d->flags & KGE_FLAG_GRAD_ROWS_TOUCHED);   // (never write an untouched row)
  A.gent = d->grad_out[0];
  A.grel = d->grad_out[1];
  A.grel_aux = d->grad_out[2];
  A.gent_aux = d->grad_out[3];
  A.given = sm.kind == KGE_SAMPLER_GIVEN;
  A.pw = d->score_kind == KGE_SCORE_LP_POW;
  A.rel_half = model == KGE_MODEL_ROTATE;
  A.B = B;
  A.Keff = Keff;
  A.Kside = Kside;
  A.side_mode = d->corrupt_side;
  A.smp = make_sampler_view(sm);
  A.smp.i64 = A.i64;
  A.neg_user = d->neg_ids;
  A.loss_kind = d->loss_kind;
  A.margin = d->margin;
  A.temperature = d->temperature;
  const double bg = (double)B * (d->batch_scale > 0.f ? d->batch_scale : 1.f);
  A.inv_b = (float)(1.0 / bg);
  A.inv_bk = (float)(1.0 / (bg * Keff));
  A.limit = d->rotate_limit;
  A.p = d->score_p;
  A.rel_reg = (model == KGE_MODEL_DISTMULT && d->constraint) ? d->constraint_weight : 0.f;
  A.rel_dests = !rescal;
  // the owner merge's update pass (compact): relation rows by rel_seg_kernel.
  // Not in the other compact launches: there the update kernel's hot-relation
  // waves overlap its ~10^5 other waves, and the extra launch cost C5 24 us
  // the owner merge's SGD update pass as a segmented sum over the positives'
  // keys (launch_merge_segsum): no update kernel / rel_rank / rel_seg /
  // long_rows chain. (KGE_FLAG_DEBUG_NO_REL_SEG keeps the update kernel
  // summing every destination, for A-B tests.)
  int seg_npad = 64;
  if (3 * B > kSegMaxKeys) seg_npad = 2 * kSegMaxKeys;   // (too many keys for one workgroup's sort)
  while (seg_npad < 3 * B) seg_npad <<= 1;
  const bool seg_merge = omerge && d->optimizer == KGE_OPT_SGD && seg_npad <= kSegMaxKeys && rowlen <= 1024 &&
                         entc % 4 == 0 && rowlen % 4 == 0 && (rescal ? entc : relc) % 4 == 0 &&
                         !(d->flags & KGE_FLAG_DEBUG_NO_REL_SEG);
  A.seg_merge = seg_merge;
  A.seg_npad = seg_npad;
  A.rel_seg = compact && omerge && !seg_merge && !(d->flags & KGE_FLAG_DEBUG_NO_REL_SEG);
  A.dense = rescal && A.train;
  A.dense_ent = rescal ? (float)(2.0 * d->constraint_weight / (double)E) : 0.f;
  A.lr = d->lr;
  A.clip_norm = d->clip_norm;
  A.wpp = wpp;
  A.nP = nP;
  A.SW = SW;
  A.nWG = (int32_t)nWG;
  A.cap = (int32_t)cap;
  A.kshift = kshift;
  A.nkeyneg = (uint32_t)(B << kshift);
  A.npos3 = (uint32_t)(3 * B);
  A.nkeys = (uint32_t)T;
  A.snap_cols = (int32_t)entc;
  A.gcols = (int32_t)rowlen;
  A.rel_gcols = (int32_t)(rescal ? entc : relc);
  A.loss_out = d->loss_out;
  A.loss_accum = d->loss_accum;
  A.pos_score_out = d->pos_score_out;
  A.neg_score_out = d->neg_score_out;
  A.norm2_out = d->norm2_out;
  {
    // split step (the multi-GPU sparse exchange): score pass, then update pass
    const bool ps = d->flags & KGE_FLAG_PHASE_SCORE, pu = d->flags & KGE_FLAG_PHASE_UPDATE;
    if (ps || pu) {
      if (ps && pu) return fail(KGE_EINVAL, "KGE_FLAG_PHASE_SCORE and KGE_FLAG_PHASE_UPDATE are exclusive");
      if (rescal || transr || proj)
        return fail(KGE_EUNSUPPORTED, "the split step covers the element-wise family (TransE, DistMult, RotatE)");
      const bool own_val = (own || omerge) && ps && d->optimizer == KGE_OPT_NONE;   // owner validation step
      if (d->optimizer != KGE_OPT_SGD && !own_val) return fail(KGE_EINVAL, "the split step runs KGE_OPT_SGD");
      if (!own_val && (!d->norm2_out || !d->grad_out[1]))
        return fail(KGE_EINVAL, "the split step needs norm2_out and grad_out[1] (relation gradients)");
      if (fuse_norm_plan) return fail(KGE_EINVAL, "the split step needs KGE_FLAG_NO_TABLE_CONSTRAINT");
    }
    A.run_score = !pu;
    A.run_update = !ps;
    A.mark_pending = ps;
    if (pu) {
      A.scale_from_norm2 = true;
      A.rel_grad = true;
      A.grel = d->grad_out[1];
      A.remote_from = d->remote_rows_from > 0 ? d->remote_rows_from : INT64_MAX;
      A.abort_flag = d->abort_flag;
    }
  }
  A.status = d->status;
  P.own = own;
  P.omerge = omerge;
  if (own || omerge) {
    A.own_G = d->owner_world;
    A.own_g = d->owner_rank;
    A.own_Bq = std::max<int64_t>(d->owner_batch, 1);
    A.own_planes = d->corrupt_side == KGE_SIDE_HT ? 2 : 1;
    A.own_rows_from = d->owner_rows_from;
    A.own_rec = d->owner_records;
    A.rec_cols = kRecHead + (model == KGE_MODEL_TRANSE && P.sk != SK_DOT ? 2 : 3) * FL;   // rec_img<M>
    A.own_stats = d->owner_stats;
    A.own_stats_out = d->owner_stats_out;
    A.own_cap = (uint32_t)(own ? T : 0);
    A.own_err = d->owner_err;
    A.own_flags_in = d->owner_flags_in;
    A.own_flags_out = d->owner_flags_out;
    A.own_sticky = d->owner_sticky;
    A.own_keys = own;
    A.n_ent = own ? d->global_entities : E;   // (merge: ids are the caller's table rows)
  }

  uint64_t off = 0;
  auto take = [&](uint64_t bytes) { const uint64_t o = off; off += round_up((int64_t)bytes, 256); return o; };
  const int nsnap = model == KGE_MODEL_ROTATE ? 3 : (transr || proj) ? 0 : 2;
  // zero-state words first: control block, per-destination counters
  P.o_ctl = take(sizeof(StepCtl));
  P.o_cnt = take((uint64_t)(compact ? 1 : ndest) * 4);
  P.o_htab = take((uint64_t)(compact ? nlists : 1) * 8);
  P.o_coef = take((uint64_t)(B << kshift) * 8);   // indexed by destination code
  P.o_snap = take((uint64_t)B * nsnap * entc * 4);
  P.o_gpos = take((uint64_t)(own ? 1 : B * 3 * rowlen) * 4);   // (the owner pass keeps no positive gradients)
  P.o_part = take((uint64_t)((transr || proj) ? std::max<int64_t>(nWG, B) : nWG) * 8 * 4);   // one partial per positive
  P.o_list = take((uint64_t)nlists * cap * 4);
  P.o_ovf = take((uint64_t)T * 8);
  P.o_upart = take((uint64_t)P.G.gridU * 2 * 4);   // gradient norm^2 | entity norm^2 (dense mode)
  P.o_leaders = take((uint64_t)(compact ? (int64_t)P.G.gridU * kUpdWaves * kUpdKeysPerWave : 1) * 16);
  P.hbits = hbits;
  if (rescal) {
    const int64_t nct = ceil_div(d->dim, 16);
    P.o_sorted = take((uint64_t)B * 4);
    P.o_srel = take((uint64_t)B * 4);
    P.o_gproj = take((uint64_t)B * 2 * entc * 4);
    P.o_rpart = take((uint64_t)R * nct * 2 * 4);   // gradient norm^2 | ||R||^2 per strip
    P.o_regpart = take((uint64_t)kRegWGs * 2 * 4);
    if (d->optimizer == KGE_OPT_SGD) {   // dense gradients (KGE_OPT_GRAD: the caller's grad_out)
      P.o_gent = take((uint64_t)E * entc * 4);
      P.o_grel = take((uint64_t)R * relc * 4);
    }
  }
  if (rescal || transr) P.o_relseg = take((uint64_t)R * 2 * 4);
  if (transr) {
    P.o_sorted = take((uint64_t)B * 4);
    P.o_srel = take((uint64_t)B * 4);
    P.o_gneg = take((uint64_t)(B << kshift) * entc * 4);
    P.o_dm = take((uint64_t)B * d->dim * d->dim_rel * 4);
  }
  if (proj) {
    P.o_gneg = take((uint64_t)(B << kshift) * entc * 4);
    if (td) P.o_gnegp = take((uint64_t)(B << kshift) * entc * 4);
    P.o_gpos2 = take((uint64_t)B * 3 * rowlen * 4);
    if (P.pj_dense) {
      if (d->optimizer == KGE_OPT_SGD) {   // KGE_OPT_GRAD: the caller's grad_out
        P.o_gdense[0] = take((uint64_t)E * entc * 4);
        P.o_gdense[1] = take((uint64_t)R * relc * 4);
        P.o_gdense[2] = take((uint64_t)R * relc * 4);
      }
      P.o_dpart = take((uint64_t)kPjDenseWGs * 4 * 4);
    }
  }
  if (own) P.o_owncodes = take((uint64_t)T * 4);
  const bool rel_seg = A.rel_seg;
  if (rel_seg) {   // launch_rel_rank's output for rel_seg_kernel
    P.o_rsorted = take((uint64_t)B * 4);
    P.o_rsrel = take((uint64_t)B * 4);
    P.o_rsbeg = take((uint64_t)R * 2 * 4);
  }
  // owner merge, SGD update pass: long destination lists deferred (kLongN)
  const bool pos_only = omerge && compact && !seg_merge && d->optimizer == KGE_OPT_SGD && !fuse_norm_plan &&
                        entc <= 256 * kLongCPT;
  P.seg = seg_merge;
  if (seg_merge) {
    P.o_segraw = take((uint64_t)3 * B * 8);
    P.o_segkeys = take((uint64_t)3 * B * 8);
    P.o_segpart = take((uint64_t)2 * ceil_div(3 * B, 4) * rowlen * 4);   // (chunks of >= 4 keys)
  }
  const uint32_t lng_cap = (uint32_t)(T / kLongN + 1);
  if (pos_only) P.o_lng = take((uint64_t)lng_cap * 16);
  P.pos_only = pos_only;
  P.lng_cap = lng_cap;
  P.ws_bytes = std::max<uint64_t>(off, 256);
  // the plan's workspace signature (kge_hip.h): FNV-1a over everything that
  // decides where a counter, list or ticket lives and what it means
  {
    const int64_t f[] = {model, B, Keff, Kside, d->corrupt_side, E, R, entc, relc, rowlen, d->dim, d->dim_rel,
                         (int64_t)compact, cap, hbits, kshift, nWG, P.G.gridU, vec, ncp, wpp, SW, d->optimizer,
                         d->flags & ~(KGE_FLAG_PHASE_SCORE | KGE_FLAG_PHASE_UPDATE), d->constraint,
                         d->shard_count, (int64_t)P.ws_bytes,
                         (int64_t)P.o_cnt, (int64_t)P.o_htab, (int64_t)P.o_coef, (int64_t)P.o_snap,
                         (int64_t)P.o_gpos, (int64_t)P.o_part, (int64_t)P.o_list, (int64_t)P.o_ovf,
                         (int64_t)P.o_upart, (int64_t)P.o_leaders, (int64_t)P.o_sorted, (int64_t)P.o_relseg,
                         (int64_t)P.o_gneg, (int64_t)P.o_dpart, (int64_t)P.o_owncodes, (int64_t)P.o_segraw, (int64_t)P.o_segkeys,
                         (int64_t)P.o_segpart, T,
                         (int64_t)d->owner_world, (int64_t)d->owner_batch};
    uint32_t h = 2166136261u;
    for (const int64_t v : f)
      for (int b = 0; b < 8; ++b) h = (h ^ (uint32_t)((uint64_t)v >> (8 * b) & 0xFF)) * 16777619u;
    P.sig = (h == 0u || h == kPoisonedSig) ? 1u : h;   // (0: a fresh workspace; kPoisonedSig: refused)
    A.sig = P.sig;
  }
  return KGE_OK;
}

// ------------------------------------------------------------ sampler kernel
__global__ __launch_bounds__(256) void sample_kernel(SamplerView s, const void* X, int64_t n, int side,
                                                      int K, void* out, int64_t E, int32_t* status) {
  const int64_t total = n * (int64_t)K;
  int err = 0;
  for (int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; q < total;
       q += (int64_t)gridDim.x * blockDim.x) {
    const int64_t i = q / K;
    int64_t e = 0;
    const int64_t x = load_idx(X, i * 3 + (side == KGE_SIDE_H ? 0 : 2), s.i64);
    if (s.kind == KGE_SAMPLER_TYPED && (x < 0 || x >= E)) err = KGE_ERANGE;
    else {
      e = sample_entity(s, s.offset, (uint64_t)q, x, &err);
      if (e < 0) e = 0;
    }
    store_idx(out, q, e, s.i64);
  }
  if (err) set_status(status, err);
}

// ------------------------------------------------------------ phase gate
// The first launch of a PHASE_UPDATE call (include/kge_hip.h, "split step").
// The update pass consumes the lists, coefficients and context rows its
// PHASE_SCORE call left in the workspace; it may run only if that score pass
// ran on this plan since the last update pass. The score pass's last
// workgroup leaves its plan signature in ctl->score_pending; the gate takes
// it (resets the word) and, finding none -- a fresh or re-zeroed workspace,
// another plan's score pass, a second update pass -- stamps kPoisonedSig as
// the workspace's plan, so every guarded kernel of the update pass (and of
// any later step, until the caller zeroes the workspace) refuses it: status
// KGE_EWORKSPACE, no table written. The gate also zero-fills the relation
// gradient rows the update pass accumulates into (n floats at zero).
__global__ __launch_bounds__(256) void phase_gate_kernel(StepCtl* ctl, uint32_t sig, int32_t* status,
                                                         float* zero, int64_t n) {
  for (int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; q < n; q += (int64_t)gridDim.x * blockDim.x)
    zero[q] = 0.f;
  if (blockIdx.x == 0 && threadIdx.x == 0) phase_gate_check(ctl, sig, status);   // (kge_owner.h)
}

static void launch_phase_gate(StepCtl* ctl, uint32_t sig, int32_t* status, float* zero, int64_t n, hipStream_t st) {
  const int64_t blocks = std::max<int64_t>(1, std::min<int64_t>(ceil_div(n, 256 * 4), 256));
  hipLaunchKernelGGL(phase_gate_kernel, dim3((unsigned)blocks), dim3(256), 0, st, ctl, sig, status, zero, n);
}

// ------------------------------------------------------------ apply rows
// rows[i] of var += -lr * clip * g[i]: one wave per listed row
__global__ __launch_bounds__(256) void apply_rows_kernel(float* __restrict__ w, int64_t ld, int32_t cols,
                                                          const int64_t* __restrict__ rows, int64_t n,
                                                          const float* __restrict__ g, int64_t gld,
                                                          const float* __restrict__ norm2, float lr, float clip) {
  const float cs = clip / fmaxf(sqrtf(*norm2), clip);
  const int64_t nw = (int64_t)gridDim.x * (blockDim.x / KGE_WAVE);
  for (int64_t i = (int64_t)blockIdx.x * (blockDim.x / KGE_WAVE) + wave_id(); i < n; i += nw) {
    float* wr = w + rows[i] * ld;
    const float* gr = g + i * gld;
    for (int c = lane_id(); c < cols; c += KGE_WAVE) wr[c] = wr[c] + (gr[c] * cs) * (-lr);
  }
}

}  // namespace

namespace kge {
void kge_set_error(const char* msg) { g_err = msg; }
}  // namespace kge

extern "C" {

kge_status kge_apply_rows(const kge_apply_rows_desc* d, void* stream) {
  if (!d) return fail(KGE_EINVAL, "null descriptor");
  const kge_table& t = d->var;
  if (!t.data || t.rows < 0 || t.cols <= 0 || t.ld < t.cols) return fail(KGE_EINVAL, "kge_apply_rows: bad table");
  if (d->n < 0) return fail(KGE_EINVAL, "kge_apply_rows: n must be >= 0");
  if (d->n == 0) return KGE_OK;
  if (!d->rows || !d->grad || !d->norm2 || d->grad_ld < t.cols)
    return fail(KGE_EINVAL, "kge_apply_rows: null rows / grad / norm2 or grad_ld < cols");
  if (!(d->clip_norm > 0.f)) return fail(KGE_EINVAL, "kge_apply_rows: clip_norm must be > 0");
  const int64_t blocks = std::min<int64_t>(ceil_div(d->n, kWaves), 8192);
  hipLaunchKernelGGL(apply_rows_kernel, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)stream, t.data, t.ld,
                     (int32_t)t.cols, d->rows, d->n, d->grad, d->grad_ld, d->norm2, d->lr, d->clip_norm);
  return hip_check("kge_apply_rows");
}

static kge_status apply_args(const kge_apply_desc* d, ApplyArgs* out, const char* who) {
  if (!d) return fail(KGE_EINVAL, "%s: null descriptor", who);
  const kge_table& t = d->var;
  if (!t.data || t.rows < 0 || t.cols <= 0 || t.ld < t.cols) return fail(KGE_EINVAL, "%s: bad table", who);
  if (d->optimizer != KGE_OPT_SGD && d->optimizer != KGE_OPT_ADAM)
    return fail(KGE_EINVAL, "%s: optimizer must be KGE_OPT_SGD or KGE_OPT_ADAM", who);
  if (!d->grad || !d->norm2) return fail(KGE_EINVAL, "%s: null grad / norm2", who);
  if (!(d->clip_norm > 0.f)) return fail(KGE_EINVAL, "%s: clip_norm must be > 0", who);
  const bool adam = d->optimizer == KGE_OPT_ADAM;
  double lr_t = 0.0;
  if (adam) {
    if (!d->m || !d->v) return fail(KGE_EINVAL, "%s: Adam needs m and v slots", who);
    if (d->iteration < 1) return fail(KGE_EINVAL, "%s: Adam iteration must be >= 1", who);
    const double it = (double)d->iteration;
    lr_t = (double)d->lr * std::sqrt(1.0 - std::pow((double)d->beta_2, it)) / (1.0 - std::pow((double)d->beta_1, it));
  }
  ApplyArgs a{};
  a.w = t.data; a.rows = t.rows; a.cols = (int32_t)t.cols; a.ld = t.ld;
  a.g = d->grad; a.norm2 = d->norm2; a.lr = d->lr; a.clip = d->clip_norm;
  a.adam = adam ? 1 : 0; a.m = d->m; a.v = d->v;
  a.b1 = d->beta_1; a.b2 = d->beta_2; a.eps = d->epsilon; a.lr_t = (float)lr_t;
  a.abort = d->abort_flag;
  *out = a;
  return KGE_OK;
}

kge_status kge_apply(const kge_apply_desc* d, void* stream) {
  ApplyArgs a;
  const kge_status s = apply_args(d, &a, "kge_apply");
  if (s != KGE_OK) return s;
  launch_apply(a, (hipStream_t)stream);
  return hip_check("kge_apply");
}

kge_status kge_apply_many(const kge_apply_desc* d, int32_t n, void* stream) {
  if (n < 0 || n > kMaxApply) return fail(KGE_EINVAL, "kge_apply_many: n must be in [0, %d]", kMaxApply);
  if (n > 0 && !d) return fail(KGE_EINVAL, "kge_apply_many: null descriptor array");
  ApplyArgs a[kMaxApply];
  for (int i = 0; i < n; ++i) {
    const kge_status s = apply_args(d + i, &a[i], "kge_apply_many");
    if (s != KGE_OK) return s;
  }
  launch_apply_many(a, n, (hipStream_t)stream);
  return hip_check("kge_apply_many");
}

kge_status kge_stream_batch(const kge_stream_desc* d, void* stream) {
  if (!d) return fail(KGE_EINVAL, "null descriptor");
  if (d->abi_version != KGE_ABI_VERSION)
    return fail(KGE_EINVAL, "abi_version %d != library %d", d->abi_version, KGE_ABI_VERSION);
  if (d->idx_dtype != KGE_IDX_I32 && d->idx_dtype != KGE_IDX_I64)
    return fail(KGE_EINVAL, "kge_stream_batch: idx_dtype must be KGE_IDX_I32 or KGE_IDX_I64");
  if (d->n_rows <= 0) return fail(KGE_EINVAL, "kge_stream_batch: n_rows must be > 0 (empty triple set)");
  if (d->start < 0 || d->batch < 0) return fail(KGE_EINVAL, "kge_stream_batch: start and batch must be >= 0");
  if (d->n_rows > (int64_t)1 << 62) return fail(KGE_ERANGE, "kge_stream_batch: n_rows exceeds 2^62");
  if (d->batch == 0) return KGE_OK;
  if (d->start > INT64_MAX - d->batch) return fail(KGE_ERANGE, "kge_stream_batch: stream position overflows");
  if (!d->triples || !d->out) return fail(KGE_EINVAL, "kge_stream_batch: null triples / out");
  if (d->shuffle != 0 && d->shuffle != 1) return fail(KGE_EINVAL, "kge_stream_batch: shuffle must be 0 or 1");
  launch_stream(d->triples, d->idx_dtype == KGE_IDX_I64, d->n_rows, d->start, d->batch, d->seed, d->shuffle, d->out,
                (hipStream_t)stream);
  return hip_check("kge_stream_batch");
}

static kge_status stream_check(const kge_stream_desc* d, const char* fn) {
  if (!d) return fail(KGE_EINVAL, "null descriptor");
  if (d->abi_version != KGE_ABI_VERSION)
    return fail(KGE_EINVAL, "abi_version %d != library %d", d->abi_version, KGE_ABI_VERSION);
  if (d->n_rows <= 0) return fail(KGE_EINVAL, "%s: n_rows must be > 0 (empty triple set)", fn);
  if (d->n_rows > INT32_MAX) return fail(KGE_ERANGE, "%s: n_rows exceeds 2^31 - 1 (int32 permutation)", fn);
  return KGE_OK;
}

kge_status kge_stream_permutation(const kge_stream_desc* d, int64_t epoch, int32_t* perm, void* stream) {
  if (kge_status s = stream_check(d, "kge_stream_permutation")) return s;
  if (epoch < 0) return fail(KGE_EINVAL, "kge_stream_permutation: epoch must be >= 0");
  if (!perm) return fail(KGE_EINVAL, "kge_stream_permutation: null perm");
  if (d->shuffle != 1) return fail(KGE_EINVAL, "kge_stream_permutation: shuffle must be 1 (epoch order needs none)");
  launch_stream_perm(d->n_rows, d->seed, epoch, perm, (hipStream_t)stream);
  return hip_check("kge_stream_permutation");
}

kge_status kge_stream_batch_perm(const kge_stream_desc* d, const int32_t* perm_lo, const int32_t* perm_hi,
                                 int64_t epoch_lo, void* stream) {
  if (kge_status s = stream_check(d, "kge_stream_batch_perm")) return s;
  if (d->idx_dtype != KGE_IDX_I32 && d->idx_dtype != KGE_IDX_I64)
    return fail(KGE_EINVAL, "kge_stream_batch_perm: idx_dtype must be KGE_IDX_I32 or KGE_IDX_I64");
  if (d->start < 0 || d->batch < 0) return fail(KGE_EINVAL, "kge_stream_batch_perm: start and batch must be >= 0");
  if (d->batch == 0) return KGE_OK;
  if (d->start > INT64_MAX - d->batch) return fail(KGE_ERANGE, "kge_stream_batch_perm: stream position overflows");
  if (!d->triples || !d->out || !perm_lo) return fail(KGE_EINVAL, "kge_stream_batch_perm: null triples / out / perm_lo");
  const int64_t e0 = d->start / d->n_rows, e1 = (d->start + d->batch - 1) / d->n_rows;
  if (e0 != epoch_lo || e1 > epoch_lo + 1)
    return fail(KGE_EINVAL, "kge_stream_batch_perm: the batch spans epochs %lld..%lld, permutations given for %lld..%lld",
                (long long)e0, (long long)e1, (long long)epoch_lo, (long long)(epoch_lo + 1));
  if (e1 != e0 && !perm_hi) return fail(KGE_EINVAL, "kge_stream_batch_perm: the batch straddles epochs: perm_hi needed");
  launch_stream_gather(d->triples, d->idx_dtype == KGE_IDX_I64, d->n_rows, d->start, d->batch, perm_lo,
                       perm_hi ? perm_hi : perm_lo, epoch_lo, d->out, (hipStream_t)stream);
  return hip_check("kge_stream_batch_perm");
}

kge_status kge_histogram(const float* x, int64_t n, const double* lo_width, int32_t buckets,
                         unsigned long long* counts, void* stream) {
  if (n < 0 || buckets < 1 || buckets > 256) return fail(KGE_EINVAL, "kge_histogram: n >= 0, 1 <= buckets <= 256");
  if (n == 0) return KGE_OK;
  if (!x || !lo_width || !counts) return fail(KGE_EINVAL, "kge_histogram: null x / lo_width / counts");
  launch_histogram(x, n, lo_width, buckets, counts, (hipStream_t)stream);
  return hip_check("kge_histogram");
}

kge_status kge_copy16(const void* src, void* dst, int64_t n16, void* stream) {
  if (n16 < 0 || n16 > ((int64_t)1 << 40)) return fail(KGE_EINVAL, "kge_copy16: n16 must be in [0, 2^40]");
  if (n16 == 0) return KGE_OK;
  if (!src || !dst || ((uintptr_t)src | (uintptr_t)dst) & 15)
    return fail(KGE_EINVAL, "kge_copy16: null or unaligned src / dst");
  launch_copy16(src, dst, n16, (hipStream_t)stream);
  return hip_check("kge_copy16");
}

int32_t kge_abi_version(void) { return KGE_ABI_VERSION; }

const char* kge_last_error(void) { return g_err.c_str(); }

uint64_t kge_step_workspace_bytes(const kge_step_desc* d) {
  Plan P;
  if (make_plan(d, &P) != KGE_OK) return 0;
  return P.ws_bytes;
}

uint32_t kge_step_plan_signature(const kge_step_desc* d) {
  Plan P;
  if (make_plan(d, &P) != KGE_OK) return 0;
  return P.sig;
}

int64_t kge_owner_record_floats(const kge_step_desc* d) {
  Plan P;
  if (make_plan(d, &P) != KGE_OK) return 0;
  return P.A.rec_cols > 0 ? P.A.rec_cols
                         : kRecHead + (d->model == KGE_MODEL_TRANSE && P.sk != SK_DOT ? 2 : 3) * 64 * P.G.vec * P.G.nc;
}

kge_status kge_step(const kge_step_desc* d, void* stream) {
  Plan P;
  kge_status s = make_plan(d, &P);
  if (s != KGE_OK) return s;
  if (d->workspace_bytes < P.ws_bytes || !d->workspace)
    return fail(KGE_ENOMEM_WORKSPACE, "workspace of %llu bytes < required %llu",
                (unsigned long long)d->workspace_bytes, (unsigned long long)P.ws_bytes);
  hipStream_t st = (hipStream_t)stream;
  StepArgs& A = P.A;
  unsigned char* ws = (unsigned char*)d->workspace;
  A.ctl = (StepCtl*)(ws + P.o_ctl);
  A.cnt = (uint32_t*)(ws + P.o_cnt);
  A.coef = (float2*)(ws + P.o_coef);
  A.snap = (float*)(ws + P.o_snap);
  A.gpos = (float*)(ws + P.o_gpos);
  A.part = (float*)(ws + P.o_part);
  A.list = (uint32_t*)(ws + P.o_list);
  A.ovf = (uint64_t*)(ws + P.o_ovf);
  A.upart = (float*)(ws + P.o_upart);
  A.leaders = (uint4*)(ws + P.o_leaders);
  A.htab = (unsigned long long*)(ws + P.o_htab);
  A.hshift = (uint32_t)(P.hbits < 32 ? 32 - P.hbits : 0);
  A.hmask = (uint32_t)((1LL << P.hbits) - 1);
  A.gpe = A.gpos;
  A.gpe_stride = 3 * A.gcols;
  A.gpe_toff = 2 * A.gcols;
  if (P.own) A.own_codes = (uint32_t*)(ws + P.o_owncodes);
  if (A.rel_seg) {
    A.rs_sorted = (int32_t*)(ws + P.o_rsorted);
    A.rs_srel = (int32_t*)(ws + P.o_rsrel);
    A.rs_beg = (int32_t*)(ws + P.o_rsbeg);
  }
  if (P.pos_only) {
    A.pos_only = true;
    A.lng = (uint4*)(ws + P.o_lng);
    A.lng_cap = P.lng_cap;
  }
  if (P.seg) {
    A.seg_raw = (unsigned long long*)(ws + P.o_segraw);
    A.seg_keys = (unsigned long long*)(ws + P.o_segkeys);
    A.seg_part = (float*)(ws + P.o_segpart);
  }
  if (P.own || P.omerge) {
    // owner-side scoring: OWNER | SCORE (owner pass), OWNER | UPDATE
    // (coefficients + the owned rows' update), OWNER_MERGE | SCORE (merge),
    // OWNER_MERGE | UPDATE (the positives' rows: the split step's update pass)
    hipEvent_t const* ev = (hipEvent_t const*)d->prof_events;
    if (ev) { (void)hipEventRecord(ev[0], st); (void)hipEventRecord(ev[1], st); }
    const bool upd = d->flags & KGE_FLAG_PHASE_UPDATE;
    if (d->batch > 0) {
      // the phase gate; the merge's relation gradients start from zero
      // (rel_seg writes every row's every column itself)
      if (upd && !P.own && !(P.omerge && P.seg)) {   // (owner_coef_kernel and the segmented merge update gate themselves)
        const bool zero = P.omerge && !(A.rel_seg && A.rel_gcols == A.rel.cols);
        launch_phase_gate(A.ctl, A.sig, A.status, zero ? d->grad_out[1] : nullptr,
                          zero ? A.rel.rows * (int64_t)A.rel_gcols : 0, st);
      }
      const int phase = upd ? 1 : P.own ? 0 : 2;
      if (!upd || P.own) {
        s = d->model == KGE_MODEL_TRANSE ? launch_owner_transe(A, P.G, P.sk, phase, st)
                                         : launch_owner_other(A, P.G, d->model, P.sk, phase, st);
        if (s != KGE_OK) return fail(s, "no owner-pass instance for model %d / score %d", d->model, P.sk);
      }
      if (ev && !upd) (void)hipEventRecord(ev[2], st);
      if (upd && P.omerge && P.seg) {
        launch_merge_segsum(A, st);
      } else if (upd) {
        A.run_score = false;
        s = launch_step_elementwise(A, P.G, d->model, P.sk, st, ev);
        if (s != KGE_OK) return fail(s, "no kernel instance for model %d / score %d", d->model, P.sk);
      }
    } else if (!upd) {
      (void)hipMemsetAsync(d->loss_out, 0, sizeof(float), st);
    }
    if (ev) (void)hipEventRecord(ev[3], st);
    return hip_check(P.own ? "kge_step(owner pass)" : "kge_step(owner merge)");
  }
  RelArgs RA{};
  TrArgs TA{};
  if (P.transr) {
    A.gneg = (float*)(ws + P.o_gneg);
    RA.ent = A.ent;
    RA.rel = A.rel;
    RA.pos = A.pos;
    RA.i64 = A.i64;
    RA.B = A.B;
    RA.sorted = (int32_t*)(ws + P.o_sorted);
    RA.srel = (int32_t*)(ws + P.o_srel);
    RA.rel_beg = (int32_t*)(ws + P.o_relseg);
    RA.rel_cnt = RA.rel_beg + A.rel.rows;
    RA.status = A.status;
    TA.proj = TabView{d->rel_aux.data, d->rel_aux.ld, (int32_t)(d->dim * d->dim_rel), d->rel_aux.rows};
    TA.d = d->dim;
    TA.k = d->dim_rel;
    TA.clip = d->constraint != 0;
    TA.dmpart = (float*)(ws + P.o_dm);
    TA.sorted = RA.sorted;
    TA.rel_beg = RA.rel_beg;
    TA.rel_cnt = RA.rel_cnt;
    TA.gproj_out = d->optimizer == KGE_OPT_GRAD ? d->grad_out[2] : nullptr;
  }
  if (P.rescal) {
    A.gpe = (float*)(ws + P.o_gproj);
    A.gpe_stride = 2 * d->dim;
    A.gpe_toff = d->dim;
    if (d->optimizer == KGE_OPT_SGD) A.gent = (float*)(ws + P.o_gent);
    RA.ent = A.ent;
    RA.rel = A.rel;
    RA.pos = A.pos;
    RA.i64 = A.i64;
    RA.B = A.B;
    RA.d = d->dim;
    RA.sorted = (int32_t*)(ws + P.o_sorted);
    RA.srel = (int32_t*)(ws + P.o_srel);
    RA.rel_beg = (int32_t*)(ws + P.o_relseg);
    RA.rel_cnt = RA.rel_beg + A.rel.rows;
    RA.snap = A.snap;
    RA.gpos = A.gpos;
    RA.gcols = A.gcols;
    RA.gproj = A.gpe;
    RA.grel = d->optimizer == KGE_OPT_SGD ? (float*)(ws + P.o_grel) : d->grad_out[1];
    RA.rpart = (float*)(ws + P.o_rpart);
    RA.dense_rel = (float)(2.0 * d->constraint_weight / (double)A.rel.rows);
    RA.ctl = A.ctl;
    RA.norm2_out = A.norm2_out;
    RA.status = A.status;
    RA.sig = A.sig;
    RA.loss_out = A.loss_out;
  }

  PjPlan J{};
  if (P.proj) {
    A.gneg = (float*)(ws + P.o_gneg);
    J.P.raux = TabView{d->rel_aux.data, d->rel_aux.ld, (int32_t)d->rel_aux.cols, d->rel_aux.rows};
    J.raux_tab = J.P.raux;
    if (P.td) {
      J.P.eaux = TabView{d->ent_aux.data, d->ent_aux.ld, (int32_t)d->ent_aux.cols, d->ent_aux.rows};
      J.eaux_tab = J.P.eaux;
      J.P.gnegp = (float*)(ws + P.o_gnegp);
    } else {
      J.P.eaux = A.ent;   // never read
    }
    J.P.gpos2 = (float*)(ws + P.o_gpos2);
    J.P.clip = P.td && d->constraint != 0;
    J.P.kmin = std::min(d->dim, d->dim_rel > 0 ? d->dim_rel : d->dim);
    J.td = P.td;
    J.dense = P.pj_dense;
    J.grads = P.pj_dense && d->optimizer != KGE_OPT_NONE;
    J.lam = d->constraint_weight;
    if (J.grads) {
      for (int v = 0; v < 3; ++v)
        J.gdense[v] = d->optimizer == KGE_OPT_GRAD ? d->grad_out[v] : (float*)(ws + P.o_gdense[v]);
    }
    if (P.pj_dense) J.dpart = (float*)(ws + P.o_dpart);
  }
  hipEvent_t const* ev = (hipEvent_t const*)d->prof_events;
  if (ev) (void)hipEventRecord(ev[0], st);
  const bool phase_update = d->flags & KGE_FLAG_PHASE_UPDATE;
  if (phase_update) {
    // the update pass alone (the score pass ran in the previous call): the
    // phase gate, which also zero-fills the relation gradients it accumulates
    if (d->batch > 0) launch_phase_gate(A.ctl, A.sig, A.status, d->grad_out[1], A.rel.rows * (int64_t)A.rel_gcols, st);
    if (ev) (void)hipEventRecord(ev[1], st);
    if (d->batch > 0) s = launch_step_elementwise(A, P.G, d->model, P.sk, st, ev);
    if (s != KGE_OK) return fail(s, "no kernel instance for model %d / score %d", d->model, P.sk);
    if (ev) (void)hipEventRecord(ev[3], st);
    return hip_check("kge_step(update pass)");
  }
  const bool zero_ent = !(d->flags & KGE_FLAG_GRAD_ROWS_TOUCHED);
  // (RESCAL's dense passes write every row; so does a non-compact update
  // launch in grad mode, zeros for the untouched ones)
  if (A.grad_mode && !P.rescal && (!A.zero_untouched || d->batch == 0)) {
    if (zero_ent) (void)hipMemsetAsync(d->grad_out[0], 0, (size_t)A.ent.rows * A.ent.cols * sizeof(float), st);
    (void)hipMemsetAsync(d->grad_out[1], 0, (size_t)A.rel.rows * A.rel_gcols * sizeof(float), st);
    if (P.transr) (void)hipMemsetAsync(d->grad_out[2], 0, (size_t)TA.proj.rows * TA.proj.cols * sizeof(float), st);
    if (P.proj) (void)hipMemsetAsync(d->grad_out[2], 0, (size_t)d->rel_aux.rows * d->rel_aux.cols * sizeof(float), st);
    if (P.td && zero_ent)
      (void)hipMemsetAsync(d->grad_out[3], 0, (size_t)d->ent_aux.rows * d->ent_aux.cols * sizeof(float), st);
  }
  if (P.pj_dense && d->optimizer == KGE_OPT_SGD && d->batch > 0) {
    // the update passes write only the touched rows of the dense gradients
    (void)hipMemsetAsync(J.gdense[0], 0, (size_t)A.ent.rows * A.ent.cols * sizeof(float), st);
    (void)hipMemsetAsync(J.gdense[1], 0, (size_t)A.rel.rows * A.rel.cols * sizeof(float), st);
    (void)hipMemsetAsync(J.gdense[2], 0, (size_t)d->rel_aux.rows * d->rel_aux.cols * sizeof(float), st);
  }
  if (P.proj && d->constraint && !(d->flags & KGE_FLAG_NO_TABLE_CONSTRAINT)) {
    // _constraint_loss assigns: TransH normalises rel_hyper (TransH.py:202);
    // TransD clips ent_emb and rel_emb (TransD.py:238-240)
    const kge_table& t0 = P.td ? d->ent : d->rel_aux;
    const int64_t blocks = std::min<int64_t>(ceil_div(t0.rows + (P.td ? d->rel.rows : 0), kWaves), 4096);
    hipLaunchKernelGGL(constrain_rows_kernel, dim3((unsigned)blocks), dim3(256), 0, st, t0.data, t0.rows,
                       (int32_t)t0.cols, t0.ld, P.td ? 1 : 0, 1.0f, A.ctl, A.sig, A.status,
                       P.td ? d->rel.data : (float*)nullptr, d->rel.rows, (int32_t)d->rel.cols, d->rel.ld);
  }
  if (P.transr && d->constraint && !(d->flags & KGE_FLAG_NO_TABLE_CONSTRAINT)) {
    // _constraint_loss assigns (TransR.py:207-209): clip every entity and relation row to norm <= 1
    const int64_t blocks = std::min<int64_t>(ceil_div(d->ent.rows + d->rel.rows, kWaves), 4096);
    hipLaunchKernelGGL(constrain_rows_kernel, dim3((unsigned)blocks), dim3(256), 0, st, d->ent.data, d->ent.rows,
                       (int32_t)d->ent.cols, d->ent.ld, 1, 1.0f, A.ctl, A.sig, A.status, d->rel.data, d->rel.rows,
                       (int32_t)d->rel.cols, d->rel.ld);
  }
  // _constraint_loss assigns before scoring (BaseModel.py:319): fused into
  // the score / update kernels on the SGD path (A.fuse_norm), else K0
  const bool renorm = d->constraint && !(d->flags & KGE_FLAG_NO_TABLE_CONSTRAINT) &&
                      (d->model == KGE_MODEL_TRANSE || d->model == KGE_MODEL_DISTMULT);
  if (renorm && !(A.fuse_norm && d->batch > 0)) {
    const int64_t blocks = std::min<int64_t>(ceil_div(d->ent.rows, kWaves), 4096);
    hipLaunchKernelGGL(constrain_rows_kernel, dim3((unsigned)blocks), dim3(256), 0, st, d->ent.data,
                       d->ent.rows, (int32_t)d->ent.cols, d->ent.ld, 0, 1.0f, A.ctl, A.sig, A.status,
                       (float*)nullptr, (int64_t)0, 0, (int64_t)0);
  }
  if (d->batch == 0) {
    (void)hipMemsetAsync(d->loss_out, 0, sizeof(float), st);
    return hip_check("kge_step(empty batch)");
  }
  if (ev) (void)hipEventRecord(ev[1], st);
  if (P.proj) {
    s = launch_step_proj(A, P.G, J, P.sk, st, ev);
  } else if (P.transr) {
    s = launch_step_transr(A, P.G, TA, RA, P.sk, st, ev);
  } else if (P.rescal) {
    // (SGD: the dense applies are the chain's last launch, BaseModel.py:327-328)
    RA.lazy_absent = d->optimizer == KGE_OPT_SGD && rescal_apply_fused_ok(RA, A.ent, A.gent);
    s = launch_step_rescal(A, P.G, RA, d->constraint ? d->constraint_weight : 0.f,
                           (float*)(ws + P.o_regpart), st, ev);
  } else {
    s = launch_step_elementwise(A, P.G, d->model, P.sk, st, ev);
  }
  if (s != KGE_OK) return fail(s, "no kernel instance for model %d / score %d", d->model, P.sk);
  if (ev) (void)hipEventRecord(ev[3], st);
  return hip_check("kge_step");
}

kge_status kge_sample(const kge_sample_desc* d, void* stream) {
  if (!d) return fail(KGE_EINVAL, "null descriptor");
  const kge_sampler_desc& sm = d->sampler;
  if (sm.kind != KGE_SAMPLER_UNIFORM && sm.kind != KGE_SAMPLER_TYPED)
    return fail(KGE_EINVAL, "kge_sample: sampler kind must be UNIFORM or TYPED");
  if (d->side != KGE_SIDE_H && d->side != KGE_SIDE_T) return fail(KGE_EINVAL, "side must be 'h' or 't'");
  if (d->n < 0 || d->negative_ratio < 0) return fail(KGE_EINVAL, "negative sizes");
  if (sm.n_entities <= 0) return fail(KGE_EINVAL, "sampler: n_entities must be > 0");
  if (sm.kind == KGE_SAMPLER_TYPED &&
      (!sm.ent_type || !sm.type_offsets || !sm.type_members || !sm.pos_in_type || sm.n_types <= 0))
    return fail(KGE_EINVAL, "typed sampler: missing type tables");
  const int64_t total = d->n * (int64_t)d->negative_ratio;
  if (total == 0) return KGE_OK;
  if (!d->X || !d->out) return fail(KGE_EINVAL, "null X / out");
  SamplerView v = make_sampler_view(sm);
  const int64_t blocks = std::min<int64_t>(ceil_div(total, 256), 8192);
  const int64_t E = sm.n_entities;
  hipLaunchKernelGGL(sample_kernel, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)stream, v, d->X,
                     d->n, d->side, d->negative_ratio, d->out, E, d->status);
  return hip_check("kge_sample");
}

kge_status kge_rank(const kge_rank_desc* d, void* stream) {
  if (!d) return fail(KGE_EINVAL, "null descriptor");
  if (d->abi_version != KGE_ABI_VERSION)
    return fail(KGE_EINVAL, "abi_version %d != library %d", d->abi_version, KGE_ABI_VERSION);
  if (d->mode < KGE_RANK_TRANS || d->mode > KGE_RANK_DOT) return fail(KGE_EINVAL, "unknown rank mode %d", d->mode);
  if (d->proj < KGE_RPROJ_NONE || d->proj > KGE_RPROJ_RANK1 || (d->proj != KGE_RPROJ_NONE && d->mode != KGE_RANK_TRANS))
    return fail(KGE_EINVAL, "bad projection %d for rank mode %d", d->proj, d->mode);
  if (d->corrupt_side != KGE_SIDE_H && d->corrupt_side != KGE_SIDE_T)
    return fail(KGE_EINVAL, "corrupt_side must be 'h' or 't'");
  if (d->n < 0) return fail(KGE_EINVAL, "n must be >= 0");
  if (d->n == 0) return KGE_OK;
  if (!d->cand.data || d->cand.rows <= 0 || d->cand.ld < d->cand.cols) return fail(KGE_EINVAL, "bad candidate table");
  if (d->dim <= 0 || !d->q0 || d->ldq < d->dim || !d->true_ids || !d->rank_out || !d->pos_score_out)
    return fail(KGE_EINVAL, "null query rows / ids / outputs");
  const bool hside = d->corrupt_side == KGE_SIDE_H;
  const bool rank1 = d->proj == KGE_RPROJ_RANK1, hyper = d->proj == KGE_RPROJ_HYPER;
  if (hside && d->mode != KGE_RANK_DOT && !d->q1)
    return fail(KGE_EINVAL, "q1 rows needed for corrupt_side 'h'");
  if ((hyper || rank1) && !d->qw) return fail(KGE_EINVAL, "qw rows needed for the projection");
  if (rank1 && (!d->cand_aux.data || d->cand_aux.rows != d->cand.rows || d->cand_aux.cols != d->cand.cols))
    return fail(KGE_EINVAL, "RANK1 needs ent_proj rows shaped like the candidates");
  if (d->mode == KGE_RANK_ROT && (d->dim % 2 || d->cand.cols != d->dim))
    return fail(KGE_EINVAL, "RotatE rows are [d, 2] pairs");
  if (!rank1 && d->cand.cols < d->dim) return fail(KGE_EINVAL, "candidate rows shorter than dim");
  if ((d->filt_beg == nullptr) != (d->filt_end == nullptr) || (d->filt_beg && !d->filt_ent))
    return fail(KGE_EINVAL, "filter needs filt_beg, filt_end and filt_ent");
  const float p = d->score_p;
  if (d->score_kind != KGE_SCORE_DOT && !(p > 0.f))
    return fail(KGE_EINVAL, "Lp score needs p > 0 (got %g)", (double)p);
  if (3 * kRankQ * ((d->dim + 3) & ~3) * 4 > 64 * 1024) return fail(KGE_EUNSUPPORTED, "query rows too wide");
  RankArgs A{};
  A.cand = d->cand.data;
  A.cand_ld = d->cand.ld;
  A.E = d->cand.rows;
  A.caux = d->cand_aux.data;
  A.caux_ld = d->cand_aux.ld;
  A.dim = d->dim;
  A.ecols = (int32_t)d->cand.cols;
  A.kmin = (int32_t)std::min<int64_t>(d->dim, d->cand.cols);
  A.clip = d->clip != 0;
  A.hside = hside;
  A.pw = d->score_kind == KGE_SCORE_LP_POW;
  A.p = p;
  A.q0 = d->q0;
  A.q1 = d->q1;
  A.qw = d->qw;
  A.ldq = d->ldq;
  A.true_ids = d->true_ids;
  A.i64 = d->idx_dtype == KGE_IDX_I64;
  A.n = d->n;
  if (d->flags & ~KGE_RANK_FLAG_LANE_PASS) return fail(KGE_EINVAL, "kge_rank: unknown flags 0x%x", d->flags);
  A.lane_pass = (d->flags & KGE_RANK_FLAG_LANE_PASS) != 0;
  A.fbeg = d->filt_beg;
  A.fend = d->filt_end;
  A.fent = d->filt_ent;
  if (d->filt_bits && d->filt_beg) {   // (no filter: the bitmap is ignored)
    A.fw = (A.E + 31) / 32;
    if (d->filt_bits_words < d->n * A.fw)
      return fail(KGE_EINVAL, "filt_bits: %lld words < n * ceil(E / 32) = %lld", (long long)d->filt_bits_words,
                  (long long)(d->n * A.fw));
    if (d->n > 0x7fffffffLL) return fail(KGE_EINVAL, "filt_bits: more than 2^31 - 1 queries per call");
    A.fbits = d->filt_bits;
  }
  A.rank = (unsigned long long*)d->rank_out;
  A.pos = d->pos_score_out;
  A.status = d->status;
  hipStream_t st = (hipStream_t)stream;
  (void)hipMemsetAsync(d->rank_out, 0, (size_t)d->n * sizeof(int64_t), st);
  const int sk = d->score_kind == KGE_SCORE_DOT ? SK_DOT : score_sk(d->score_kind, p);
  if (launch_rank(A, d->mode, d->proj, sk, st) != KGE_OK)
    return fail(KGE_EUNSUPPORTED, "no ranking instance for mode %d / score %d", d->mode, d->score_kind);
  return hip_check("kge_rank");
}

kge_status kge_constrain_rows(kge_table t, int32_t kind, float value, void* stream) {
  if (!t.data || t.rows < 0 || t.cols <= 0 || t.ld < t.cols) return fail(KGE_EINVAL, "bad table");
  if (kind != 0 && kind != 1) return fail(KGE_EINVAL, "kind must be 0 (normalize) or 1 (clip)");
  if (t.rows == 0) return KGE_OK;
  const int64_t blocks = std::min<int64_t>(ceil_div(t.rows, kWaves), 4096);
  hipLaunchKernelGGL(constrain_rows_kernel, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)stream, t.data,
                     t.rows, (int32_t)t.cols, t.ld, kind, value, (StepCtl*)nullptr, 0u,
                     (int32_t*)nullptr, (float*)nullptr, (int64_t)0, 0, (int64_t)0);
  return hip_check("kge_constrain_rows");
}

}  // extern "C"
