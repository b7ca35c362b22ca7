/*
 * kge_hip.h -- C-ABI of libkge_hip.so, the MI355X (gfx950) native training
 * step for knowledge-graph embeddings.
 *
 * This is the drop-in boundary for the hot path of
 * melissakou/knowledge-graph-embedding (pure-Python TF 2.5; no native code of
 * its own). Every entry point below replaces a Python/TF call site of the
 * reference; the citation is given per entry point. The host side that binds
 * it is the Python package `KGE` (ctypes, knowledge-graph-embedding_amd/KGE/_hip.py);
 * INTEGRATION.md shows the binding.
 *
 * Rules of the ABI
 *  - Plain C types only: device pointers, sizes, enums. No torch / HIP types
 *    in signatures; streams are passed as `void*` (a hipStream_t, NULL = the
 *    legacy default stream).
 *  - The library never allocates device memory: the caller passes a
 *    workspace of at least kge_step_workspace_bytes() bytes, ZERO-FILLED when
 *    it is allocated (a fresh workspace must be zeroed once). Between calls of
 *    one plan its tickets and per-destination counters reset themselves. One
 *    workspace serves one stream at a time.
 *  - The workspace belongs to ONE plan: kge_step_plan_signature() (a hash of
 *    the workspace layout -- model, batch, negatives, table shapes, optimizer
 *    mode, flags) is stamped into the workspace's control block by the first
 *    step that uses it. A step whose plan differs from the stamped one (the
 *    caller changed batch size, tables, ... and reused the buffer without
 *    re-zeroing it) is REFUSED on the device: none of its kernels writes a
 *    table or an output, the status word gets KGE_EWORKSPACE and *loss_out is
 *    NaN. Re-zero the workspace (or allocate a zeroed one) whenever the
 *    signature changes.
 *  - Split steps (KGE_FLAG_PHASE_SCORE, then KGE_FLAG_PHASE_UPDATE): the
 *    update pass consumes what its score pass left in the workspace, so a
 *    PHASE_UPDATE call runs only after a PHASE_SCORE call of the same plan on
 *    the same workspace, once. One that finds no such pending score pass (a
 *    fresh or re-zeroed workspace, a second update, another plan's score
 *    pass) is REFUSED on the device: no table written, status KGE_EWORKSPACE,
 *    and the workspace stays refused for every later step until the caller
 *    zero-fills it (then: PHASE_SCORE again).
 *  - Calls are stream-ordered, re-entrant and never throw. They return a
 *    kge_status; kge_last_error() gives a thread-local message.
 *  - Device-side range violations (entity / relation ids out of range) are
 *    recorded in the caller's `status` word (KGE_ERANGE) and the offending
 *    triple is skipped; the host checks the word at its next sync.
 *  - Tables are fp32, row-major, with a row stride `ld` >= cols (floats).
 */
#ifndef KGE_HIP_H
#define KGE_HIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define KGE_ABI_VERSION 8

typedef enum kge_status {
  KGE_OK = 0,
  KGE_EINVAL = 1,            /* bad argument (reference: Python assert / TF InvalidArgument) */
  KGE_ERANGE = 2,            /* id out of range (reference: TF gather InvalidArgument on CPU) */
  KGE_EHIP = 3,              /* HIP runtime error */
  KGE_ENOMEM_WORKSPACE = 4,  /* workspace smaller than kge_step_workspace_bytes() */
  KGE_EUNSUPPORTED = 5,      /* combination not implemented natively */
  KGE_EWORKSPACE = 6         /* device status: workspace stamped by another plan (step refused) */
} kge_status;

/* models: KGE/models/translating_based/<Model>.py, KGE/models/semantic_based/<Model>.py */
enum {
  KGE_MODEL_TRANSE = 0,   /* TransE.py:127-174   */
  KGE_MODEL_TRANSH = 1,   /* TransH.py:149-213   */
  KGE_MODEL_TRANSR = 2,   /* TransR.py:154-211   */
  KGE_MODEL_TRANSD = 3,   /* TransD.py:170-242   */
  KGE_MODEL_ROTATE = 4,   /* RotatE.py:126-181   */
  KGE_MODEL_DISTMULT = 5, /* DistMult.py:118-167 */
  KGE_MODEL_RESCAL = 6    /* RESCAL.py:140-200   */
};

/* score kinds: KGE/score.py */
enum {
  KGE_SCORE_LP = 0,       /* LpDistance(p)    score.py:49-63 */
  KGE_SCORE_LP_POW = 1,   /* LpDistancePow(p) score.py:65-76 */
  KGE_SCORE_DOT = 2       /* Dot()            score.py:78-89 */
};

/* loss kinds: KGE/loss.py */
enum {
  KGE_LOSS_HINGE = 0,     /* PairwiseHingeLoss                    loss.py:49-82   */
  KGE_LOSS_LOGISTIC = 1,  /* PairwiseLogisticLoss                 loss.py:85-113  */
  KGE_LOSS_BCE = 2,       /* BinaryCrossEntropyLoss               loss.py:116-143 */
  KGE_LOSS_SANS = 3,      /* SelfAdversarialNegativeSamplingLoss  loss.py:146-182 */
  KGE_LOSS_SQERR = 4      /* SquareErrorLoss                      loss.py:185-204 */
};

/* corrupt_side: BaseModel.py:332-408 */
enum { KGE_SIDE_H = 0, KGE_SIDE_T = 1, KGE_SIDE_HT = 2 };

/* index dtype of triples / sampled ids (int64 from numpy, int32 from CSV:
 * data_utils.py:182, ns_strategy.py:57) */
enum { KGE_IDX_I32 = 0, KGE_IDX_I64 = 1 };

/* negative samplers: KGE/ns_strategy.py */
enum {
  KGE_SAMPLER_UNIFORM = 0, /* UniformStrategy ns_strategy.py:39-64            */
  KGE_SAMPLER_TYPED = 1,   /* TypedStrategy   ns_strategy.py:94-132, utils.py:11-16 */
  KGE_SAMPLER_GIVEN = 2    /* negatives supplied by the caller (neg_ids input) */
};

/* optimizer applied by the step (BaseModel.py:325-328)
 *  KGE_OPT_NONE  validation step (BaseModel.py:141-145): loss only
 *  KGE_OPT_SGD   keras SGD sparse apply (ResourceScatterAdd(var, idx, -lr*clip(g)))
 *  KGE_OPT_GRAD  no update: the step writes each variable's duplicate-summed,
 *                UN-clipped gradient into the dense buffers grad_out[v] (rows not
 *                touched are zeroed) and its slice norm^2 into norm2_out[v];
 *                kge_apply() then clips and applies it (Adam, or a multi-GPU
 *                step that reduces gradients across ranks first).
 *  KGE_OPT_ADAM  kge_apply() only: keras Adam (OptimizerV2, TF 2.5). */
enum { KGE_OPT_NONE = 0, KGE_OPT_SGD = 1, KGE_OPT_GRAD = 2, KGE_OPT_ADAM = 3 };

/* kge_step_desc.flags */
enum {
  KGE_FLAG_NO_TABLE_CONSTRAINT = 1, /* caller already applied the full-table
                                       _constraint_loss assigns (e.g. on its shard) */
  KGE_FLAG_DEBUG_LIST_CAP = 2,      /* test hook: 4-entry destination lists, so the
                                       update kernel's overflow path runs */
  KGE_FLAG_DEBUG_UNFUSED_CONSTRAINT = 4, /* test hook: run the full-table renormalisation
                                       as its own kernel even on the SGD path */
  KGE_FLAG_GRAD_ROWS_TOUCHED = 8,    /* KGE_OPT_GRAD: the caller needs only the entity
                                       gradient rows the batch touches: grad_out[0/3] are
                                       written at those rows only (no zero-fill), so they may
                                       address just the range the batch's ids fall in */
  KGE_FLAG_GRAD_RENORM = 16,         /* KGE_OPT_GRAD, TransE / DistMult with constraint:
                                       the renormalisation assign runs inside the step as on
                                       the SGD path (rows scored normalised in registers) and
                                       the step writes every entity row back normalised; the
                                       caller applies its update to those rows (no full-table
                                       pass of its own) */
  /* Split step (the multi-GPU sparse exchange, KGE/sharded.py; TransE /
   * DistMult / RotatE with KGE_OPT_SGD): the same descriptor is passed twice
   * with the same workspace --
   *   PHASE_SCORE   the draws and the score pass: loss_out and norm2_out get
   *                 THIS call's (local) loss and per-variable slice norm^2; no
   *                 update;
   *   PHASE_UPDATE  the update pass alone, its clip scales from norm2_out (the
   *                 caller may have all-reduced them in between); entity rows
   *                 >= remote_rows_from receive their summed raw gradient IN
   *                 PLACE of the row (rows fetched from another rank, sent back
   *                 to their owner), the others the clipped SGD update;
   *                 relation rows' summed raw gradients go to grad_out[1]
   *                 (zero-filled by the call) for the caller to reduce and apply;
   *                 nothing at all when abort_flag is set and *abort_flag != 0.
   *                 Refused (KGE_EWORKSPACE) unless this plan's PHASE_SCORE
   *                 call ran on the workspace since the last update pass (see
   *                 the ABI rules above). */
  KGE_FLAG_PHASE_SCORE = 32,
  KGE_FLAG_PHASE_UPDATE = 64,
  /* Owner-side scoring (the multi-GPU "owner" step, KGE/sharded.py; TransE /
   * DistMult / RotatE): entity e lives on rank e mod owner_world, local row
   * e div owner_world. Each flag is passed with PHASE_SCORE, then (training)
   * PHASE_UPDATE, same descriptor and workspace:
   *   OWNER | PHASE_SCORE   batch = owner_world * owner_batch "virtual"
   *       positives, every rank's (pos = their all-gathered global triples,
   *       rows of positive v at owner_rows_from + 2v (h) and + 2v + 1 (t) of
   *       ent). Each draws its slots exactly as its own rank q draws them
   *       (sampler planes offset + q * (2 for 'h+t', else 1); GIVEN: neg_ids
   *       [batch * K_eff] all-gathered); the slots whose entity this rank owns
   *       are scored here and one record per positive is written to
   *       owner_records (kge_owner_record_floats() floats): partial softmax
   *       state, loss and slice-norm^2 partials, h / r / t gradient
   *       accumulators. No update.
   *   OWNER_MERGE | PHASE_SCORE   batch = owner_batch (this rank's positives,
   *       pos in ent rows): the owner_world records of each positive
   *       (owner_records [owner_world, batch, R], source-major) merged into its
   *       loss, this rank's loss_out / norm2_out shares (the caller all-reduces
   *       them), its row gradients, and owner_stats_out [batch, 4] (softmax
   *       max, 1/Z, positive score) that the caller all-gathers.
   *   OWNER | PHASE_UPDATE   the owned negatives' coefficients from
   *       owner_stats (all ranks' merge outputs) and their rows' SGD update
   *       with the clip scales of norm2_out (all-reduced). Run it BEFORE
   *       OWNER_MERGE | PHASE_UPDATE (whose in-place rows then add to it).
   *   OWNER_MERGE | PHASE_UPDATE   the positives' rows as the split step's
   *       update pass (remote_rows_from, relation gradients to grad_out[1]). */
  KGE_FLAG_OWNER = 128,
  KGE_FLAG_OWNER_MERGE = 256,
  KGE_FLAG_DEBUG_NO_REL_SEG = 512   /* test hook: the owner merge's update pass sums the
                                       relation rows in the update kernel (one wave per
                                       relation) instead of the per-relation segment pass
                                       (same sums up to their order) */
};

typedef struct kge_table {
  float* data;   /* device pointer, row-major                    */
  int64_t rows;
  int64_t cols;  /* floats per row                               */
  int64_t ld;    /* row stride in floats (>= cols)               */
} kge_table;

/*
 * Counter-based sampler state. Draw n of a call uses Philox4x32-10 with
 * key = (seed lo, seed hi) and counter = (block lo, block hi, plane lo,
 * plane hi), block = n / P, P = 4 (int32 ids: one 32-bit word per draw) or
 * 2 (int64 ids: words 2q | 2q+1 << 32), and maps bits -> bits % range as
 * TF's UniformDistribution does. A 'h+t' step uses plane `offset` for the
 * head side and `offset + 1` for the tail side, i.e. exactly two standalone
 * kge_sample() calls (the reference calls the strategy h-side first,
 * BaseModel.py:353-356).
 */
typedef struct kge_sampler_desc {
  int32_t kind;               /* KGE_SAMPLER_*                                  */
  int32_t idx_dtype;          /* KGE_IDX_*                                      */
  uint64_t seed;
  uint64_t offset;            /* counter plane of the first side                */
  int64_t n_entities;         /* uniform: pool length (E unless `pool` given)   */
  const void* pool;           /* uniform: optional pool [n_entities] (idx_dtype); NULL = range(E) */
  const int32_t* ent_type;    /* typed: [E] type id of each entity              */
  const int32_t* type_offsets;/* typed: [n_types+1] CSR offsets                 */
  const int32_t* type_members;/* typed: [E] entity ids grouped by type, ascending*/
  const int32_t* pos_in_type; /* typed: [E] position of entity in its group     */
  int32_t n_types;
  int32_t _pad;
} kge_sampler_desc;

/* Standalone sampler: NegativeSampler.__call__(X, negative_ratio, side)
 * (ns_strategy.py:39-64 uniform, :94-132 typed). out[n*negative_ratio]. */
typedef struct kge_sample_desc {
  kge_sampler_desc sampler;
  const void* X;              /* [n,3] idx_dtype                                */
  int64_t n;
  int32_t side;               /* KGE_SIDE_H or KGE_SIDE_T                       */
  int32_t negative_ratio;
  void* out;                  /* [n*negative_ratio] idx_dtype                   */
  int32_t* status;            /* device status word (nullable)                  */
} kge_sample_desc;

/*
 * One training (or validation) step: KGEModel.__run_single_batch
 * (BaseModel.py:293-330) for the built-in models and plugins:
 *   negative sampling (:316, :332-408) -> _constraint_loss (:319) ->
 *   score_hrt(pos), score_hrt(neg) (:320-321) -> loss_fn (:322-323) ->
 *   gradients (:326) -> clip_by_norm(g, clip_norm) per variable (:327) ->
 *   optimizer.apply_gradients (:328).
 * Variables (per-variable clipping, norm2_out order): 0 ent_emb, 1 the main
 * relation table (rel_emb / rel_inter), 2 rel_aux (rel_hyper / rel_proj),
 * 3 ent_aux (ent_proj).
 */
typedef struct kge_step_desc {
  int32_t abi_version;        /* KGE_ABI_VERSION                                */
  int32_t model;              /* KGE_MODEL_*                                    */
  kge_table ent;              /* ent_emb [E, d]  (RotatE: [E, 2d] = [E,d,2])    */
  kge_table rel;              /* rel_emb / rel_inter [R, d_rel]                 */
  kge_table ent_aux;          /* TransD ent_proj [E, d]                         */
  kge_table rel_aux;          /* TransH rel_hyper [R,d]; TransD rel_proj [R,d_rel] */
  int32_t dim;                /* entity embedding size d                        */
  int32_t dim_rel;            /* relation embedding size                        */

  const void* pos;            /* positives [batch, 3] (h, r, t)                 */
  int32_t idx_dtype;          /* KGE_IDX_*                                      */
  int32_t batch;
  int32_t negative_ratio;
  int32_t corrupt_side;       /* KGE_SIDE_*                                     */

  kge_sampler_desc sampler;
  void* neg_ids;              /* [batch*K_eff] idx_dtype: input for GIVEN, output otherwise (nullable) */

  int32_t score_kind;         /* KGE_SCORE_*                                    */
  float score_p;              /* 1, 2 or +inf                                   */
  int32_t loss_kind;          /* KGE_LOSS_*                                     */
  float margin;
  float temperature;
  float batch_scale;          /* global-batch normalisation (world size), 1 on one device */
  int32_t constraint;         /* model's `constraint` flag                      */
  float constraint_weight;
  float rotate_limit;         /* RotatE self.limit (RotatE.py:93)              */

  int32_t optimizer;          /* KGE_OPT_NONE (validation step) or KGE_OPT_SGD  */
  float lr;
  float clip_norm;            /* 5.0 in the reference (BaseModel.py:327)        */

  float* loss_out;            /* [1] batch loss (device)                        */
  float* loss_accum;          /* [1] += batch loss (device, nullable)           */
  float* pos_score_out;       /* [batch] (nullable)                             */
  float* neg_score_out;       /* [batch*K_eff] (nullable)                       */
  float* norm2_out;           /* [4] per-variable gradient norm^2 (nullable)    */
  int32_t* status;            /* device status word (nullable)                  */

  void* workspace;            /* zero-filled once at allocation (see the ABI rules) */
  uint64_t workspace_bytes;
  void* const* prof_events;   /* optional: 4 hipEvent_t recorded before K0, KS,
                                 KU and after KU (kernel timing; nullable)      */
  int32_t flags;              /* KGE_FLAG_*                                     */
  int32_t _pad;
  float* grad_out[4];         /* KGE_OPT_GRAD: dense [rows, cols] gradient per
                                 variable (order as norm2_out; row stride cols) */
  /* multi-GPU (KGE/sharded.py): ent / ent_aux hold shard_count all-gathered
   * shards of shard_rows rows each, entity id e at row
   * (e mod shard_count) * shard_rows + e div shard_count; ids (triples and
   * draws) stay global, in [0, global_entities). shard_count <= 1: identity. */
  int64_t shard_rows;
  int64_t global_entities;
  int32_t shard_count;
  int32_t _pad3;
  /* KGE_FLAG_PHASE_UPDATE (see the flags): */
  int64_t remote_rows_from;   /* entity rows >= this get their raw gradient in place (0: none) */
  const float* abort_flag;    /* device [1]; nonzero: the update pass does nothing (nullable) */
  /* KGE_FLAG_OWNER / KGE_FLAG_OWNER_MERGE (see the flags): */
  int32_t owner_world;        /* ranks, >= 1                                    */
  int32_t owner_rank;         /* this rank                                      */
  int64_t owner_batch;        /* positives per rank                             */
  int64_t owner_rows_from;    /* OWNER: rows of virtual positive v: h at owner_rows_from + 2v, t at + 1 */
  float* owner_records;       /* OWNER: out [batch, R]; OWNER_MERGE: in [owner_world, batch, R] */
  const float* owner_stats;   /* OWNER | PHASE_UPDATE: [batch, 4] in            */
  float* owner_stats_out;     /* OWNER_MERGE | PHASE_SCORE: [batch, 4] out      */
  int64_t owner_key_capacity; /* OWNER: key positions for the owned negatives (0: 5/4 of the
                                 expected owner_batch * K_eff, + 4096)          */
  float* owner_err;           /* OWNER: set to 2 when the owned negatives exceed the capacity
                                 (their keys are dropped: the caller voids the step; nullable) */
  /* ABI 7: the step's overflow flags without host-side launches (nullable):
   * OWNER_MERGE | PHASE_SCORE: owner_flags_in [2] (exchange flag, owner_err)
   *   -> owner_flags_out [3] = (in[0], in[1], in[0] + in[1]), then in zeroed
   *   for the next step (the caller all-reduces out: each slot counts the
   *   ranks that raised it, the last is the abort word);
   * OWNER | PHASE_UPDATE: owner_sticky [2] = max(owner_sticky, owner_flags_out[0..1])
   *   (the all-reduced flags, read before the abort check). */
  float* owner_flags_in;
  float* owner_flags_out;
  float* owner_sticky;
} kge_step_desc;

/*
 * Optimizer apply for one variable (BaseModel.py:327-328): clip_by_norm(g,
 * clip_norm) with the variable's global slice norm (TF-2.5 IndexedSlices:
 * duplicates not summed), then
 *   SGD : var -= lr * clip(g)                         (rows with g == 0 unchanged)
 *   ADAM: m = b1*m + (1-b1)*g; v = b2*v + (1-b2)*g^2  over ALL rows (keras
 *         sparse Adam decays every row), var -= lr_t * m / (sqrt(v) + eps),
 *         lr_t = lr * sqrt(1 - b2^t) / (1 - b1^t).
 * g is the duplicate-summed gradient written by a KGE_OPT_GRAD step (and
 * reduced across ranks by the caller, if any).
 */
typedef struct kge_apply_desc {
  int32_t optimizer;          /* KGE_OPT_SGD or KGE_OPT_ADAM                    */
  int32_t _pad;
  kge_table var;              /* rows to update (a whole table or one shard)   */
  const float* grad;          /* [var.rows, var.cols], row stride var.cols     */
  const float* norm2;         /* device [1]: ||g slices||^2 of this variable   */
  float lr;
  float clip_norm;
  float* m;                   /* ADAM slots [var.rows, var.cols], stride cols  */
  float* v;
  float beta_1, beta_2, epsilon;
  int32_t _pad2;
  int64_t iteration;          /* ADAM step t >= 1 (optimizer.iterations + 1)   */
  const float* abort_flag;    /* device [1]; nonzero: nothing is applied (nullable; the
                                 multi-GPU step's all-reduced exchange error flag) */
} kge_apply_desc;

/*
 * Batched filtered ranking: KGEModel.evaluate / get_rank (BaseModel.py:578-654)
 * for n evaluation triples at once. Query q ranks its true entity among all
 * E candidates of the corrupted side:
 *   rank[q] = 1 + #{ e : e not in filter(q), score(q, e) > score(q, true_q) }
 * (strict >, the reference's tensor_scatter_nd_update(-inf) filter :650 and
 * count :654; counted in int64 -- the reference's int16 overflows).
 * The caller prepares each query's rows in the model's op order (KGE/engine.py
 * rank_queries); the library scores the candidates:
 *   KGE_RANK_TRANS  translating: P(e) = e (NONE), e - (w.e) w (HYPER, w = qw),
 *                   clip(qw (e_p.e) + I e) (RANK1, e_p = cand_aux);
 *                   't': s(q0, P(e)), 'h': s(P(e) + q0, q1)
 *   KGE_RANK_ROT    RotatE complex rows: 't': s(q0, e), 'h': s(e o q0, q1)
 *   KGE_RANK_MUL    DistMult: 't': sum(q0 * e), 'h': sum((e * q0) * q1)
 *   KGE_RANK_DOT    sum(q0 * e) (RESCAL context rows)
 * s = the score kind (score.py:49-89). filt_beg / filt_end index query q's
 * filtered entities in filt_ent (ranges may be shared between queries; NULL =
 * no filter). Stream-ordered; rank_out and pos_score_out are outputs.
 */
enum { KGE_RANK_TRANS = 0, KGE_RANK_ROT = 1, KGE_RANK_MUL = 2, KGE_RANK_DOT = 3 };
/* KGE_RANK_FLAG_LANE_PASS: count with the lane-per-candidate pass even where
 * the register-tiled pass applies (TRANS without a projection, MUL, DOT).
 * Both give the same scores bit for bit, hence the same ranks (A-B / tests). */
enum { KGE_RANK_FLAG_LANE_PASS = 1 };
enum { KGE_RPROJ_NONE = 0, KGE_RPROJ_HYPER = 1, KGE_RPROJ_RANK1 = 2 };

typedef struct kge_rank_desc {
  int32_t abi_version;        /* KGE_ABI_VERSION                                */
  int32_t mode;               /* KGE_RANK_*                                     */
  int32_t proj;               /* KGE_RPROJ_* (KGE_RANK_TRANS only)              */
  int32_t corrupt_side;       /* KGE_SIDE_H or KGE_SIDE_T                       */
  kge_table cand;             /* candidate rows [E, cols] (TransR: the group's projected table) */
  kge_table cand_aux;         /* RANK1: ent_proj [E, cols]                      */
  int32_t dim;                /* floats per query / projected row (RotatE: 2d)  */
  int32_t clip;               /* RANK1: projected rows clipped to norm <= 1     */
  const float* q0;            /* [n, ldq] query rows                            */
  const float* q1;            /* [n, ldq] (h side / MUL; nullable otherwise)    */
  const float* qw;            /* [n, ldq] HYPER w / RANK1 r_p (nullable)        */
  int64_t ldq;
  const void* true_ids;       /* [n] the true entity of each query (idx_dtype)  */
  int32_t idx_dtype;          /* KGE_IDX_* of true_ids / filt_ent               */
  int32_t score_kind;         /* KGE_SCORE_*                                    */
  float score_p;              /* 1, 2 or +inf                                   */
  int32_t flags;              /* KGE_RANK_FLAG_* (0: default)                   */
  int64_t n;                  /* queries                                        */
  const int64_t* filt_beg;    /* [n] (nullable: no filter)                      */
  const int64_t* filt_end;    /* [n]                                            */
  const void* filt_ent;       /* filtered entity ids (idx_dtype)                */
  int64_t* rank_out;          /* [n]                                            */
  float* pos_score_out;       /* [n] the true triples' scores                   */
  int32_t* status;            /* device status word (nullable)                  */
  /* ABI 8: the filter as a bitmap (nullable). With a filter and filt_bits,
   * the library builds bit e of words [q * W, (q + 1) * W), W = ceil(E / 32),
   * for every entity e of query q's filter list and the count pass skips the
   * marked candidates, instead of rescoring the filtered entities in a pass
   * of its own (one workgroup per query: the thousands of known heads of a
   * popular (r, t) make it the slow tail of the h side). Same ranks bit for
   * bit. filt_bits_words >= n * W; contents on entry are ignored. */
  uint32_t* filt_bits;
  int64_t filt_bits_words;
} kge_rank_desc;

/* Batched filtered ranking (see kge_rank_desc). */
kge_status kge_rank(const kge_rank_desc* d, void* stream);

/*
 * Sparse SGD apply of one variable on listed rows (the owner-side update of
 * the multi-GPU step, KGE/sharded.py): for i < n,
 *   var[rows[i]] += -lr * clip_norm / max(sqrt(*norm2), clip_norm) * grad[i]
 * (keras SGD ResourceScatterAdd after clip_by_norm, BaseModel.py:327-328).
 * rows must be unique (the caller sums duplicates first); grad row stride
 * grad_ld floats.
 */
typedef struct kge_apply_rows_desc {
  kge_table var;              /* the owned rows (a shard)                       */
  const int64_t* rows;        /* [n] local row indices, unique                  */
  int64_t n;
  const float* grad;          /* [n, grad_ld] summed gradient rows              */
  int64_t grad_ld;
  const float* norm2;         /* device [1]: global ||g slices||^2 of the variable */
  float lr;
  float clip_norm;
} kge_apply_rows_desc;

kge_status kge_apply_rows(const kge_apply_rows_desc* d, void* stream);

/* Device-resident input stream (§8 f2; replaces data_utils.py:176-196's
 * tf.data shuffle -> repeat -> batch): batch rows [start, start + batch) of
 * the endless stream over a resident [n_rows, 3] triple array. Stream
 * position p is row pi_e(p mod n_rows) of epoch e = p div n_rows, so a batch
 * straddles epochs exactly like repeat().batch(). With shuffle = 0 pi_e is
 * the identity; otherwise it is a fresh permutation per epoch
 * (reshuffle_each_iteration): a 4-round balanced Feistel network on w-bit
 * values (w = the smallest even width >= 2 with 2^w >= n_rows, halves of
 * h = w/2 bits), round r of (L, R) -> (R, L ^ F_r(R)) with
 * F_r(R) = word 0 of Philox4x32-10(counter = (R, r, e lo, e hi),
 * key = (seed lo, seed hi)) masked to h bits, cycle-walked (re-applied while
 * the value is >= n_rows) so that it permutes [0, n_rows). No permutation is
 * stored: each output row computes its own source row. */
typedef struct kge_stream_desc {
  int32_t abi_version;        /* KGE_ABI_VERSION                                */
  int32_t idx_dtype;          /* KGE_IDX_* of triples and out                   */
  const void* triples;        /* [n_rows, 3], device-resident                   */
  int64_t n_rows;             /* > 0                                            */
  int64_t start;              /* stream position of the batch's first row, >= 0 */
  int64_t batch;              /* rows to produce, >= 0                          */
  uint64_t seed;
  int32_t shuffle;            /* 0: epoch order, 1: per-epoch permutation       */
  int32_t _pad;
  void* out;                  /* [batch, 3] idx_dtype                           */
} kge_stream_desc;

kge_status kge_stream_batch(const kge_stream_desc* d, void* stream);

/* The same stream with each epoch's permutation materialised once instead of
 * cycle-walked per row and per batch (the walk is a dependent chain of Philox
 * rounds: ~23 us per FB15k-237 batch on the row that walks longest).
 * kge_stream_permutation: perm[k] = pi_epoch(k) for k in [0, n_rows) (int32:
 * n_rows <= 2^31 - 1; d->shuffle must be 1; start / batch / out unused).
 * kge_stream_batch_perm: kge_stream_batch's output (shuffle = 1) from
 * perm_lo = pi_{epoch_lo} and perm_hi = pi_{epoch_lo + 1}: the batch's stream
 * positions must lie in those two epochs with epoch_lo = start div n_rows
 * (perm_hi may be NULL when the batch does not straddle). */
kge_status kge_stream_permutation(const kge_stream_desc* d, int64_t epoch, int32_t* perm, void* stream);
kge_status kge_stream_batch_perm(const kge_stream_desc* d, const int32_t* perm_lo, const int32_t* perm_hi,
                                 int64_t epoch_lo, void* stream);

/* Weight-histogram counts for the per-epoch logs (BaseModel.py's
 * tf.summary.histogram calls; TensorBoard's bucketing): for every x[i], i < n,
 * bucket k = clamp(floor((x[i] - lo) / width), 0, buckets - 1) evaluated in
 * double (a NaN counts in bucket 0), lo = lo_width[0], width = lo_width[1]
 * read on the device (the caller's device-side min / max: no host round trip);
 * counts[k] += 1 (uint64, the caller zero-fills or accumulates over chunks).
 * 1 <= buckets <= 256. Integer counts: exact whatever the order. */
kge_status kge_histogram(const float* x, int64_t n, const double* lo_width, int32_t buckets,
                         unsigned long long* counts, void* stream);

/* Device copy of n16 16-byte elements (n16 <= 2^40), src -> dst
 * (non-overlapping, both 16-byte aligned): one pass, each workgroup a
 * contiguous 16 KiB, non-temporal loads and stores, every load issued before
 * any store. A streaming copy: bench.py times it on a buffer far larger than
 * the Infinity Cache as the box's measured HBM copy peak, the second
 * denominator of the step's roofline fraction. */
kge_status kge_copy16(const void* src, void* dst, int64_t n16, void* stream);

/*
 * Multi-GPU sparse row exchange (KGE/sharded.py; the reference has no
 * counterpart, BaseModel.py:19-21 is single-device). Entity row e lives on
 * rank e mod G at local row e div G. A rank's step needs the rows of its
 * batch's ids; those another rank owns travel in FIXED-CAPACITY blocks of cap
 * rows per owner, so every collective has static sizes and nothing waits on
 * the host. A rank's extended entity table is [local_rows owned rows | G blocks
 * of cap fetched rows] (block `rank` holds own rows only with loopback).
 *
 * kge_exchange_plan: the step's id occurrences (positives' h and t, the
 * negatives) -> the same arrays in extended-table rows (pos_out, neg_out), and
 * per owner the distinct ids requested from it (req_ids [world, cap],
 * req_cnt [world]). Own ids map to their shard row directly (loopback: every
 * id through its owner's block -- a one-GPU rehearsal of the remote path). A
 * block past cap, or an id out of range, sets *err_flag: the caller's step is
 * then void (its update pass and every owner apply check the all-reduced flag).
 */
typedef struct kge_exchange_desc {
  int32_t abi_version;        /* KGE_ABI_VERSION                                */
  int32_t idx_dtype;          /* KGE_IDX_* of pos / neg / req_ids / outputs      */
  const void* pos;            /* [batch, 3] global ids                           */
  const void* neg;            /* [n_neg] global negative ids                     */
  int64_t batch, n_neg;
  int64_t n_entities;         /* global E (range check), < 2^32 - 1              */
  int32_t world, rank;
  int32_t loopback;           /* 1: own ids fetched through block `rank` as well */
  int32_t _pad;
  int64_t local_rows;         /* owned rows at the head of the extended table    */
  int64_t cap;                /* rows per owner block                            */
  unsigned long long* htab;   /* [hslots], zero-filled by the caller before each call */
  int64_t hslots;             /* power of two >= 2 (2 batch + n_neg)             */
  void* pos_out;              /* [batch, 3]: h, t remapped, r copied              */
  void* neg_out;              /* [n_neg] remapped                                */
  void* req_ids;              /* [world, cap] out                                */
  int32_t* req_cnt;           /* [world] out, zero-filled by the caller          */
  float* err_flag;            /* device [1]: set to 1 on an overflow / bad id (nullable) */
  int32_t* status;            /* KGE_ERANGE on an id out of range (nullable)     */
  void* zero_next;            /* ABI 7: zero-filled by this call (nullable; e.g. the other half of
                                 a double-buffered [htab | req_cnt] the NEXT call will use: no
                                 fill launch between steps). Must not overlap this call's arrays */
  int64_t zero_next_bytes;    /* multiple of 4                                   */
} kge_exchange_desc;

kge_status kge_exchange_plan(const kge_exchange_desc* d, void* stream);

/* Owner side of the exchange, over requested ids [world, cap] (cnt [world]),
 * or (POS) over a batch of remapped triples:
 *  KGE_XROWS_GATHER  rows[s][q] = shard row (ids[s][q] div world), every block
 *                    (source < 0) or block `source`;
 *  KGE_XROWS_SGD     shard row += -lr * clip / max(sqrt(*norm2), clip) * rows[s][q]
 *                    for block s = source (keras SGD after clip_by_norm,
 *                    BaseModel.py:327-328); one call per source, in rank order,
 *                    so a row several ranks touched gets their sums in that order;
 *  KGE_XROWS_ACCUM   acc row += rows[s][q] for block `source` (Adam: the dense
 *                    gradient of the shard, kge_apply follows);
 *  KGE_XROWS_POS     (ABI 7) rows[2i] = shard row ids[3i], rows[2i + 1] = shard
 *                    row ids[3i + 2] for i < cap: the positives' h / t rows of a
 *                    batch remapped by kge_exchange_plan (shard = the extended
 *                    table; cnt, world, rank, source unused).
 * SGD / ACCUM do nothing when abort_flag is set and *abort_flag != 0. */
enum { KGE_XROWS_GATHER = 0, KGE_XROWS_SGD = 1, KGE_XROWS_ACCUM = 2, KGE_XROWS_POS = 3 };

typedef struct kge_exchange_rows_desc {
  int32_t mode;               /* KGE_XROWS_*                                     */
  int32_t idx_dtype;          /* of ids                                          */
  kge_table shard;            /* owned rows (a view: one table's columns, ld = row stride) */
  const void* ids;            /* [world, cap]                                    */
  const int32_t* cnt;         /* [world]                                         */
  int32_t world, rank;
  int32_t source;             /* block (GATHER: -1 = every block)                */
  int32_t _pad;
  int64_t cap;
  float* rows;                /* [world, cap] rows, stride rows_ld (GATHER out, SGD / ACCUM in) */
  int64_t rows_ld;
  float* acc;                 /* ACCUM: [shard.rows, shard.cols], stride shard.cols */
  const float* norm2;         /* SGD: the variable's global slice norm^2         */
  float lr, clip_norm;
  const float* abort_flag;    /* nullable                                        */
  int32_t* status;            /* KGE_ERANGE on an id this rank does not own (nullable) */
} kge_exchange_rows_desc;

kge_status kge_exchange_rows(const kge_exchange_rows_desc* d, void* stream);

/* ABI version compiled into the library. */
int32_t kge_abi_version(void);

/* Thread-local message for the last non-OK status. */
const char* kge_last_error(void);

/* Workspace needed by kge_step for this descriptor (0 on error). */
uint64_t kge_step_workspace_bytes(const kge_step_desc* d);

/* Signature of the workspace layout this descriptor's plan uses (never 0;
 * 0 on error): a workspace stamped with another value must be re-zeroed
 * before this plan uses it (see the ABI rules above). */
uint32_t kge_step_plan_signature(const kge_step_desc* d);

/* Floats per owner record (KGE_FLAG_OWNER / KGE_FLAG_OWNER_MERGE) of this
 * descriptor's plan: 16 header floats + 3 gradient-accumulator images (0 on error). */
int64_t kge_owner_record_floats(const kge_step_desc* d);

/* One training / validation step (see kge_step_desc). */
kge_status kge_step(const kge_step_desc* d, void* stream);

/* Standalone negative sampling (ns_strategy.py:39-64, :94-132). */
kge_status kge_sample(const kge_sample_desc* d, void* stream);

/* Optimizer apply of one variable (see kge_apply_desc). */
kge_status kge_apply(const kge_apply_desc* d, void* stream);
/* n (<= 4) kge_apply calls in ONE launch -- a step's variables (ent / rel /
 * rel_aux / ent_aux) after a multi-GPU reduction or a grad-mode step. Same
 * result as the n calls in order; the variables must not overlap. */
kge_status kge_apply_many(const kge_apply_desc* d, int32_t n, void* stream);

/* Row constraints over a whole table (constraint.py:4-31, :70-99):
 * kind 0 = normalized_embeddings(p=2, value), 1 = clip_constraint(p=2, value).
 * Used by the models' _constraint_loss (TransE.py:171-172, TransR.py:207-209,
 * TransD.py:238-240) and _init_embeddings (TransE.py:108-109). */
kge_status kge_constrain_rows(kge_table t, int32_t kind, float value, void* stream);

#ifdef __cplusplus
}
#endif

#endif /* KGE_HIP_H */
