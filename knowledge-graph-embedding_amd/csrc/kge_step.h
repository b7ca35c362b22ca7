// Kernel-argument structs shared by the step kernels and the C-ABI layer.
#pragma once
#include <type_traits>

#include "kge_models.h"

namespace kge {

#ifndef KGE_STEP_WAVES
#define KGE_STEP_WAVES 8           // waves per score workgroup (tuning knob)
#endif
constexpr int kStepWaves = KGE_STEP_WAVES;
constexpr int kStepThreads = kStepWaves * KGE_WAVE;
constexpr int kUpdWaves = 4;       // waves per update workgroup (one destination row per wave)
constexpr int kUpdThreads = kUpdWaves * KGE_WAVE;
#ifndef KGE_UPD_KR
#define KGE_UPD_KR 4               // compact update launch: key positions per wave (tuning knob)
#endif
constexpr int kUpdKeysPerWave = KGE_UPD_KR;
constexpr int kMaxWpp = kStepWaves > 8 ? kStepWaves : 8;   // waves per positive, at most
#ifndef KGE_SLOTS_PER_WAVE
#define KGE_SLOTS_PER_WAVE 64      // score kernel: negative slots a wave streams, at most (tuning knob)
#endif
#ifndef KGE_SCORE_WPE
#define KGE_SCORE_WPE 4            // score kernel: amdgpu_waves_per_eu (tuning knob)
#endif
#ifndef KGE_SCORE_WPE_WIDE
#define KGE_SCORE_WPE_WIDE 2       // ... for rows of two or more fragment chunks (register room, no spills)
#endif
constexpr int kMergeStride = kMaxWpp + 24;   // floats of per-positive merge state in the score kernel's LDS
constexpr int kSortMax = 1024;     // update kernel: longest destination list sorted in LDS (per wave)
// owner merge update: destinations with more than kLongN (and at most
// kLongMax) keys go to long_rows_kernel (kLongWGs workgroups, kLongU rows in flight)
#ifndef KGE_LONG_N
#define KGE_LONG_N 64   // (tuning knob)
#endif
#ifndef KGE_LONG_WGS
#define KGE_LONG_WGS 64   // (tuning knob)
#endif
constexpr int kLongN = KGE_LONG_N, kLongMax = 4096, kLongWGs = KGE_LONG_WGS, kLongU = 16, kLongCPT = 4;   // (rows <= 1024 floats)

// Control block at the head of the workspace. The caller zero-fills the
// workspace once when it allocates it; every kernel that uses a word puts it
// back to zero before the step ends (self-resetting tickets and counters).
struct StepCtl {
  uint32_t score_ticket;   // score workgroups done (the last one reduces the partials)
  uint32_t ovf_count;      // overflow-list appends of the running score kernel
  uint32_t ovf_len;        // overflow-list length for the update kernel (set by the last score workgroup)
  uint32_t upd_ticket;     // dense-gradient update workgroups done (entity norm^2)
  float scale[4];          // -lr * clip / max(||g_v||, clip) per variable
  float loss;
  uint32_t rel_ticket;     // relation-matrix gradient workgroups done (rel norm^2)
  uint32_t reg_ticket;     // regulariser-loss workgroups done
  float dn2[4];            // norm^2 of the dense (duplicate-summed) gradient per variable
  float reg_r2;            // RESCAL train step: sum_r ||R_r||_F^2 (rel_dr partials)
  uint32_t plan_sig;       // signature of the plan that last used the workspace (0: fresh)
  uint32_t score_pending;  // split step: the plan signature, set by a PHASE_SCORE pass's last
                           // workgroup and consumed by the next PHASE_UPDATE call (phase gate)
  uint32_t own_count;      // owner score pass: key positions taken (per-workgroup blocks)
  uint32_t own_len;        // ... handed to the coefficient / update passes by the last workgroup
  uint32_t lng_count;      // merge update: long destinations deferred to long_rows_kernel (reset by the merge)
  uint32_t pad2;
};

// Workspace plan guard (include/kge_hip.h, "workspace"). Every kernel of a
// step that writes a table or a caller-visible output calls this first. A
// fresh (zero-filled) workspace is claimed by the first guarded kernel; one
// last used by a different plan -- its counters and lists laid out for other
// sizes -- is refused by every guarded kernel of the step, so nothing is
// written: the status word gets KGE_EWORKSPACE and the loss NaN. The value
// only ever goes 0 -> sig, so every workgroup of every kernel of a step takes
// the same decision. The word is read with a plain uniform load at kernel
// entry (a scalar load: a launch of 10^5 waves must not queue 10^5 requests on
// the one L2 channel that holds it -- an atomic load there cost C2-50M's
// update kernel 120 us); it is written only with a vector store.
__device__ __noinline__ bool ws_refused_slow(StepCtl* ctl, uint32_t s, uint32_t sig, int32_t* status,
                                             float* loss_out) {
  const bool lead = blockIdx.x == 0 && blockIdx.y == 0 && threadIdx.x == 0;
  if (s == 0u) {
    if (lead) __hip_atomic_store(&ctl->plan_sig, sig, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return false;
  }
  if (lead) {
    set_status(status, KGE_EWORKSPACE);
    if (loss_out) loss_out[0] = __builtin_nanf("");
  }
  return true;
}
// A plan signature no plan has (make_plan maps it away): the phase gate
// stamps it when a PHASE_UPDATE call finds no pending score pass of its plan,
// so every guarded kernel refuses the workspace until the caller zeroes it.
constexpr uint32_t kPoisonedSig = 0xFFFFFFFFu;
__device__ __forceinline__ bool ws_refused(StepCtl* ctl, uint32_t sig, int32_t* status, float* loss_out) {
  const uint32_t s = *reinterpret_cast<const uint32_t*>(&ctl->plan_sig);
  // the common case (the workspace is this plan's) is one scalar compare; the
  // claim / refusal path is out of line so it costs the kernel no registers
  if (__builtin_expect(s == sig, 1)) return false;
  return ws_refused_slow(ctl, s, sig, status, loss_out);
}

// sets the thread-local message kge_last_error() returns (kge_abi.hip)
void kge_set_error(const char* msg);

// Optimizer apply over a whole table (kge_apply, and the dense-gradient
// steps' in-step SGD): clip_by_norm with the variable's norm^2, then SGD or
// keras Adam (kge_hip.h kge_apply_desc). Guarded when launched by a step
// (ctl != nullptr).
struct ApplyArgs {
  float* w; int64_t rows; int32_t cols; int64_t ld;
  const float* g; const float* norm2;
  float lr, clip;
  int adam; float* m; float* v; float b1, b2, eps, lr_t;
  StepCtl* ctl; uint32_t sig; int32_t* status;
  const float* abort = nullptr;   // nonzero *abort: nothing applied
};
void launch_apply(const ApplyArgs& a, hipStream_t st);
// up to kMaxApply variables in one launch (blocks split between them by size)
constexpr int kMaxApply = 4;
void launch_apply_many(const ApplyArgs* a, int n, hipStream_t st);

// Everything a step kernel needs, passed by value (kernarg segment).
struct StepArgs {
  TabView ent, rel, ent_aux, rel_aux;
  const void* pos;
  bool i64;
  bool train;
  bool given;
  bool pw;          // LpDistancePow
  bool rel_half;    // RotatE: relation row is the phase half-row
  bool grad_mode;   // KGE_OPT_GRAD: write summed gradients, no update
  bool zero_untouched;   // grad mode, every row visited: untouched rows get a zero gradient row
                         // (the gradient outputs need no zero-fill)
  bool fuse_norm;   // _constraint_loss renormalisation fused into the step (SGD path)
  int64_t B;
  int32_t Keff;     // negatives per positive actually produced
  int32_t Kside;    // draws per side
  int32_t side_mode;
  SamplerView smp;
  void* neg_user;   // user-visible negative ids (idx dtype), nullable
  int32_t loss_kind;
  float margin, temperature;
  float inv_b;      // 1 / (B * batch_scale)
  float inv_bk;     // 1 / (B * Keff * batch_scale)
  float limit;
  float p;          // LpDistance p (SK_PGEN)
  float rel_reg;    // DistMult constraint_weight (0 = off): lambda * mean_i ||r_i||^2
  float lr, clip_norm;
  // dense-gradient variables (a full-table regulariser term makes TF's
  // gradient dense: RESCAL.py:190-198): the update kernel visits every row,
  // adds dense_ent * row, writes the summed gradient to gent and reduces its
  // norm^2 (clip_by_norm of the dense tensor); the apply pass follows
  bool dense;
  bool rel_dests;   // relation rows are update-kernel destinations (false: RESCAL's dR pass)
  float dense_ent;  // d(regulariser)/d(row) coefficient of every entity row
  // positives' own entity-row gradients: row h at gpe + i*gpe_stride, t at + gpe_toff
  float* gpe;
  int32_t gpe_stride, gpe_toff;
  float* upart;     // [gridU] update-kernel norm^2 partials (dense mode)
  float* gneg;      // materialised family: [B << kshift, ent.cols] negatives' entity-row gradients
  // compact update launch (tables much larger than a step's keys): the score
  // pass writes, for every key position, (destination, code) when the key
  // is its destination's first (list position 0), else code ~0 -- no
  // append counter; the update launch (one wave per key position) visits
  // only those leaders' rows (untouched rows are not read or written)
  bool compact;
  uint4* leaders;   // per key position: (destination, code or ~0, hash slot, 0)
  // compact launches key the destination lists by a hash slot instead of the
  // destination row (the E-sized counter / list arrays of a 50M-row table
  // would sit in HBM; the 2T-slot table stays in L2 / MALL): per slot
  // (destination + 1) << 32 | count, 0 = empty, linear probing; the lists
  // are [slot, cap], the leader's update wave empties its slot
  unsigned long long* htab;
  uint32_t hshift;  // slot = (dest * 2654435761) >> hshift (32 - log2 slots)
  uint32_t hmask;
  uint32_t npos3;    // 3 B: key positions [0, 3B) are the positives' (3 i + part), then B * Keff negatives
  uint32_t nkeys;    // B * (Keff + 3) key positions
  // multi-table update passes (TransH / TransD): the aux-table pass runs
  // first over the same destination lists and leaves the counters for the
  // main pass; scale[] slots of the pass's entity / relation variable
  bool keep_cnt = false;
  bool rel_only = false;   // visit the relation destinations only (TransH rel_hyper pass)
  // owner merge update (compact): the relation rows are summed by
  // rel_seg_kernel (a workgroup per relation, the positives' rows in
  // ascending order) instead of by one update wave per relation -- a
  // Zipf-hot relation's list (~250 keys at C5) was a serial chain there that
  // nothing else overlapped; the update kernel only empties their list slots
  bool rel_seg = false;
  // rel_seg's relation segments (launch_rel_rank over the batch first):
  // positives in relation order (stable), first position and count per relation
  int32_t* rs_sorted = nullptr;
  int32_t* rs_srel = nullptr;
  int32_t* rs_beg = nullptr;
  // merge update (KGE_FLAG_OWNER_MERGE | PHASE_UPDATE, SGD): every key is a
  // positive's own row gradient; a destination with more than kLongN of them
  // (a Zipf-hot head or tail) is handed to long_rows_kernel (lng[], up to
  // lng_cap) instead of being summed by one wave two rows at a time
  bool pos_only = false;
  uint4* lng = nullptr;
  uint32_t lng_cap = 0;
  // merge update as a segmented sum (launch_merge_segsum, kge_step.hip): the
  // positives' 3 B keys (destination, code) sorted once, summed in chunks of
  // 4-16 keys by many waves (a Zipf-hot destination is split over
  // chunks, no serial chain), chunk-spanning runs combined in chunk order.
  // Replaces the update kernel, rel_rank, rel_seg and long_rows of the merge's
  // update pass; the merge files no keys
  bool seg_merge = false;
  unsigned long long* seg_raw = nullptr;    // [3 B] the merge's keys (destination << 32 | code), positive order
  unsigned long long* seg_keys = nullptr;   // [3 B] the same, sorted
  float* seg_part = nullptr;                // [2 * chunks, gcols] head / tail partial rows
  int32_t seg_npad = 0;                     // (a power of two >= 3 B, <= kSegMaxKeys: the key staging bound)
  // entity ids -> table rows: n_ent global ids; rG > 1: the table is G
  // all-gathered shards of rEs rows, id e at (e mod rG) * rEs + e div rG
  int64_t n_ent = 0;
  int32_t rG = 1;
  int64_t rEs = 0;
  int32_t sc_ent_idx = 0, sc_rel_idx = 1;
  // geometry
  int32_t wpp;      // waves per positive (1, 2, 4, 8)
  int32_t nP;       // positives per score workgroup = kStepWaves / wpp
  int32_t SW;       // negative slots per wave
  int32_t nWG;      // score workgroups
  int32_t cap;      // destination list capacity (entries per destination)
  int32_t snap_cols, gcols, rel_gcols;
  uint32_t nkeyneg; // B << kshift: codes below are negatives (i << kshift | j), above positive rows (+4i+c)
  int32_t kshift;   // log2 of the slot stride (next power of two >= Keff)
  // workspace
  StepCtl* ctl;
  float2* coef;     // [B*Keff] (alpha, reduced value) per negative
  float* snap;      // [B, NSNAP, snap_cols] positive contexts
  float* gpos;      // [B, 3, gcols] positive h / r / t row gradients
  float* part;      // [nWG, 8] loss, norm^2 x4 partials
  uint32_t* cnt;    // [E + R] entries per destination (zero between steps; not compact)
  uint32_t* list;   // [E + R, cap] codes per destination (arrival order; compact: [slots, cap])
  uint64_t* ovf;    // [B * (Keff + 3)] dest << 32 | code past a full list
  // KGE_OPT_GRAD outputs: dense [E, ent.cols] / [R, rel_gcols]
  float* gent;
  float* grel;
  float* gent_aux;  // TransD ent_proj (grad_out[3])
  float* grel_aux;  // rel_hyper / rel_proj (grad_out[2])
  // outputs
  float* loss_out;
  float* loss_accum;
  float* pos_score_out;
  float* neg_score_out;
  float* norm2_out;
  int32_t* status;
  uint32_t sig;     // plan signature (ws_refused)
  // split step (KGE_FLAG_PHASE_*, the multi-GPU sparse exchange)
  bool run_score = true, run_update = true;
  bool mark_pending = false;   // PHASE_SCORE: the last score workgroup sets ctl->score_pending = sig
  bool scale_from_norm2 = false;   // update pass: clip scales from norm2_out (all-reduced by the caller)
  bool rel_grad = false;           // update pass: relation rows' raw gradients -> grel (no update)
  int64_t remote_from = INT64_MAX; // entity rows >= this: raw gradient written in place of the row
  const float* abort_flag = nullptr;   // update pass does nothing when *abort_flag != 0
  // owner-side scoring (KGE_FLAG_OWNER / KGE_FLAG_OWNER_MERGE; KGE/sharded.py
  // "owner" mode). The owner pass scores every rank's positives (a virtual
  // batch of own_G x own_Bq, positive v = q own_Bq + i of rank q) against the
  // negatives this rank owns (entity e on rank e mod own_G, local row e div
  // own_G), and leaves per positive one record: its partial softmax state,
  // loss / norm partials and the h / r / t gradient accumulators. The merge
  // pass (the positive's rank) combines the records of every owner.
  int32_t own_G = 1, own_g = 0;
  int64_t own_Bq = 0;
  int32_t own_planes = 1;           // sampler planes a rank's step draws from
  int64_t own_rows_from = 0;        // owner: virtual positive v's h / t rows at own_rows_from + 2 v (+ 1)
  float* own_rec = nullptr;         // owner: [B, rec_cols] out; merge: [own_G, B, rec_cols] in (source-major)
  int32_t rec_cols = 0;             // 16 header floats + 3 accumulator images of FL floats
  const float* own_stats = nullptr; // owner update: [B, 4] (Ms, 1/Z, positive score, -) per virtual positive
  float* own_stats_out = nullptr;   // merge: [B, 4] out
  uint32_t* own_codes = nullptr;    // owner: [own_cap] destination code per key position (~0: padding)
  uint32_t own_cap = 0;             // owner: key positions available (grid of the update launch)
  float* own_err = nullptr;         // owner: set to 2 when the owned keys exceed own_cap
  float* own_flags_in = nullptr;    // merge: the step's [exchange, owner] flags (read, then zeroed)
  float* own_flags_out = nullptr;   // merge: out [3]; owner update: the all-reduced copy (read)
  float* own_sticky = nullptr;      // owner update: [2] running max of the all-reduced flags
  bool own_keys = false;            // update kernel: compact key positions [0, ctl->own_len)
};
// accumulator images per owner record: M::REC_IMG when the model declares it
// (TransE: h, t), else 3 (h, r, t)
template <class M, class = void> struct rec_img { static constexpr int n = 3; };
template <class M> struct rec_img<M, std::void_t<decltype(M::REC_IMG)>> { static constexpr int n = M::REC_IMG; };
constexpr int kRecHead = 16;        // owner record: Ms, Z, loss part, hinge / logistic weight, norm^2 x4, -

struct StepGeom {
  int vec, nc;
  int nWG, gridU;
  size_t lds_score;
};

kge_status launch_step_elementwise(const StepArgs& A, const StepGeom& G, int model, int sk,
                                   hipStream_t st, hipEvent_t const* ev);
// per-family instances (kge_step_<family>.hip)
kge_status launch_transe(const StepArgs& A, const StepGeom& G, int sk, hipStream_t st, hipEvent_t const* ev);
kge_status launch_distmult(const StepArgs& A, const StepGeom& G, hipStream_t st, hipEvent_t const* ev);
kge_status launch_rotate(const StepArgs& A, const StepGeom& G, int sk, hipStream_t st, hipEvent_t const* ev);

// ---- relation-matrix models (kge_rel.hip): RESCAL's MFMA passes
struct RelArgs {
  TabView ent, rel;          // rel rows are d x d matrices (ld >= d*d)
  const void* pos;
  bool i64;
  int64_t B;
  int32_t d;
  int32_t* sorted;           // [B] positives in relation order (stable)
  int32_t* srel;             // [B] relation of sorted position p
  int32_t* rel_beg;          // [R] first sorted position of relation r
  int32_t* rel_cnt;          // [R] positives of relation r
  float* snap;               // [B, 2, d] u = R^T h, v = R t
  const float* gpos;         // [B, 3, gcols] A, b, B (score kernel)
  int32_t gcols;
  float* gproj;              // [B, 2, d] g_h = R A, g_t = R^T B
  float* grel;               // [R, d*d] dense relation gradient
  float* rpart;              // [R * ceil(d/16)] norm^2 partials
  float dense_rel;           // 2 lambda / R (0: no regulariser)
  StepCtl* ctl;
  float* norm2_out;
  int32_t* status;
  uint32_t sig;              // plan signature (ws_refused)
  float* loss_out;
  bool lazy_absent;          // SGD step: absent relations' dense gradient re-derived by the apply (not stored)
};
void launch_rel_rank(const RelArgs& R, hipStream_t st);
void launch_histogram(const float* x, int64_t n, const double* lw, int bc, unsigned long long* counts,
                      hipStream_t st);   // kge_stream.hip (kge_histogram)
void launch_copy16(const void* src, void* dst, int64_t n16, hipStream_t st);   // kge_stream.hip (kge_copy16)
constexpr int kSegMaxKeys = 8192;
// the owner merge's update pass (StepArgs::seg_merge): phase gate + relation
// gradient zero-fill + key sort, chunk sums, combine (kge_step.hip)
void launch_merge_segsum(const StepArgs& A, hipStream_t st);
void launch_rel_post(const RelArgs& R, hipStream_t st);     // dR (+ dense term, norm^2 partials)
// train step tail: both passes' norms + the loss term, then both SGD applies in one launch
void launch_rescal_norms(const RelArgs& P, const float* upart, int nu, float lam, float lr, float clip,
                         float* loss_accum, hipStream_t st);
bool rescal_apply_fused_ok(const RelArgs& P, const TabView& ent, const float* gent);
void launch_rescal_apply(const RelArgs& P, const TabView& ent, const float* gent, float lr, float clip,
                         hipStream_t st);
// lambda * (mean_e ||e||^2 + mean_r ||R_r||_F^2) added to the step loss (RESCAL.py:190-198)
void launch_reg_loss(const TabView& ent, const TabView& rel, float lam, float* part, StepCtl* ctl,
                     float* loss_out, float* loss_accum, uint32_t sig, int32_t* status, hipStream_t st);
constexpr int kRegWGs = 1024;   // regulariser sweep workgroups (256-float chunks dealt round-robin)

// first sorted position in [lo, hi) whose relation is >= r (srel ascending)
__device__ __forceinline__ int64_t rel_lower(const int32_t* srel, int64_t lo, int64_t hi, int64_t r) {
  while (lo < hi) {
    const int64_t m = (lo + hi) >> 1;
    if ((int64_t)srel[m] < r) lo = m + 1; else hi = m;
  }
  return lo;
}

// ---- TransR (kge_transr.hip): one workgroup per positive, three MFMA products
struct TrArgs {
  TabView proj;      // rel_proj [R, d * k] (M_r row-major [d][k])
  int32_t d, k;      // entity / relation embedding sizes
  bool clip;         // constraint: projected vectors clipped to norm <= 1 (TransR.py:187-189)
  float* dmpart;     // [B, d * k] per-positive dM partials (summed per relation by the apply pass)
  const int32_t* sorted;
  const int32_t* rel_beg;
  const int32_t* rel_cnt;
  float* gproj_out;  // KGE_OPT_GRAD: dense [R, d * k] rel_proj gradient (else null)
};
constexpr int kTrWaves = 8;
constexpr int kTrThreads = kTrWaves * KGE_WAVE;
constexpr int kTrMaxSlots = 72;   // K + 1 slots over 8 waves, 9 per wave in registers
constexpr int kTrMaxDim = 256;    // d, k (MFMA k-steps held in registers)
// GEMM1 / GEMM2 inner dimensions run over NC whole 16-column chunks, a
// compile-time count (straight-line MFMA code, B columns in 4*NC registers):
// the smallest of 4, 8, 13, 16 covering max(d, k)
__host__ __device__ inline int tr_nc(int d, int k) {
  const int c = ((d > k ? d : k) + 15) / 16;
  return c <= 4 ? 4 : c <= 8 ? 8 : c <= 13 ? 13 : 16;
}
// LDS carve of the TransR kernel (floats): X [NR16][LX] | P [NR16][LP], later
// S [SR16][LP] over both; then per-row / per-slot scalars and partials.
// Rows are W = 16 NC floats (zero past d / k) plus 4: the stride mod 32 banks
// is 4 or 20, so the 8 rows served together by a ds_read_b128 operand fetch
// hit disjoint bank quads.
struct TrLds {
  int NC, W, LX, LP, NR16, SR16;
  int pn, xx, xh, xt, sS, sR, sT, sA, rp, ids, misc, total_floats;
};
__host__ __device__ inline TrLds tr_lds(int d, int k, int K) {
  TrLds L;
  L.NC = tr_nc(d, k);
  L.W = 16 * L.NC;
  L.LX = L.W + 4;
  L.LP = L.W + 4;
  L.NR16 = (K + 2 + 15) & ~15;
  L.SR16 = (2 * K + 4 + 15) & ~15;
  int o = L.NR16 * (L.LX + L.LP);
  if (L.SR16 * L.LP > o) o = L.SR16 * L.LP;
  L.pn = o; o += L.NR16;
  L.xx = o; o += L.NR16;
  L.xh = o; o += L.NR16;
  L.xt = o; o += L.NR16;
  L.sS = o; o += (K + 4) & ~3;
  L.sR = o; o += (K + 4) & ~3;
  L.sT = o; o += (K + 4) & ~3;
  L.sA = o; o += (K + 4) & ~3;
  L.rp = o; o += kTrWaves * L.LP;
  L.ids = o; o += (K + 3) & ~3;
  L.misc = o; o += 64;
  L.total_floats = o;
  return L;
}
kge_status launch_step_transr(const StepArgs& A, const StepGeom& G, const TrArgs& T, const RelArgs& P, int sk,
                              hipStream_t st, hipEvent_t const* ev);
kge_status launch_step_rescal(const StepArgs& A, const StepGeom& G, const RelArgs& P, float lam, float* regpart,
                              hipStream_t st, hipEvent_t const* ev);

// ---- batched filtered ranking (kge_rank.hip): BaseModel.py:578-654
constexpr int kRankQ = 8;          // queries per count workgroup
constexpr int kRankThreads = 256;  // candidates per count workgroup

struct RankArgs {
  const float* cand; int64_t cand_ld; int64_t E;
  const float* caux; int64_t caux_ld;    // TransD ent_proj
  int32_t dim;                            // floats per query row / projected row
  int32_t ecols;                          // floats per candidate row (RotatE 2d; TransD d)
  int32_t kmin;                           // TransD identity block
  bool clip;                              // TransD: projected rows clipped to norm <= 1
  bool hside;                             // corrupt_side 'h'
  bool pw;                                // LpDistancePow
  bool lane_pass;                         // KGE_RANK_FLAG_LANE_PASS
  float p;                                // LpDistance p (SK_PGEN)
  const float* q0; const float* q1; const float* qw; int64_t ldq;
  const void* true_ids; bool i64; int64_t n;
  const int64_t* fbeg; const int64_t* fend; const void* fent;
  const uint32_t* fbits; int64_t fw;       // filter bitmap (ABI 8): query q's words at q * fw, or null
  unsigned long long* rank;
  float* pos;
  int32_t* status;
};

kge_status launch_rank(const RankArgs& A, int mode, int proj, int sk, hipStream_t st);
void launch_stream(const void* tri, bool i64, int64_t n, int64_t start, int64_t batch, uint64_t seed, int shuffle,
                   void* out, hipStream_t st);
void launch_stream_perm(int64_t n, uint64_t seed, int64_t epoch, int32_t* perm, hipStream_t st);
void launch_stream_gather(const void* tri, bool i64, int64_t n, int64_t start, int64_t batch, const int32_t* plo,
                          const int32_t* phi, int64_t e0, void* out, hipStream_t st);

__global__ void constrain_rows_kernel(float* t, int64_t rows, int32_t cols, int64_t ld, int kind,
                                      float value, StepCtl* ctl, uint32_t sig, int32_t* status,
                                      float* t2, int64_t rows2, int32_t cols2, int64_t ld2);

// Byte offsets of the score kernel's dynamic LDS carve (shared by host and
// device so the launch size always matches the kernel's view).
struct ScoreLds {
  int pos, ids, sR, sT, st, mrg, red, posg, misc, jmap, total;
};

__host__ __device__ inline int lds_align16(int x) { return (x + 15) & ~15; }

__host__ __device__ inline ScoreLds score_lds(int FL, int nP, int Keff, bool own = false) {
  ScoreLds L;
  int o = 0;
  L.pos = o;  o += lds_align16(nP * 3 * 8);
  L.ids = o;  o += lds_align16(nP * Keff * 4);
  L.sR = o;   o += lds_align16(nP * Keff * 4);
  L.sT = o;   o += lds_align16(nP * Keff * 4);
  L.st = o;   o += lds_align16(kStepWaves * 8 * 4);
  L.mrg = o;  o += lds_align16(nP * kMergeStride * 4);
  L.red = o;  o += lds_align16(kStepWaves * 3 * FL * 4);
  L.posg = o; o += lds_align16(nP * 3 * FL * 4);
  L.misc = o; o += lds_align16(kStepWaves * 8 * 4);
  L.jmap = o; o += lds_align16(own ? 2 * nP * Keff * 4 : 0);   // owner pass: compacted slot -> slot | -> row
  L.total = o;
  return L;
}

}  // namespace kge
