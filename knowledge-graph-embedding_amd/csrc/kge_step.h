// Kernel-argument structs shared by the step kernels and the C-ABI layer.
#pragma once

#include "kge_models.h"

namespace kge {

constexpr int kStepWaves = 8;      // waves per score workgroup
constexpr int kStepThreads = kStepWaves * KGE_WAVE;
constexpr int kUpdWaves = 4;       // waves per update workgroup (one destination row per wave)
constexpr int kUpdThreads = kUpdWaves * KGE_WAVE;
constexpr int kMaxWpp = 8;         // waves per positive, at most
constexpr int kMergeStride = 32;   // floats of per-positive merge state in the score kernel's LDS

// Control block at the head of the workspace. The caller zero-fills the
// workspace once when it allocates it; every kernel that uses a word puts it
// back to zero before the step ends (self-resetting tickets and counters).
struct StepCtl {
  uint32_t score_ticket;   // score workgroups done (the last one reduces the partials)
  uint32_t ovf_count;      // overflow-list appends of the running score kernel
  uint32_t ovf_len;        // overflow-list length for the update kernel (set by the last score workgroup)
  uint32_t pad0;
  float scale[4];          // -lr * clip / max(||g_v||, clip) per variable
  float loss;
  float pad1[7];
};

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
  float rel_reg;    // DistMult constraint_weight (0 = off): lambda * mean_i ||r_i||^2
  float lr, clip_norm;
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
  uint32_t* cnt;    // [E + R] entries per destination (zero between steps)
  uint32_t* list;   // [E + R, cap] codes per destination (arrival order)
  uint64_t* ovf;    // [B * (Keff + 3)] dest << 32 | code past a full list
  // KGE_OPT_GRAD outputs: dense [E, ent.cols] / [R, rel_gcols]
  float* gent;
  float* grel;
  // outputs
  float* loss_out;
  float* loss_accum;
  float* pos_score_out;
  float* neg_score_out;
  float* norm2_out;
  int32_t* status;
};

struct StepGeom {
  int vec, nc;
  int nWG, gridU;
  size_t lds_score;
};

kge_status launch_step_elementwise(const StepArgs& A, const StepGeom& G, int model, int sk,
                                   hipStream_t st, hipEvent_t const* ev);

__global__ void constrain_rows_kernel(float* t, int64_t rows, int32_t cols, int64_t ld, int kind,
                                      float value);

// Byte offsets of the score kernel's dynamic LDS carve (shared by host and
// device so the launch size always matches the kernel's view).
struct ScoreLds {
  int pos, ids, sR, sT, st, mrg, red, posg, misc, total;
};

__host__ __device__ inline int lds_align16(int x) { return (x + 15) & ~15; }

__host__ __device__ inline ScoreLds score_lds(int FL, int nP, int Keff) {
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
  L.total = o;
  return L;
}

}  // namespace kge
