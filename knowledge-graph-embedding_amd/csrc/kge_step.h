// Kernel-argument structs shared by the step kernels and the C-ABI layer.
#pragma once

#include "kge_models.h"

namespace kge {

constexpr int kStepWaves = 8;      // waves per workgroup, score and update kernels
constexpr int kStepThreads = kStepWaves * KGE_WAVE;
constexpr int kUCap = 4096;        // update kernel: LDS list capacity (entries)
constexpr int kMaxBuckets = 8192;  // score kernel: LDS bucket counters

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
  int32_t Kp;       // per-positive stride of the LDS score arrays (>= Keff + 1)
  int32_t slotmax;  // keys per score workgroup = nP * (Keff + 3)
  int32_t P;        // destination buckets (= entity/relation workgroups of the update kernel)
  int64_t bs;       // destinations per bucket; destinations = [0, E) entities, [E, E+R) relations
  int32_t snap_cols, gcols, rel_gcols;
  // workspace
  float2* coef;     // [B*Keff] (alpha, reduced value) per negative
  float* snap;      // [B, NSNAP, snap_cols] positive contexts
  float* gpos;      // [B, 3, gcols] positive h / r / t row gradients
  float* part;      // [nWG, 8] loss, norm^2 x4 partials
  uint64_t* sorted; // [nWG, slotmax] keys dest << 32 | code, grouped by bucket
  uint32_t* bmap;   // [P, nWG] start << 16 | count of bucket b in workgroup w
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
  size_t lds_score, lds_update;
};

kge_status launch_step_elementwise(const StepArgs& A, const StepGeom& G, int model, int sk,
                                   hipStream_t st, hipEvent_t const* ev);

__global__ void constrain_rows_kernel(float* t, int64_t rows, int32_t cols, int64_t ld, int kind,
                                      float value);

}  // namespace kge

namespace kge {

// Byte offsets of the score kernel's dynamic LDS carve (shared by host and
// device so the launch size always matches the kernel's view).
struct ScoreLds {
  int red, sR, sti, ssc, sM, ids, bkt, misc, sw, pos, cnt, total;
};

__host__ __device__ inline int lds_align16(int x) { return (x + 15) & ~15; }

__host__ __device__ inline ScoreLds score_lds(int FL, int nP, int Kp, int Keff, int slotmax, int P) {
  ScoreLds L;
  int o = 0;
  L.red = o;  o += lds_align16(kStepWaves * 3 * FL * 4);
  L.sR = o;   o += lds_align16(nP * Kp * 4);
  L.sti = o;  o += lds_align16(nP * Kp * 4);
  L.ssc = o;  o += lds_align16(nP * Kp * 4);
  L.sM = o;   o += lds_align16(nP * Kp * 4);
  L.ids = o;  o += lds_align16(nP * Keff * 4);
  L.bkt = o;  o += lds_align16(slotmax * 4);
  L.misc = o; o += lds_align16(kStepWaves * 8 * 4);
  L.sw = o;   o += lds_align16(16 * 4);
  L.pos = o;  o += lds_align16(nP * 3 * 8);
  L.cnt = o;  o += lds_align16((P + 1) * 4);
  L.total = o;
  return L;
}

}  // namespace kge
