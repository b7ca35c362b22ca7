// Kernel-argument structs shared by the step kernels and the C-ABI layer.
#pragma once

#include "kge_models.h"

namespace kge {

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
  int32_t nP, nWG, Kpad, idpad, sortpad, slotmax, P, ucap;
  int64_t bs;
  int32_t snap_cols, gcols, rel_gcols;
  // workspace
  int32_t* ids;
  float2* coef;
  float* snap;
  float* gpos;
  float* part;
  uint64_t* sorted;
  int32_t* starts;
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
