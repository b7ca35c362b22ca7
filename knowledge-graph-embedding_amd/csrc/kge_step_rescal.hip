// RESCAL instances of the fused step kernels (RESCAL.py:140-200); the
// relation-matrix MFMA passes live in kge_rel.hip.
#include "kge_step_impl.h"

namespace kge {

#ifndef KGE_ONLY_ONE
// Fixed-order sum of n per-workgroup norm^2 partials into ctl->dn2[slot]
// (and norm2_out[slot]): one workgroup, launched right after the producer.
// Train steps also finish the regulariser loss here: part[n + w] holds the
// update workgroups' ||e||^2 partials, ctl->reg_r2 the relation term summed
// by rel_dr_norm_kernel (lam = 0: no loss term).
__global__ __launch_bounds__(256) void partials_norm_kernel(const float* part, int n, StepCtl* ctl, int slot,
                                                            float* norm2_out, float lam, float inv_e, float inv_r,
                                                            float* loss_out, float* loss_accum, uint32_t sig,
                                                            int32_t* status) {
  if (ws_refused(ctl, sig, status, loss_out)) return;
  __shared__ float s_n2[4], s_e2[4];
  const int lane = lane_id(), wv = wave_id();
  float s = 0.f, e = 0.f;
  for (int w = threadIdx.x; w < n; w += blockDim.x) {
    s += part[w];
    if (lam != 0.f) e += part[n + w];
  }
  s = wave_sum(s);
  e = wave_sum(e);
  if (lane == 0) { s_n2[wv] = s; s_e2[wv] = e; }
  __syncthreads();
  if (threadIdx.x == 0) {
    const float t = s_n2[0] + s_n2[1] + s_n2[2] + s_n2[3];
    ctl->dn2[slot] = t;
    if (norm2_out) norm2_out[slot] = t;
    if (lam != 0.f) {   // lambda * (mean_e ||e||^2 + mean_r ||R_r||_F^2), RESCAL.py:190-198
      const float add = lam * ((s_e2[0] + s_e2[1] + s_e2[2] + s_e2[3]) * inv_e + ctl->reg_r2 * inv_r);
      loss_out[0] += add;
      if (loss_accum) loss_accum[0] += add;
    }
  }
}

// RESCAL: relation rank -> score (its waves form u = R^T h, v = R t, stream
// the negatives as dot products against them, then g_h = R A, g_t = R^T B)
// -> regulariser loss -> dR pass -> update kernel (dense entity gradient)
template <int VEC, int NC>
static kge_status rescal_vn(const StepArgs& A, const StepGeom& G, const RelArgs& P, float lam, float* regpart,
                            hipStream_t st, hipEvent_t const* ev) {
  if (A.train) launch_rel_rank(P, st);   // (the dR pass's relation groups)
  launch_score<Rescal, VEC, NC, SK_DOT>(A, G, st);
  // train steps fold the regulariser loss into passes that read every row
  // anyway (rel_dr: each R_r; the dense update: each entity row)
  if (lam != 0.f && !A.train) launch_reg_loss(A.ent, A.rel, lam, regpart, A.ctl, A.loss_out, A.loss_accum, A.sig, A.status, st);
  if (ev) (void)hipEventRecord(ev[2], st);
  if (A.train) {
    launch_rel_post(P, st);
    hipLaunchKernelGGL((update_kernel<Rescal, VEC, NC, SK_DOT>), dim3(G.gridU), dim3(kUpdThreads), 0, st, A);
    hipLaunchKernelGGL(partials_norm_kernel, dim3(1), dim3(256), 0, st, A.upart, (int)G.gridU, A.ctl, 0, A.norm2_out,
                       lam, 1.f / (float)A.ent.rows, 1.f / (float)A.rel.rows, A.loss_out, A.loss_accum, A.sig,
                       A.status);
  }
  return KGE_OK;
}

kge_status launch_step_rescal(const StepArgs& A, const StepGeom& G, const RelArgs& P, float lam, float* regpart,
                              hipStream_t st, hipEvent_t const* ev) {
  if (G.vec == 4) {
    if (G.nc == 1) return rescal_vn<4, 1>(A, G, P, lam, regpart, st, ev);
    if (G.nc == 2) return rescal_vn<4, 2>(A, G, P, lam, regpart, st, ev);
    return rescal_vn<4, 4>(A, G, P, lam, regpart, st, ev);
  }
  if (G.nc == 1) return rescal_vn<1, 1>(A, G, P, lam, regpart, st, ev);
  if (G.nc == 2) return rescal_vn<1, 2>(A, G, P, lam, regpart, st, ev);
  return rescal_vn<1, 4>(A, G, P, lam, regpart, st, ev);
}
#endif  // KGE_ONLY_ONE


}  // namespace kge
