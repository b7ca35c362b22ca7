// RESCAL instances of the fused step kernels (RESCAL.py:140-200); the
// relation-matrix MFMA passes live in kge_rel.hip.
#include "kge_step_impl.h"

namespace kge {

#ifndef KGE_ONLY_ONE
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
    // (the dR pass and the dense entity update are independent, but a second
    // stream costs more than it overlaps: ~11 us per cross-queue event wait,
    // measured, profiles/r03/rescal_side_stream.txt)
    launch_rel_post(P, st);   // dR strips: dense relation gradient + norm^2 / ||R||^2 partials
    hipLaunchKernelGGL((update_kernel<Rescal, VEC, NC, SK_DOT>), dim3(G.gridU), dim3(kUpdThreads), 0, st, A);
    // both dense norms, the regulariser loss term, the SGD scales
    launch_rescal_norms(P, A.upart, G.gridU, lam, A.lr, A.clip_norm, A.loss_accum, st);
    if (!A.grad_mode) {
      // keras SGD on the dense gradients (KGE_OPT_GRAD: the caller applies)
      if (P.lazy_absent) {
        launch_rescal_apply(P, A.ent, A.gent, A.lr, A.clip_norm, st);
      } else {
        const TabView tabs[2] = {A.ent, P.rel};
        const float* gs[2] = {A.gent, P.grel};
        for (int v = 0; v < 2; ++v) {
          ApplyArgs a{};
          a.w = tabs[v].p; a.rows = tabs[v].rows; a.cols = tabs[v].cols; a.ld = tabs[v].ld;
          a.g = gs[v]; a.norm2 = &A.ctl->dn2[v]; a.lr = A.lr; a.clip = A.clip_norm;
          a.ctl = A.ctl; a.sig = A.sig; a.status = A.status;
          launch_apply(a, st);
        }
      }
    }
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
