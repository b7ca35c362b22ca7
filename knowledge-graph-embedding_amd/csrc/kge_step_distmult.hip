// DistMult instances of the fused step kernels (DistMult.py:118-167).
#include "kge_step_impl.h"

namespace kge {

#ifndef KGE_ONLY_ONE
// DistMult: its own trilinear score (score_fn unused), VEC 4 / 1
kge_status launch_distmult(const StepArgs& A, const StepGeom& G, hipStream_t st, hipEvent_t const* ev) {
  if (G.vec == 4) {
    if (G.nc == 1) return launch_family<DistMult, 4, 1, SK_DOT>(A, G, st, ev);
    if (G.nc == 2) return launch_family<DistMult, 4, 2, SK_DOT>(A, G, st, ev);
    return launch_family<DistMult, 4, 4, SK_DOT>(A, G, st, ev);
  }
  if (G.nc == 1) return launch_family<DistMult, 1, 1, SK_DOT>(A, G, st, ev);
  if (G.nc == 2) return launch_family<DistMult, 1, 2, SK_DOT>(A, G, st, ev);
  return launch_family<DistMult, 1, 4, SK_DOT>(A, G, st, ev);
}

#endif  // KGE_ONLY_ONE

}  // namespace kge
