// TransE instances of the fused step kernels (TransE.py:127-174).
#include "kge_step_impl.h"

namespace kge {

#ifndef KGE_ONLY_ONE
// TransE: every score kind, VEC 4 / 1
kge_status launch_transe(const StepArgs& A, const StepGeom& G, int sk, hipStream_t st, hipEvent_t const* ev) {
  if (G.vec == 4) {
    if (G.nc == 1) return by_sk<TransE, 4, 1>(A, G, sk, st, ev);
    if (G.nc == 2) return by_sk<TransE, 4, 2>(A, G, sk, st, ev);
    return by_sk<TransE, 4, 4>(A, G, sk, st, ev);
  }
  if (G.nc == 1) return by_sk<TransE, 1, 1>(A, G, sk, st, ev);
  if (G.nc == 2) return by_sk<TransE, 1, 2>(A, G, sk, st, ev);
  return by_sk<TransE, 1, 4>(A, G, sk, st, ev);
}

#endif  // KGE_ONLY_ONE

}  // namespace kge
