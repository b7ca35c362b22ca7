// RotatE instances of the fused step kernels (RotatE.py:126-181).
#include "kge_step_impl.h"

namespace kge {

#ifndef KGE_ONLY_ONE
// RotatE: Lp kinds on complex rows, VEC 4 / 2 (a complex pair never splits)
kge_status launch_rotate(const StepArgs& A, const StepGeom& G, int sk, hipStream_t st, hipEvent_t const* ev) {
  if (G.vec == 4) {
    if (G.nc == 1) return by_sk_lp<RotatE, 4, 1>(A, G, sk, st, ev);
    if (G.nc == 2) return by_sk_lp<RotatE, 4, 2>(A, G, sk, st, ev);
    return by_sk_lp<RotatE, 4, 4>(A, G, sk, st, ev);
  }
  if (G.nc == 1) return by_sk_lp<RotatE, 2, 1>(A, G, sk, st, ev);
  if (G.nc == 2) return by_sk_lp<RotatE, 2, 2>(A, G, sk, st, ev);
  return by_sk_lp<RotatE, 2, 4>(A, G, sk, st, ev);
}

#endif  // KGE_ONLY_ONE

}  // namespace kge
