// DistMult and RotatE instances of the owner-side scoring passes (kge_owner.h;
// DistMult.py:118-167, RotatE.py:126-165).
#include "kge_owner.h"

namespace kge {

template <int VEC, int NC>
static kge_status owner_rotate_sk(const StepArgs& A, const StepGeom& G, int sk, int phase, hipStream_t st) {
  switch (sk) {
    case SK_P1: return launch_owner_family<RotatE, VEC, NC, SK_P1>(A, G, phase, st);
    case SK_P2: return launch_owner_family<RotatE, VEC, NC, SK_P2>(A, G, phase, st);
    case SK_PINF: return launch_owner_family<RotatE, VEC, NC, SK_PINF>(A, G, phase, st);
    case SK_PGEN: return launch_owner_family<RotatE, VEC, NC, SK_PGEN>(A, G, phase, st);
    default: return KGE_EUNSUPPORTED;
  }
}

kge_status launch_owner_other(const StepArgs& A, const StepGeom& G, int model, int sk, int phase, hipStream_t st) {
  if (model == KGE_MODEL_DISTMULT) {
    if (G.vec == 4) {
      if (G.nc == 1) return launch_owner_family<DistMult, 4, 1, SK_DOT>(A, G, phase, st);
      if (G.nc == 2) return launch_owner_family<DistMult, 4, 2, SK_DOT>(A, G, phase, st);
      return launch_owner_family<DistMult, 4, 4, SK_DOT>(A, G, phase, st);
    }
    if (G.nc == 1) return launch_owner_family<DistMult, 1, 1, SK_DOT>(A, G, phase, st);
    if (G.nc == 2) return launch_owner_family<DistMult, 1, 2, SK_DOT>(A, G, phase, st);
    return launch_owner_family<DistMult, 1, 4, SK_DOT>(A, G, phase, st);
  }
  if (model != KGE_MODEL_ROTATE) return KGE_EUNSUPPORTED;
  if (G.vec == 4) {
    if (G.nc == 1) return owner_rotate_sk<4, 1>(A, G, sk, phase, st);
    if (G.nc == 2) return owner_rotate_sk<4, 2>(A, G, sk, phase, st);
    return owner_rotate_sk<4, 4>(A, G, sk, phase, st);
  }
  if (G.nc == 1) return owner_rotate_sk<2, 1>(A, G, sk, phase, st);
  if (G.nc == 2) return owner_rotate_sk<2, 2>(A, G, sk, phase, st);
  return owner_rotate_sk<2, 4>(A, G, sk, phase, st);
}

}  // namespace kge
