// TransE instances of the owner-side scoring passes (kge_owner.h;
// TransE.py:127-174 scored where the negatives' rows live).
#include "kge_owner.h"

namespace kge {

template <int VEC, int NC>
static kge_status owner_transe_sk(const StepArgs& A, const StepGeom& G, int sk, int phase, hipStream_t st) {
  switch (sk) {
    case SK_P1: return launch_owner_family<TransE, VEC, NC, SK_P1>(A, G, phase, st);
    case SK_P2: return launch_owner_family<TransE, VEC, NC, SK_P2>(A, G, phase, st);
    case SK_PINF: return launch_owner_family<TransE, VEC, NC, SK_PINF>(A, G, phase, st);
    case SK_PGEN: return launch_owner_family<TransE, VEC, NC, SK_PGEN>(A, G, phase, st);
    default: return launch_owner_family<TransE, VEC, NC, SK_DOT>(A, G, phase, st);
  }
}

kge_status launch_owner_transe(const StepArgs& A, const StepGeom& G, int sk, int phase, hipStream_t st) {
  if (G.vec == 4) {
    if (G.nc == 1) return owner_transe_sk<4, 1>(A, G, sk, phase, st);
    if (G.nc == 2) return owner_transe_sk<4, 2>(A, G, sk, phase, st);
    return owner_transe_sk<4, 4>(A, G, sk, phase, st);
  }
  if (G.nc == 1) return owner_transe_sk<1, 1>(A, G, sk, phase, st);
  if (G.nc == 2) return owner_transe_sk<1, 2>(A, G, sk, phase, st);
  return owner_transe_sk<1, 4>(A, G, sk, phase, st);
}

}  // namespace kge
