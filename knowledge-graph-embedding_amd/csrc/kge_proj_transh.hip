// TransH instances of the projection-family score kernel (TransH.py:149-185).
#include "kge_proj.h"

namespace kge {

template <int VEC, int NC, int SK>
static void pj_launch(const StepArgs& A, const PjArgs& P, hipStream_t st) {
  const PjLds L = pj_lds(A.Keff, KGE_WAVE * VEC * NC, false);
  hipLaunchKernelGGL((proj_kernel<false, VEC, NC, SK>), dim3((unsigned)A.B), dim3(kPjThreads),
                     (size_t)L.total * 4, st, A, P);
}

template <int VEC, int NC>
static void pj_sk(const StepArgs& A, const PjArgs& P, int sk, hipStream_t st) {
  switch (sk) {
    case SK_P1: pj_launch<VEC, NC, SK_P1>(A, P, st); break;
    case SK_P2: pj_launch<VEC, NC, SK_P2>(A, P, st); break;
    case SK_PINF: pj_launch<VEC, NC, SK_PINF>(A, P, st); break;
    case SK_PGEN: pj_launch<VEC, NC, SK_PGEN>(A, P, st); break;
    default: pj_launch<VEC, NC, SK_DOT>(A, P, st); break;
  }
}

kge_status launch_proj_transh(const StepArgs& A, const StepGeom& G, const PjArgs& P, int sk, hipStream_t st) {
  if (G.nc > 2) return KGE_EUNSUPPORTED;
  if (G.vec == 4) { if (G.nc == 1) pj_sk<4, 1>(A, P, sk, st); else pj_sk<4, 2>(A, P, sk, st); }
  else if (G.vec == 2) { if (G.nc == 1) pj_sk<2, 1>(A, P, sk, st); else pj_sk<2, 2>(A, P, sk, st); }
  else { if (G.nc == 1) pj_sk<1, 1>(A, P, sk, st); else pj_sk<1, 2>(A, P, sk, st); }
  return KGE_OK;
}

}  // namespace kge
