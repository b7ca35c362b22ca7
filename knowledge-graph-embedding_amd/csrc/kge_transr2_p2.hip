// transr2_kernel instances for SK_P2 (kge_transr2.h).
#include "kge_transr2.h"

namespace kge {
template void launch_transr2<SK_P2>(const StepArgs&, const TrArgs&, hipStream_t);
}  // namespace kge

#ifdef KGE_PHASE_PROF
// profiling builds (tools/transr_prof.py): this unit's phase counters
extern "C" int kge_trprof2_read(unsigned long long* out, int n) {
  if (n > 64) n = 64;
  if (hipMemcpyFromSymbol(out, HIP_SYMBOL(kge::g_kge_prof), n * sizeof(unsigned long long)) != hipSuccess) return 1;
  unsigned long long z[64] = {0};
  return hipMemcpyToSymbol(HIP_SYMBOL(kge::g_kge_prof), z, sizeof(z)) != hipSuccess;
}
#endif
