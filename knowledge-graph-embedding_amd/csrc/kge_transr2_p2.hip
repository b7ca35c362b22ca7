// transr2_kernel instances for SK_P2 (kge_transr2.h).
#include "kge_transr2.h"

namespace kge {
template void launch_transr2<SK_P2>(const StepArgs&, const TrArgs&, hipStream_t);
}  // namespace kge
