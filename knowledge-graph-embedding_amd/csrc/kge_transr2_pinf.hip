// transr2_kernel instances for SK_PINF (kge_transr2.h).
#include "kge_transr2.h"

namespace kge {
template void launch_transr2<SK_PINF>(const StepArgs&, const TrArgs&, hipStream_t);
}  // namespace kge
