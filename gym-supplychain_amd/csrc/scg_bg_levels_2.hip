// Explicit instantiation of the BeerGame launchers for levels 5-8 (see
// scg_beergame_kernels.h): one of four units compiled in parallel.
#include "scg_beergame_kernels.h"

namespace scg {
SCG_BG_LAUNCHERS(, 5)
SCG_BG_LAUNCHERS(, 6)
SCG_BG_LAUNCHERS(, 7)
SCG_BG_LAUNCHERS(, 8)
}  // namespace scg
