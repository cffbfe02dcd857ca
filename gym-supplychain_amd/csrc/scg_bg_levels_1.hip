// Explicit instantiation of the BeerGame launchers for levels 1-4 (see
// scg_beergame_kernels.h): one of four units compiled in parallel.
#include "scg_beergame_kernels.h"

namespace scg {
SCG_BG_LAUNCHERS(, 1)
SCG_BG_LAUNCHERS(, 2)
SCG_BG_LAUNCHERS(, 3)
SCG_BG_LAUNCHERS(, 4)
}  // namespace scg
