// Explicit instantiation of the BeerGame launchers for levels 9-12 (see
// scg_beergame_kernels.h): one of four units compiled in parallel.
#include "scg_beergame_kernels.h"

namespace scg {
SCG_BG_LAUNCHERS(, 9)
SCG_BG_LAUNCHERS(, 10)
SCG_BG_LAUNCHERS(, 11)
SCG_BG_LAUNCHERS(, 12)
}  // namespace scg
