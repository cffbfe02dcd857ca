// Explicit instantiation of the BeerGame launchers for levels 13-16 (see
// scg_beergame_kernels.h): one of four units compiled in parallel.
#include "scg_beergame_kernels.h"

namespace scg {
SCG_BG_LAUNCHERS(, 13)
SCG_BG_LAUNCHERS(, 14)
SCG_BG_LAUNCHERS(, 15)
SCG_BG_LAUNCHERS(, 16)
}  // namespace scg
