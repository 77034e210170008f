// gsdr-mi355x: tuning probes for the headline FIR (FC, D = 4), reachable only through
// gsdrxFirFCVariant(variant >= 100). Not used by any gsdr* entry point.
//   100: staging only (HBM -> LDS, no FIR arithmetic)        101: compute only (no HBM loads)
//   102: full kernel built with -fno-slp-vectorize (scalar v_fma_f32 instead of v_pk_fma_f32)
// This file is compiled with -fno-slp-vectorize (see Makefile), which only matters for 102.
#include <hip/hip_runtime.h>

#include "fir_dispatch.hpp"

namespace gsdr {

hipError_t launch_fc_probe(const FirJob& j, hipStream_t s) {
  switch (j.variant) {
    case 100:
      return launch_poly<float, float2, 4, 8, 16, 128, kModeFir, 1>(j, s);
    case 101:
      return launch_poly<float, float2, 4, 8, 16, 128, kModeFir, 2>(j, s);
    case 102:
      return launch_poly<float, float2, 4, 8, 16, 128, kModeFir, 0>(j, s);
    default:
      return hipErrorInvalidValue;
  }
}

}  // namespace gsdr
