// mpjx_k_band.hip — kernel instantiations for the BAND (src/mpi/Band<Type>.java) functors (one op family per
// translation unit so hipcc compiles them in parallel). Type codes are mpi.Datatype base types
// (src/mpi/Datatype.java:57-66).
#include "mpjx_kernels.hpp"

namespace mpjx {
hipError_t launch_band(int type, int kind, int P, const PwayArgs& a, hipStream_t s, bool vec) {
  switch (type) {
    case 1: /* BYTE */ return launch_functor<Band<uint8_t>>(kind, P, a, s, vec);
    case 2: /* CHAR */ return launch_functor<Band<uint16_t>>(kind, P, a, s, vec);
    case 3: /* SHORT */ return launch_functor<Band<uint16_t>>(kind, P, a, s, vec);
    case 5: /* INT */ return launch_functor<Band<uint32_t>>(kind, P, a, s, vec);
    case 6: /* LONG */ return launch_functor<Band<uint64_t>>(kind, P, a, s, vec);
  }
  return hipErrorInvalidValue;
}

}  // namespace mpjx
