// mpjx_k_bxor.hip — kernel instantiations for the BXOR (src/mpi/Bxor<Type>.java) functors (one op family per
// translation unit so hipcc compiles them in parallel). Type codes are mpi.Datatype base types
// (src/mpi/Datatype.java:57-66).
#include "mpjx_kernels.hpp"

namespace mpjx {
hipError_t launch_bxor(int type, int kind, int P, const PwayArgs& a, hipStream_t s, bool vec) {
  switch (type) {
    case 1: /* BYTE */ return launch_functor<Bxor<uint8_t>>(kind, P, a, s, vec);
    case 2: /* CHAR */ return launch_functor<Bxor<uint16_t>>(kind, P, a, s, vec);
    case 3: /* SHORT */ return launch_functor<Bxor<uint16_t>>(kind, P, a, s, vec);
    case 5: /* INT */ return launch_functor<Bxor<uint32_t>>(kind, P, a, s, vec);
    case 6: /* LONG */ return launch_functor<Bxor<uint64_t>>(kind, P, a, s, vec);
  }
  return hipErrorInvalidValue;
}

}  // namespace mpjx
