// mpjx_k_bor.hip — kernel instantiations for the BOR (src/mpi/Bor<Type>.java) functors (one op family per
// translation unit so hipcc compiles them in parallel). Type codes are mpi.Datatype base types
// (src/mpi/Datatype.java:57-66).
#include "mpjx_kernels.hpp"

namespace mpjx {
hipError_t launch_bor(int type, int kind, int P, const PwayArgs& a, hipStream_t s, bool vec) {
  switch (type) {
    case 1: /* BYTE */ return launch_functor<Bor<uint8_t>>(kind, P, a, s, vec);
    case 2: /* CHAR */ return launch_functor<Bor<uint16_t>>(kind, P, a, s, vec);
    case 3: /* SHORT */ return launch_functor<Bor<uint16_t>>(kind, P, a, s, vec);
    case 5: /* INT */ return launch_functor<Bor<uint32_t>>(kind, P, a, s, vec);
    case 6: /* LONG */ return launch_functor<Bor<uint64_t>>(kind, P, a, s, vec);
  }
  return hipErrorInvalidValue;
}

}  // namespace mpjx
