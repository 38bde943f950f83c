// mpjx_k_sum.hip — kernel instantiations for the SUM (src/mpi/Sum<Type>.java) functors (split from the other op families so
// hipcc compiles them in parallel). Type codes are mpi.Datatype base types (src/mpi/Datatype.java:57-66).
#include "mpjx_kernels.hpp"

namespace mpjx {
hipError_t launch_sum(int type, int kind, int P, const PwayArgs& a, hipStream_t s, bool vec) {
  switch (type) {
    case 1: /* BYTE */ return launch_functor<Sum<uint8_t>>(kind, P, a, s, vec);
    case 2: /* CHAR */ return launch_functor<Sum<uint16_t>>(kind, P, a, s, vec);
    case 3: /* SHORT */ return launch_functor<Sum<uint16_t>>(kind, P, a, s, vec);
    case 5: /* INT */ return launch_functor<Sum<uint32_t>>(kind, P, a, s, vec);
    case 6: /* LONG */ return launch_functor<Sum<uint64_t>>(kind, P, a, s, vec);
    case 7: /* FLOAT */ return launch_functor<Sum<float>>(kind, P, a, s, vec);
    case 8: /* DOUBLE */ return launch_functor<Sum<double>>(kind, P, a, s, vec);
  }
  return hipErrorInvalidValue;
}

}  // namespace mpjx
