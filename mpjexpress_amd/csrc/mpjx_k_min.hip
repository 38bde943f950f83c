// mpjx_k_min.hip — kernel instantiations for the MIN (src/mpi/Min<Type>.java) functors (split from the other op families so
// hipcc compiles them in parallel). Type codes are mpi.Datatype base types (src/mpi/Datatype.java:57-66).
#include "mpjx_kernels.hpp"

namespace mpjx {
hipError_t launch_min(int type, int kind, int P, const PwayArgs& a, hipStream_t s, bool vec) {
  switch (type) {
    case 1: /* BYTE */ return launch_functor<Min<int8_t>>(kind, P, a, s, vec);
    case 2: /* CHAR */ return launch_functor<Min<uint16_t>>(kind, P, a, s, vec);
    case 3: /* SHORT */ return launch_functor<Min<int16_t>>(kind, P, a, s, vec);
    case 5: /* INT */ return launch_functor<Min<int32_t>>(kind, P, a, s, vec);
    case 6: /* LONG */ return launch_functor<Min<int64_t>>(kind, P, a, s, vec);
    case 7: /* FLOAT */ return launch_functor<Min<float>>(kind, P, a, s, vec);
    case 8: /* DOUBLE */ return launch_functor<Min<double>>(kind, P, a, s, vec);
  }
  return hipErrorInvalidValue;
}

}  // namespace mpjx
