// mpjx_k_prod.hip — kernel instantiations for the PROD (src/mpi/Prod<Type>.java) functors (split from the other op families so
// hipcc compiles them in parallel). Type codes are mpi.Datatype base types (src/mpi/Datatype.java:57-66).
#include "mpjx_kernels.hpp"

namespace mpjx {
hipError_t launch_prod(int type, int kind, int P, const PwayArgs& a, hipStream_t s, bool vec) {
  switch (type) {
    case 1: /* BYTE */ return launch_functor<Prod<uint8_t>>(kind, P, a, s, vec);
    case 2: /* CHAR */ return launch_functor<Prod<uint16_t>>(kind, P, a, s, vec);
    case 3: /* SHORT */ return launch_functor<Prod<uint16_t>>(kind, P, a, s, vec);
    case 5: /* INT */ return launch_functor<Prod<uint32_t>>(kind, P, a, s, vec);
    case 6: /* LONG */ return launch_functor<Prod<uint64_t>>(kind, P, a, s, vec);
    case 7: /* FLOAT */ return launch_functor<Prod<float>>(kind, P, a, s, vec);
    case 8: /* DOUBLE */ return launch_functor<Prod<double>>(kind, P, a, s, vec);
  }
  return hipErrorInvalidValue;
}

}  // namespace mpjx
