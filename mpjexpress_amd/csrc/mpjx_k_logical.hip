// mpjx_k_logical.hip — kernel instantiations for the LAND/LOR/LXOR (src/mpi/{Land,Lor,Lxor}Boolean.java) and the
// FAITHFUL BOR/BXOR no-op (Keep) functors (split from the other op families so
// hipcc compiles them in parallel). Type codes are mpi.Datatype base types (src/mpi/Datatype.java:57-66).
#include "mpjx_kernels.hpp"

namespace mpjx {
hipError_t launch_logical(int op, int kind, int P, const PwayArgs& a, hipStream_t s, bool vec) {
  switch (op) {
    case 5: return launch_functor<Land>(kind, P, a, s, vec);  /* LAND */
    case 7: return launch_functor<Lor>(kind, P, a, s, vec);   /* LOR */
    case 9: return launch_functor<Lxor>(kind, P, a, s, vec);  /* LXOR */
  }
  return hipErrorInvalidValue;
}

hipError_t launch_keep(int type, int kind, int P, const PwayArgs& a, hipStream_t s, bool vec) {
  switch (type) {
    case 1: return launch_functor<Keep<uint8_t>>(kind, P, a, s, vec);
    case 2: case 3: return launch_functor<Keep<uint16_t>>(kind, P, a, s, vec);
    case 5: return launch_functor<Keep<uint32_t>>(kind, P, a, s, vec);
    case 6: return launch_functor<Keep<uint64_t>>(kind, P, a, s, vec);
  }
  return hipErrorInvalidValue;
}

}  // namespace mpjx
