// mpjx_k_bitwise.hip — kernel instantiations for the BAND/BOR/BXOR (src/mpi/{Band,Bor,Bxor}<Type>.java) functors (split from the other op families so
// hipcc compiles them in parallel). Type codes are mpi.Datatype base types (src/mpi/Datatype.java:57-66).
#include "mpjx_kernels.hpp"

namespace mpjx {
template <template <class> class F>
static hipError_t by_type(int type, int kind, int P, const PwayArgs& a, hipStream_t s, bool vec) {
  switch (type) {
    case 1: /* BYTE */ return launch_functor<F<uint8_t>>(kind, P, a, s, vec);
    case 2: /* CHAR */ return launch_functor<F<uint16_t>>(kind, P, a, s, vec);
    case 3: /* SHORT */ return launch_functor<F<uint16_t>>(kind, P, a, s, vec);
    case 5: /* INT */ return launch_functor<F<uint32_t>>(kind, P, a, s, vec);
    case 6: /* LONG */ return launch_functor<F<uint64_t>>(kind, P, a, s, vec);
  }
  return hipErrorInvalidValue;
}

hipError_t launch_bitwise(int op, int type, int kind, int P, const PwayArgs& a, hipStream_t s, bool vec) {
  switch (op) {
    case 6: return by_type<Band>(type, kind, P, a, s, vec);  /* BAND */
    case 8: return by_type<Bor>(type, kind, P, a, s, vec);   /* BOR */
    case 10: return by_type<Bxor>(type, kind, P, a, s, vec); /* BXOR */
  }
  return hipErrorInvalidValue;
}

}  // namespace mpjx
