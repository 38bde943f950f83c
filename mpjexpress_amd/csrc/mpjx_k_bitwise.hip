// mpjx_k_bitwise.hip — BAND/BOR/BXOR dispatch (src/mpi/{Band,Bor,Bxor}<Type>.java); the kernel
// instantiations live in mpjx_k_band.hip, mpjx_k_bor.hip and mpjx_k_bxor.hip (compiled in parallel).
#include "mpjx_kernels.hpp"

namespace mpjx {
hipError_t launch_bitwise(int op, int type, int kind, int P, const PwayArgs& a, hipStream_t s, bool vec) {
  switch (op) {
    case 6: return launch_band(type, kind, P, a, s, vec);  /* BAND */
    case 8: return launch_bor(type, kind, P, a, s, vec);   /* BOR */
    case 10: return launch_bxor(type, kind, P, a, s, vec); /* BXOR */
  }
  return hipErrorInvalidValue;
}

}  // namespace mpjx
