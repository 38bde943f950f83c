// mpjx_k_loc.hip — MAXLOC / MINLOC dispatch (src/mpi/Maxloc.java, src/mpi/Minloc.java); the kernel
// instantiations live in mpjx_k_maxloc.hip and mpjx_k_minloc.hip (compiled in parallel).
#include "mpjx_kernels.hpp"

namespace mpjx {
hipError_t launch_loc(int op, int type, int kind, int P, const PwayArgs& a, hipStream_t s, bool vec) {
  switch (op) {
    case 11: return launch_maxloc(type, kind, P, a, s, vec); /* MAXLOC */
    case 12: return launch_minloc(type, kind, P, a, s, vec); /* MINLOC */
  }
  return hipErrorInvalidValue;
}

}  // namespace mpjx
