// mpjx_k_minloc.hip — kernel instantiations for MINLOC on (value, index) pairs (src/mpi/Minloc.java;
// types SHORT2/INT2/LONG2/FLOAT2/DOUBLE2 = 0x100 | base), one op per translation unit.
#include "mpjx_kernels.hpp"

namespace mpjx {
hipError_t launch_minloc(int type, int kind, int P, const PwayArgs& a, hipStream_t s, bool vec) {
  switch (type) {
    case 0x103: return launch_functor<Minloc<int16_t>>(kind, P, a, s, vec);  /* SHORT2 */
    case 0x105: return launch_functor<Minloc<int32_t>>(kind, P, a, s, vec);  /* INT2 */
    case 0x106: return launch_functor<Minloc<int64_t>>(kind, P, a, s, vec);  /* LONG2 */
    case 0x107: return launch_functor<Minloc<float>>(kind, P, a, s, vec);    /* FLOAT2 */
    case 0x108: return launch_functor<Minloc<double>>(kind, P, a, s, vec);   /* DOUBLE2 */
  }
  return hipErrorInvalidValue;
}

}  // namespace mpjx
