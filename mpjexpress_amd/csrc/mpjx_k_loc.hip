// mpjx_k_loc.hip — kernel instantiations for MAXLOC / MINLOC on (value, index) pairs
// (src/mpi/Maxloc.java, src/mpi/Minloc.java; types SHORT2/INT2/LONG2/FLOAT2/DOUBLE2 = 0x100 | base).
#include "mpjx_kernels.hpp"

namespace mpjx {

template <template <class> class F>
static hipError_t by_pair(int type, int kind, int P, const PwayArgs& a, hipStream_t s, bool vec) {
  switch (type) {
    case 0x103: return launch_functor<F<int16_t>>(kind, P, a, s, vec);  /* SHORT2 */
    case 0x105: return launch_functor<F<int32_t>>(kind, P, a, s, vec);  /* INT2 */
    case 0x106: return launch_functor<F<int64_t>>(kind, P, a, s, vec);  /* LONG2 */
    case 0x107: return launch_functor<F<float>>(kind, P, a, s, vec);    /* FLOAT2 */
    case 0x108: return launch_functor<F<double>>(kind, P, a, s, vec);   /* DOUBLE2 */
  }
  return hipErrorInvalidValue;
}

hipError_t launch_loc(int op, int type, int kind, int P, const PwayArgs& a, hipStream_t s, bool vec) {
  switch (op) {
    case 11: return by_pair<Maxloc>(type, kind, P, a, s, vec); /* MAXLOC */
    case 12: return by_pair<Minloc>(type, kind, P, a, s, vec); /* MINLOC */
  }
  return hipErrorInvalidValue;
}

}  // namespace mpjx
