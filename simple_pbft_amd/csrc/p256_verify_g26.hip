// p256_verify_g26.hip -- verify kernels instantiated for the G table 26 bits
// geometry pairs (kernels.h PBFTV_COMBOS_G26); code in verify_kernels.h.
#include "verify_kernels.h"

namespace pbftv {
PBFTV_VERIFY_PART(g26, PBFTV_COMBOS_G26)
}  // namespace pbftv
