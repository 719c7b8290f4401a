// p256_verify_g24.hip -- verify kernels instantiated for the G table 24 bits
// geometry pairs (kernels.h PBFTV_COMBOS_G24); code in verify_kernels.h.
#include "verify_kernels.h"

namespace pbftv {
PBFTV_VERIFY_PART(g24, PBFTV_COMBOS_G24)
}  // namespace pbftv
