// p256_verify_g29.hip -- verify kernels instantiated for the G table 29 (mixed 5 x 29 + 4 x 28 bits)
// geometry pairs (kernels.h PBFTV_COMBOS_G29); code in verify_kernels.h.
#include "verify_kernels.h"

namespace pbftv {
PBFTV_VERIFY_PART(g29, PBFTV_COMBOS_G29)
}  // namespace pbftv
