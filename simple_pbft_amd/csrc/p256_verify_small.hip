// p256_verify_small.hip -- verify kernels instantiated for the G tables of 20, 16 and 8 bits
// geometry pairs (kernels.h PBFTV_COMBOS_SMALL); code in verify_kernels.h.
#include "verify_kernels.h"

namespace pbftv {
PBFTV_VERIFY_PART(small, PBFTV_COMBOS_SMALL)
}  // namespace pbftv
