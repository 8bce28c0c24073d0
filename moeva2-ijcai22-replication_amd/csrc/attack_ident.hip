// Whole-attack kernel instances for one-to-one genetic layouts (every gene is a mutable
// real/int feature: the CTU-13 botnet problems, 432 and 603 genes).
#include "attack_impl.h"

namespace mv {

hipError_t launch_attack_ident(const AttackArgs& a, size_t lds, int grid, int nt,
                               hipStream_t s) {
  if (nt == 8) return att_launch<true, 8, false, 1, SURV_NLDS / 64>(a, lds, grid, s);
  if (nt == 16) return att_launch<true, 16, false, 1, SURV_NLDS / 64>(a, lds, grid, s);
  return hipErrorNotSupported;
}

}  // namespace mv
