// Whole-attack kernel instances for one-hot genetic layouts with the LCLD financial
// constraint ops (LCLD and LCLD-augmented: <= 64 genes), for merged populations up to
// SURV_NLDS (LDS dominance bitsets) and up to SURV_NMAX (n_pop 640: HBM bitsets).
#include "attack_impl.h"

namespace mv {

hipError_t launch_attack_ohe(const AttackArgs& a, size_t lds, int grid, bool big,
                             hipStream_t s) {
  if (big) return att_launch<false, 1, true, 1, SURV_NMAX / 64>(a, lds, grid, s);
  return att_launch<false, 1, true, 1, SURV_NLDS / 64>(a, lds, grid, s);
}

}  // namespace mv
