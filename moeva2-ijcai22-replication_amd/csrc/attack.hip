// Whole-attack launch dispatcher (host side of attack_impl.h's k_attack): picks the
// kernel instance for the problem's genetic layout, or reports the shape unsupported so the
// caller runs the per-phase kernel chain instead.
#include "attack_impl.h"

namespace mv {

hipError_t launch_attack_ident(const AttackArgs& a, size_t lds, int grid, int nt,
                               hipStream_t s);
hipError_t launch_attack_ohe(const AttackArgs& a, size_t lds, int grid, bool big,
                             hipStream_t s);

size_t attack_lds_bytes(const DProblem& p, int P, int O, int R, int T) {
  const VaryOff o = vary_offsets(p);
  const size_t rows = fused_lds(o, T / 64).total;
  const size_t mlp = mlp2_lds(p);
  const int n_m = (O + 1) / 2;
  const int pslots = ((n_m * 4 + P - 1) / P) * P;
  const size_t surv = surv_offsets(P + O, R, pslots).total;
  size_t m = rows > mlp ? rows : mlp;
  return m > surv ? m : surv;
}

// The shapes the whole-attack kernel is instantiated for (the shipped botnet and LCLD
// problems and their augmented variants); anything else runs the per-phase chain.
static int attack_variant(const DProblem& p, int N, bool* ident, int* nt, bool* full, int* cj,
                          int* nw) {
  if (!p.mlp2 || p.n_layers < 2) return 0;
  const int m = p.V > p.Dm4 ? p.V : p.Dm4;
  const int ntr = (m + 63) / 64;
  *nt = ntr <= 1 ? 1 : ntr <= 2 ? 2 : ntr <= 4 ? 4 : ntr <= 8 ? 8 : 16;
  *ident = p.ident != 0;
  *full = p.full_ops != 0;
  *cj = mlp2_hmax(p) <= 64 ? 1 : 2;
  *nw = N <= SURV_NLDS ? SURV_NLDS / 64 : SURV_NMAX / 64;
  if (*cj != 1) return 0;
  if (*ident && !*full && (*nt == 8 || *nt == 16) && N <= SURV_NLDS) return 1;
  if (!*ident && *full && *nt == 1) return 1;
  return 0;
}

bool attack_supported(const DProblem& p, int P, int O, int R) {
  bool id, fu;
  int nt, cj, nw;
  if (!attack_variant(p, P + O, &id, &nt, &fu, &cj, &nw)) return false;
  return attack_lds_bytes(p, P, O, R, ATT_T) <= 160 * 1024;
}

static int cu_count_att() {
  static int n = 0;
  if (!n) {
    int dev = 0;
    hipDeviceProp_t prop;
    if (hipGetDevice(&dev) == hipSuccess && hipGetDeviceProperties(&prop, dev) == hipSuccess)
      n = prop.multiProcessorCount;
    if (n <= 0) n = 256;
  }
  return n;
}

hipError_t launch_attack(const AttackArgs& args, hipStream_t stream) {
  if (args.B <= 0) return hipSuccess;
  bool id, fu;
  int nt, cj, nw;
  if (!attack_variant(args.va.p, args.P + args.O, &id, &nt, &fu, &cj, &nw))
    return hipErrorNotSupported;
  const size_t lds = attack_lds_bytes(args.va.p, args.P, args.O, args.sa.R, ATT_T);
  const int cap = 2 * cu_count_att();
  const int grid = args.B < cap ? args.B : cap;
  if (id) return launch_attack_ident(args, lds, grid, nt, stream);
  return launch_attack_ohe(args, lds, grid, nw != SURV_NLDS / 64, stream);
}

}  // namespace mv
