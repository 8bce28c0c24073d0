// R-NSGA-III survival + tournament selection (gfx950), one workgroup per initial state:
// k_survive wraps survival.h's survive_state; k_select, k_init_pool, k_gather_pop.
#include <limits.h>

#include "check.h"
#include "engine.h"
#include "kernels.h"
#include "philox.h"
#include "survival.h"
#include "wave.h"

namespace mv {

// T = surv_threads(N): SURV_T for the LDS-bitset instance, SURV_T_BIG above SURV_NLDS
template <int NWMAX, int T>
__global__ __launch_bounds__(T) void k_survive(SurvArgs a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  survive_state<NWMAX, T>(a, blockIdx.x, a.N, a.gen, a.sel_gen, a.parents_out, smem);
}

__global__ __launch_bounds__(SURV_T) void k_select(int P, int O, uint64_t seed, uint32_t sk,
                                                   int gen, const int* pop_slot, int* parents) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int b = blockIdx.x;
  const int n_m = (O + 1) / 2;
  const int slots = ((n_m * 4 + P - 1) / P) * P;
  unsigned long long* key = (unsigned long long*)smem;
  int* perm = (int*)(key + pow2_at_least(slots));
  tournament<SURV_T>(P, O, seed, sk, gen, pop_slot ? pop_slot + (size_t)b * P : nullptr,
             parents + (size_t)b * n_m * 2, key, perm);
}

__global__ void k_init_pool(int B, int P, int O, int V, int S, const double* genes0, double* pool,
                            int* pop_slot, int* free_slot) {
  const size_t tot = (size_t)B * P * V;
  for (size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x; t < tot;
       t += (size_t)gridDim.x * blockDim.x) {
    const size_t b = t / ((size_t)P * V);
    const size_t r = t - b * P * V;
    const size_t s = r / V, g = r - s * V;
    pool[(b * S + s) * V + g] = genes0[b * V + g];
  }
  for (size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x; t < (size_t)B * S;
       t += (size_t)gridDim.x * blockDim.x) {
    const int b = (int)(t / S), s = (int)(t - (size_t)b * S);
    if (s < P)
      pop_slot[(size_t)b * P + s] = s;
    else
      free_slot[(size_t)b * O + (s - P)] = s;
  }
}

__global__ void k_gather_pop(int B, int P, int V, int Vr, int S, const int* cmap, const double* glr,
                             const int* pop_slot, const double* pool, const double* poolF,
                             double* genes, double* F) {
  const size_t tot = (size_t)B * P;
  for (size_t t = blockIdx.x; t < tot; t += gridDim.x) {
    const size_t b = t / P;
    const int s = pop_slot[t];
    if (genes)
      for (int g = threadIdx.x; g < Vr; g += blockDim.x) {
        const int c = cmap ? cmap[g] : g;
        genes[t * Vr + g] = c >= 0 ? pool[(b * S + s) * V + c] : glr[b * Vr + g];
      }
    if (F && threadIdx.x < 3) F[t * 3 + threadIdx.x] = poolF[(b * S + s) * 3 + threadIdx.x];
  }
}

MV_DEFINE_TAKE_CHECKS(take_checks_survive)

hipError_t take_survival_dump(double* out) {
#ifdef MV_CHECKS
  hipError_t e = hipMemcpyFromSymbol(out, HIP_SYMBOL(g_surv_dump), SURV_DUMP_N * sizeof(double));
  if (e != hipSuccess) return e;
  const int z = 0;
  e = hipMemcpyToSymbol(HIP_SYMBOL(g_surv_dump_owner), &z, sizeof(int));
  if (e != hipSuccess) return e;
  static double zero[SURV_DUMP_N];
  return hipMemcpyToSymbol(HIP_SYMBOL(g_surv_dump), zero, SURV_DUMP_N * sizeof(double));
#else
  for (int k = 0; k < SURV_DUMP_N; ++k) out[k] = 0.0;
  return hipSuccess;
#endif
}

size_t surv_lds_bytes(int N, int R, int Pperm, int ptab_words, int threads) {
  return surv_offsets(N, R, Pperm, ptab_words, threads).total;
}

hipError_t launch_survive(const SurvArgs& a, int B, hipStream_t stream) {
  if (B <= 0) return hipSuccess;
  const int n_m = a.parents_out ? (a.O_next + 1) / 2 : 0;
  const int pslots = a.parents_out ? ((n_m * 4 + a.n_survive - 1) / a.n_survive) * a.n_survive : 1;
  static const size_t pad = lds_pad("MV_LDS_PAD_SURV");
  const int T = a.N > SURV_NLDS ? SURV_T_BIG : (a.wide ? SURV_T_MID : SURV_T);
  const size_t lds =
      surv_lds_bytes(a.N, a.R, pslots, a.plan_hdr ? plan_tab_words(a.Vr, a.V) : 0, T) + pad;
  static bool configured = false;
  if (!configured) {
    (void)hipFuncSetAttribute((const void*)k_survive<SURV_NLDS / 64, SURV_T>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    (void)hipFuncSetAttribute((const void*)k_survive<SURV_NLDS / 64, SURV_T_MID>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    (void)hipFuncSetAttribute((const void*)k_survive<SURV_NMAX / 64, SURV_T_BIG>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    (void)hipGetLastError();
    configured = true;
  }
  if (a.N <= SURV_NLDS) {
    if (T == SURV_T_MID)
      hipLaunchKernelGGL((k_survive<SURV_NLDS / 64, SURV_T_MID>), dim3(B), dim3(SURV_T_MID), lds,
                         stream, a);
    else
      hipLaunchKernelGGL((k_survive<SURV_NLDS / 64, SURV_T>), dim3(B), dim3(SURV_T), lds, stream,
                         a);
  } else {
    if (!a.dom_g || a.dom_stride < (size_t)a.N * ((a.N + 63) / 64)) return hipErrorInvalidValue;
    hipLaunchKernelGGL((k_survive<SURV_NMAX / 64, SURV_T_BIG>), dim3(B), dim3(SURV_T_BIG), lds,
                       stream, a);
  }
  return hipGetLastError();
}

hipError_t launch_select(int B, int P, int O, uint64_t seed, uint32_t sk, int gen,
                         const int* pop_slot, int* parents, hipStream_t stream) {
  if (B <= 0) return hipSuccess;
  const int n_m = (O + 1) / 2;
  const int slots = ((n_m * 4 + P - 1) / P) * P;
  const size_t lds = (size_t)pow2_at_least(slots) * 8 + (size_t)slots * 4;
  hipLaunchKernelGGL(k_select, dim3(B), dim3(SURV_T), lds, stream, P, O, seed, sk,
                     gen, pop_slot, parents);
  return hipGetLastError();
}

hipError_t launch_init_pool(int B, int P, int O, int V, int S, const double* genes0, double* pool,
                            int* pop_slot, int* free_slot, hipStream_t stream) {
  hipLaunchKernelGGL(k_init_pool, dim3(1024), dim3(256), 0, stream, B, P, O, V, S, genes0, pool,
                     pop_slot, free_slot);
  return hipGetLastError();
}

hipError_t launch_gather_pop(int B, int P, int V, int Vr, int S, const int* cmap,
                             const double* glr, const int* pop_slot, const double* pool,
                             const double* poolF, double* genes, double* F, hipStream_t stream) {
  hipLaunchKernelGGL(k_gather_pop, dim3(2048), dim3(256), 0, stream, B, P, V, Vr, S, cmap, glr,
                     pop_slot, pool, poolF, genes, F);
  return hipGetLastError();
}

}  // namespace mv
