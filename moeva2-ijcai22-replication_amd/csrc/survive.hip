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

// Final population -> its non-dominated members (the per-state result's X / F, pymoo's
// `opt` of the last generation).  Relation of pareto_operation.py:35-51: i dominates j when
// F_i < F_j in some objective and F_i > F_j in none; a member is in the front when no other
// member dominates it (identical rows do not dominate each other).  One workgroup per state,
// the state's F in LDS (structure of arrays), one member per thread: P <= 1022 compares
// against broadcast LDS reads.  offsets[b + 1] receives the state's front size.
__global__ __launch_bounds__(256) void k_front_mask(int P, int S, const int* pop_slot,
                                                     const double* poolF, unsigned char* front,
                                                     int* offsets) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  double* fs = (double*)smem;  // [3][P]
  __shared__ int n_front;
  const int b = blockIdx.x;
  if (threadIdx.x == 0) n_front = 0;
  for (int j = threadIdx.x; j < P; j += blockDim.x) {
    const int s = MV_IDX(pop_slot[(size_t)b * P + j], S, CK_SURV_SLOT);
    const double* f = poolF + ((size_t)b * S + s) * 3;
    fs[j] = f[0];
    fs[P + j] = f[1];
    fs[2 * P + j] = f[2];
  }
  __syncthreads();
  int mine = 0;
  for (int j = threadIdx.x; j < P; j += blockDim.x) {
    const double a0 = fs[j], a1 = fs[P + j], a2 = fs[2 * P + j];
    bool dom = false;
    for (int i = 0; i < P && !dom; ++i) {
      const double c0 = fs[i], c1 = fs[P + i], c2 = fs[2 * P + i];
      const bool less = c0 < a0 || c1 < a1 || c2 < a2;
      const bool more = c0 > a0 || c1 > a1 || c2 > a2;
      dom = less && !more;
    }
    front[(size_t)b * P + j] = dom ? 0 : 1;
    mine += dom ? 0 : 1;
  }
  if (mine) atomicAdd(&n_front, mine);
  __syncthreads();
  if (threadIdx.x == 0) offsets[b + 1] = n_front;
}

// offsets[1..B] (front sizes) -> exclusive row offsets [0..B] (in place), one workgroup:
// each thread sums a contiguous run, a block scan of the run sums, then the runs rewritten.
__global__ __launch_bounds__(1024) void k_front_scan(int B, int* offsets) {
  __shared__ int part[1024];
  const int t = threadIdx.x, T = blockDim.x;
  const int per = (B + T - 1) / T, lo = t * per, hi = min(B, lo + per);
  int sum = 0;
  for (int b = lo; b < hi; ++b) sum += offsets[b + 1];
  part[t] = sum;
  __syncthreads();
  for (int d = 1; d < T; d <<= 1) {
    const int v = t >= d ? part[t - d] : 0;
    __syncthreads();
    part[t] += v;
    __syncthreads();
  }
  int run = part[t] - sum;  // exclusive prefix of this thread's run
  for (int b = lo; b < hi; ++b) {
    const int c = offsets[b + 1];
    offsets[b + 1] = run + c;
    run += c;
  }
  if (t == 0) offsets[0] = 0;
}

// Front members -> X rows offsets[b] .. offsets[b + 1] - 1 (population order), genes of every
// one of the Vr genes (as k_gather_pop) and their F.
__global__ __launch_bounds__(256) void k_front_gather(int P, int V, int Vr, int S, const int* cmap,
                                                       const double* glr, const int* pop_slot,
                                                       const double* pool, const double* poolF,
                                                       const unsigned char* front,
                                                       const int* offsets, double* X, double* Fx) {
  __shared__ int rank[1024];
  const int b = blockIdx.x, lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int nw = blockDim.x >> 6;
  if (wave == 0) {
    int base = 0;
    const unsigned long long below = (1ull << lane) - 1ull;
    for (int c = 0; c < P; c += 64) {
      const int j = c + lane;
      const bool in = j < P && front[(size_t)b * P + j];
      const unsigned long long m = __ballot(in);
      if (j < P) rank[j] = in ? base + __popcll(m & below) : -1;
      base += __popcll(m);
    }
  }
  __syncthreads();
  const size_t row0 = (size_t)offsets[b];
  for (int j = wave; j < P; j += nw) {
    const int r = rank[j];
    if (r < 0) continue;
    const int s = MV_IDX(pop_slot[(size_t)b * P + j], S, CK_SURV_SLOT);
    const double* src = pool + ((size_t)b * S + s) * V;
    if (X) {
      double* dst = X + (row0 + r) * Vr;
      for (int g = lane; g < Vr; g += 64) {
        const int c = cmap ? cmap[g] : g;
        dst[g] = c >= 0 ? src[c] : glr[(size_t)b * Vr + g];
      }
    }
    if (Fx && lane < 3) Fx[(row0 + r) * 3 + lane] = poolF[((size_t)b * S + s) * 3 + lane];
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
  const int T = a.N > SURV_NLDS ? SURV_T_BIG
                                : (a.wide == 2 ? SURV_T_BIG : a.wide ? SURV_T_MID : SURV_T);
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
    (void)hipFuncSetAttribute((const void*)k_survive<SURV_NLDS / 64, SURV_T_BIG>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    (void)hipGetLastError();
    configured = true;
  }
  if (a.N <= SURV_NLDS) {
    if (T == SURV_T_BIG)
      MV_LAUNCH((k_survive<SURV_NLDS / 64, SURV_T_BIG>), dim3(B), dim3(SURV_T_BIG), lds,
                         stream, a);
    else if (T == SURV_T_MID)
      MV_LAUNCH((k_survive<SURV_NLDS / 64, SURV_T_MID>), dim3(B), dim3(SURV_T_MID), lds,
                         stream, a);
    else
      MV_LAUNCH((k_survive<SURV_NLDS / 64, SURV_T>), dim3(B), dim3(SURV_T), lds, stream,
                         a);
  } else {
    if (!a.dom_g || a.dom_stride < (size_t)a.N * ((a.N + 63) / 64)) return hipErrorInvalidValue;
    MV_LAUNCH((k_survive<SURV_NMAX / 64, SURV_T_BIG>), dim3(B), dim3(SURV_T_BIG), lds,
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
  MV_LAUNCH(k_select, dim3(B), dim3(SURV_T), lds, stream, P, O, seed, sk,
                     gen, pop_slot, parents);
  return hipGetLastError();
}

hipError_t launch_init_pool(int B, int P, int O, int V, int S, const double* genes0, double* pool,
                            int* pop_slot, int* free_slot, hipStream_t stream) {
  MV_LAUNCH(k_init_pool, dim3(1024), dim3(256), 0, stream, B, P, O, V, S, genes0, pool,
                     pop_slot, free_slot);
  return hipGetLastError();
}

hipError_t launch_gather_pop(int B, int P, int V, int Vr, int S, const int* cmap,
                             const double* glr, const int* pop_slot, const double* pool,
                             const double* poolF, double* genes, double* F, hipStream_t stream) {
  MV_LAUNCH(k_gather_pop, dim3(2048), dim3(256), 0, stream, B, P, V, Vr, S, cmap, glr,
                     pop_slot, pool, poolF, genes, F);
  return hipGetLastError();
}

hipError_t launch_front(int B, int P, int V, int Vr, int S, const int* cmap, const double* glr,
                        const int* pop_slot, const double* pool, const double* poolF,
                        unsigned char* front, int* offsets, double* X, double* Fx,
                        hipStream_t stream) {
  if (B <= 0) return hipSuccess;
  if (P < 1 || P > 1024 || !front || !offsets) return hipErrorInvalidValue;
  MV_LAUNCH(k_front_mask, dim3(B), dim3(256), (size_t)P * 3 * sizeof(double), stream, P,
                     S, pop_slot, poolF, front, offsets);
  MV_LAUNCH(k_front_scan, dim3(1), dim3(1024), 0, stream, B, offsets);
  if (X || Fx)
    MV_LAUNCH(k_front_gather, dim3(B), dim3(256), 0, stream, P, V, Vr, S, cmap, glr,
                       pop_slot, pool, poolF, front, offsets, X, Fx);
  return hipGetLastError();
}

}  // namespace mv
