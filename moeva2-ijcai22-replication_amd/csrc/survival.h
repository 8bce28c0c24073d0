// R-NSGA-III survival of one initial state's merged population + the next tournament, as
// a workgroup-level device function (T threads): used by k_survive (one workgroup per
// state, survive.hip) and by the whole-attack kernel (attack.hip).
//
// Restates pymoo 0.4.2.2 (not vendored; [pymoo-recall]):
//   rnsga3.AspirationPointSurvival._do      ideal/worst, NDS, extreme points, nadir,
//                                           aspiration ref dirs, association, niching
//   NonDominatedSorting (fast_non_dominated_sort discovery order, n_stop_if_ranked)
//   nsga3.get_extreme_points_c / get_nadir_point / associate_to_niches / niching
//   TournamentSelection(comp_by_cv_then_random) (all CV == 0: random winner)
// with the dominance relation of src/attacks/moeva2/pareto_operation.py:35-51.
// Every floating-point expression keeps numpy's evaluation order (the library is built
// with -ffp-contract=off) so ranks, niches and survivors are bit-identical to
// oracle/moeva_oracle.py on identical objective arrays.
//
// Data: the merged population's F rows (LDS), a dominated-by bitset per individual
// (ceil(N/64) words), fronts as an ordered index array, niche CSR for the last front.
#pragma once
#include <limits.h>

#include "check.h"
#include "draws.h"
#include "engine.h"
#ifdef MV_CHECKS
namespace mv {
static __device__ int g_surv_dump_owner;
static __device__ double g_surv_dump[SURV_DUMP_N];
}  // namespace mv
#endif
#include "philox.h"
#include "wave.h"

namespace mv {

constexpr int SURV_TMAX = 1024;
// its first sweep's unroll (2: 104 VGPRs, two survival workgroups per CU; 1: 80, three)
#ifndef MV_ASSOC_UNROLL
#define MV_ASSOC_UNROLL 1
#endif  // largest survival workgroup (reduction scratch sizing)

struct SurvLds {
  double* F;        // [N*3]
  const double* ref;  // global: the reference points (read-only, L2-resident)      // [R*3]
  double* U;        // [(R+3)*3] normalised reference directions
  double4* Uf;      // [R+3] the same as double4 (association pre-filter)
  double* dist;     // [N]
  double* red;      // [waves*16] reduction scratch
  double* scal;     // [40] ideal(3) worst(3) wpop(3) . prev ext(9) at 24
  double* wsc;      // [waves*16] each wave's own wfront(3) nadir(3) ext(9)
  unsigned long long* dom;     // [N*NW]
  unsigned long long* ranked;  // [NW]
  unsigned long long* cur;     // [NW]
  int* I;           // [N] fronts concatenated
  int* pos;         // [N] position in own front
  int* front_of;    // [N]
  int* slot;        // [N]
  int* niche;       // [N]
  int* memb;        // [N]
  int* key;         // [N]
  int* surv;        // [N]
  int* sel;         // [N]
  int* fstart;      // [N+2]
  int* count;       // [R+3]
  int* remain;      // [R+3]
  int* csr_off;     // [R+4]
  int* csr;         // [N]
  int* cand;        // [R+3]
  int* ckey;        // [R+3]
  int* iscal;       // [16 + SURV_TMAX / 64]: scalars [0, 16), block-scan wave sums after
  unsigned long long* sortk;  // [max(N, n_perm_slots)] sort keys
  int* perm;        // [n_perm_slots]
  unsigned long long* dmin;  // [R+3]
  int* lround;      // [2N+2] round index of each level
};

__host__ __device__ inline size_t align16(size_t x) { return (x + 15) & ~(size_t)15; }

__host__ __device__ __forceinline__ int pow2_at_least(int n) {
  int p = 1;
  while (p < n) p <<= 1;
  return p;
}

// Ascending bitonic sort of n (a power of two) 64-bit keys in LDS by the whole workgroup;
// ends on a barrier.
template <int T>
__device__ __forceinline__ void bitonic_sort_u64(unsigned long long* k, int n) {
  for (int size = 2; size <= n; size <<= 1)
    for (int stride = size >> 1; stride > 0; stride >>= 1) {
      for (int t = threadIdx.x; t < (n >> 1); t += T) {
        const int i = 2 * t - (t & (stride - 1));  // pair (i, i + stride), bit stride of i clear
        const int j = i + stride;
        const unsigned long long x = k[i], y = k[j];
        if ((x > y) == ((i & size) == 0)) {
          k[i] = y;
          k[j] = x;
        }
      }
      __syncthreads();
    }
}

// Niching ranks the last front's members inside their niches by counting over each niche's
// members: quadratic in a niche's size.  When one niche holds more than this many members
// (the first generations, whose population is copies of one initial state, put the whole
// last front into one niche: 101 k cycles per state at configs[3], N = 963), one bitonic
// sort of all the keys replaces the counting (~7 k cycles at 1024 keys).  Only the N >
// SURV_NLDS instance, whose sort-key array is a power of two long.
constexpr int NICHE_SORT_MIN = 256;

// Byte offsets of the survival workspace inside the dynamic LDS block.
struct SurvOff {
  unsigned F, ref, U, Uf, dist, red, scal, wsc, dom, ranked, cur, I, pos, front_of, slot, niche, memb,
      key, surv, sel, fstart, count, remain, csr_off, csr, cand, ckey, iscal, sortk, perm,
      dmin, lround, ptab, total;
};

// Niching's temporaries (count, remain, csr_off, csr, cand, ckey, dmin, lround) are dead
// before the NDS ends and the dominance bitsets after it, so when the bitsets live in LDS
// (N <= SURV_NLDS) and the temporaries fit inside them they share those bytes; the
// reference points are read from global memory (L2-resident, the same for every state).
// Round 4: 68.8 -> ~53 KiB per workgroup at N = 303, R = 200 (three workgroups per CU).
// ptab_words: the variation plan's tables (geo, cmap, ginfo; 0 without a plan), staged after
// survivor selection into the F rows when they fit (F is dead then), else appended.
// Threads of the survival workgroup for N merged individuals (the kernel instance's T).
__host__ __device__ __forceinline__ int surv_threads(int N) {
  return N > SURV_NLDS ? SURV_T_BIG : SURV_T;
}

__host__ __device__ __forceinline__ SurvOff surv_offsets(int N, int R, int Pperm,
                                                         int ptab_words = 0, int threads = 0) {
  const bool dom_lds = N <= SURV_NLDS;
  const unsigned NW = (N + 63) / 64;
  const unsigned RN = R + 3;
  SurvOff o;
  unsigned off = 0;
#define TAKE(field, bytes)        \
  o.field = off;                  \
  off = (unsigned)align16(off + (size_t)(bytes));
  TAKE(F, (size_t)NW * 64 * 3 * 8)  // rows past N hold NaN (dominance padding)
  o.ref = 0;                        // unused: a.ref in global memory
  TAKE(U, (size_t)RN * 3 * 8)
  TAKE(Uf, (size_t)RN * 32)  // unit directions as double4 (association pre-filter)
  TAKE(dist, (size_t)N * 8)
  TAKE(red, ((threads ? threads : surv_threads(N)) / 64) * 16 * 8)
  TAKE(scal, 40 * 8)
  TAKE(wsc, ((threads ? threads : surv_threads(N)) / 64) * 16 * 8)
  TAKE(dom, dom_lds ? (size_t)N * NW * 8 : 0)
  TAKE(ranked, NW * 8)
  TAKE(cur, NW * 8)
  TAKE(I, N * 4)
  TAKE(pos, N * 4)
  TAKE(front_of, N * 4)
  TAKE(slot, N * 4)
  TAKE(niche, N * 4)
  TAKE(memb, N * 4)
  TAKE(key, N * 4)
  TAKE(surv, N * 4)
  TAKE(sel, N * 4)
  TAKE(fstart, (N + 2) * 4)
  TAKE(iscal, (16 + SURV_TMAX / 64) * 4)
  // the sort keys; above SURV_NLDS a power of two for niching's bitonic sort (NICHE_SORT_MIN)
  const int nsk = N > SURV_NLDS ? pow2_at_least(N) : N;
  TAKE(sortk, (size_t)(nsk > Pperm ? nsk : Pperm) * 8)
  TAKE(perm, (size_t)Pperm * 4)
  const unsigned end = off;
  // the niching temporaries: inside the dominance bitsets when they fit, else appended
  auto tsize = [&]() {
    unsigned t = 0;
    for (size_t b : {(size_t)RN * 4, (size_t)RN * 4, (size_t)(RN + 1) * 4, (size_t)N * 4,
                     (size_t)RN * 4, (size_t)RN * 4, (size_t)RN * 8, (size_t)(2 * N + 2) * 4})
      t = (unsigned)align16(t + b);
    return t;
  };
  const bool alias = dom_lds && tsize() <= (unsigned)((size_t)N * NW * 8);
  off = alias ? o.dom : end;
  TAKE(count, RN * 4)
  TAKE(remain, RN * 4)
  TAKE(csr_off, (RN + 1) * 4)
  TAKE(csr, N * 4)
  TAKE(cand, RN * 4)
  TAKE(ckey, RN * 4)
  TAKE(dmin, (size_t)RN * 8)
  TAKE(lround, (size_t)(2 * N + 2) * 4)
  unsigned total = alias ? end : off;
  if (ptab_words > 0 && (size_t)ptab_words * 4 > (size_t)NW * 64 * 3 * 8) {
    off = total;
    TAKE(ptab, (size_t)ptab_words * 4)
    total = off;
  } else {
    o.ptab = o.F;
  }
#undef TAKE
  o.total = total;
  return o;
}


__device__ __forceinline__ double min_prop(double a, double b) {  // np.min (NaN propagates)
  double r = b < a ? b : a;
  r = b != b ? b : r;
  return a != a ? a : r;
}
__device__ __forceinline__ double max_prop(double a, double b) {
  double r = b > a ? b : a;
  r = b != b ? b : r;
  return a != a ? a : r;
}

// np.argmin order: first NaN, else smallest value, ties -> smallest index
__device__ __forceinline__ bool arg_better(double v, int i, double bv, int bi) {
  const bool vn = v != v, bn = bv != bv;
  if (vn || bn) return (vn && bn) ? (i < bi) : vn;
  return v < bv || (v == bv && i < bi);
}

// Ordered stream compaction of the indices i in [0, n) with pred(i) into out[base..].
// Returns the count (uniform).  Uses red scratch as int[4+1].
// One row j = j0 + U of a dominance work item against the wave's 64 rows i (lane = i), with
// the relation of pareto_operation.py:35-51: lt = F_i < F_j in some objective, ng = F_i > F_j
// in none (ULE: a NaN padding row compares false both ways).  The compares' lane masks stay
// in SGPRs (v_cmp -> s_or / s_and, no bool -> VGPR -> mask round trip): m = lt & ng (lanes i
// that dominate j) goes to lane U of mine with v_writelane (immediate lane, so no lane-select
// hazard), d = ~(lt | ng) (j dominates lane i) sets bit U of the lane's acc.
template <int U>
__device__ __forceinline__ unsigned writelane_u(unsigned old, unsigned v) {
  unsigned r = old;
  asm("v_writelane_b32 %0, %1, %2" : "+v"(r) : "s"(v), "i"(U));
  return r;
}
// lanes set in the uniform mask m take b, the others a (one v_cndmask on the SGPR pair)
__device__ __forceinline__ unsigned select_mask(unsigned a, unsigned b, unsigned long long m) {
  unsigned r;
  asm("v_cndmask_b32_e64 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "s"(m));
  return r;
}
template <int U, int NU, class Acc>
struct DomRow {
  __device__ __forceinline__ static void run(double fi0, double fi1, double fi2, const double* fj,
                                             unsigned& mlo, unsigned& mhi, Acc& acc, int lane) {
    const double g0 = fj[U * 3], g1 = fj[U * 3 + 1], g2 = fj[U * 3 + 2];
    constexpr int OLT = 4, ULE = 13;  // llvm FCmp predicates: ordered <, unordered or <=
    const unsigned long long lt = __builtin_amdgcn_fcmp(fi0, g0, OLT) |
                                  __builtin_amdgcn_fcmp(fi1, g1, OLT) |
                                  __builtin_amdgcn_fcmp(fi2, g2, OLT);
    const unsigned long long ng = __builtin_amdgcn_fcmp(fi0, g0, ULE) &
                                  __builtin_amdgcn_fcmp(fi1, g1, ULE) &
                                  __builtin_amdgcn_fcmp(fi2, g2, ULE);
    const unsigned long long m = lt & ng;
    const unsigned long long d = ~(lt | ng);
    mlo = writelane_u<U>(mlo, (unsigned)m);
    mhi = writelane_u<U>(mhi, (unsigned)(m >> 32));
    if constexpr (U < 32) {
      const unsigned lo = (unsigned)acc;
      acc = (acc & ~(Acc)0xFFFFFFFFu) | (Acc)select_mask(lo, lo | (1u << U), d);
    } else {
      const unsigned hi = (unsigned)((unsigned long long)acc >> 32);
      acc = (acc & (Acc)0xFFFFFFFFu) |
            ((Acc)select_mask(hi, hi | (1u << (U - 32)), d) << 32);
    }
    DomRow<U + 1, NU, Acc>::run(fi0, fi1, fi2, fj, mlo, mhi, acc, lane);
  }
};
template <int NU, class Acc>
struct DomRow<NU, NU, Acc> {
  __device__ __forceinline__ static void run(double, double, double, const double*, unsigned&,
                                             unsigned&, Acc&, int) {}
};

template <int T, class Pred>
__device__ __forceinline__ int block_compact(int n, Pred pred, int* out, int base, int* wsum) {
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  int total = 0;
  for (int b0 = 0; b0 < n; b0 += T) {
    const int i = b0 + tid;
    const bool f = i < n && pred(i);
    const unsigned long long m = __ballot(f);
    const int before = __popcll(m & ((1ull << lane) - 1ull));
    if (lane == 0) wsum[wave] = __popcll(m);
    __syncthreads();
    int woff = 0, all = 0;
    for (int w = 0; w < T / 64; ++w) {
      if (w < wave) woff += wsum[w];
      all += wsum[w];
    }
    if (f) out[base + total + woff + before] = i;
    total += all;
    __syncthreads();
  }
  return total;
}

// Exclusive prefix sum of v[0, n) in place (LDS); returns the total (uniform).
template <int T>
__device__ __forceinline__ int block_scan_excl(int* v, int n, int* wsum) {
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  int carry = 0;
  for (int b0 = 0; b0 < n; b0 += T) {
    const int i = b0 + tid;
    const int x = i < n ? v[i] : 0;
    int incl = x;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const int y = __shfl_up(incl, o, 64);
      if (lane >= o) incl += y;
    }
    if (lane == 63) wsum[wave] = incl;
    __syncthreads();
    int woff = 0, tot = 0;
#pragma unroll
    for (int w = 0; w < T / 64; ++w) {
      const int sw = wsum[w];
      if (w < wave) woff += sw;
      tot += sw;
    }
    if (i < n) v[i] = carry + woff + incl - x;
    carry += tot;
    __syncthreads();
  }
  return carry;
}

// v_min_f32 without the NaN canonicalisation the compiler adds for fminf (finite operands)
__device__ __forceinline__ float vmin_f32(float a, float b) {
  float r;
  asm("v_min_f32 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
  return r;
}

__device__ __forceinline__ double wred_min(double v) {
  return wave_reduce(v, [](double a, double b) { return min_prop(a, b); });
}
__device__ __forceinline__ double wred_max(double v) {
  return wave_reduce(v, [](double a, double b) { return max_prop(a, b); });
}
// LAPACK dgetf2/dgetrs-order 3x3 solve (oracle lu_solve3).  Returns false if singular.
// Every array index is a compile-time constant after unrolling (the pivot row is swapped in
// by selects, not by a runtime index), so A and x stay in registers: indexing them by the
// pivot put both in scratch memory, ~10 k cycles of the nadir step per state.
__device__ __forceinline__ bool lu_solve3(double (&A)[3][3], double (&x)[3]) {
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    int p = k;
    double best = fabs(A[k][k]);
#pragma unroll
    for (int i = k + 1; i < 3; ++i) {
      const double v = fabs(A[i][k]);
      if (v > best) {
        best = v;
        p = i;
      }
    }
    double piv = A[k][k];
#pragma unroll
    for (int i = k + 1; i < 3; ++i) piv = p == i ? A[i][k] : piv;
    if (piv == 0.0) return false;
#pragma unroll
    for (int i = k + 1; i < 3; ++i) {
      const bool sw = p == i;
#pragma unroll
      for (int j = 0; j < 3; ++j) {
        const double t = A[k][j];
        A[k][j] = sw ? A[i][j] : t;
        A[i][j] = sw ? t : A[i][j];
      }
      const double t = x[k];
      x[k] = sw ? x[i] : t;
      x[i] = sw ? t : x[i];
    }
    const double r = 1.0 / A[k][k];
#pragma unroll
    for (int i = k + 1; i < 3; ++i) A[i][k] = A[i][k] * r;
#pragma unroll
    for (int j = k + 1; j < 3; ++j)
#pragma unroll
      for (int i = k + 1; i < 3; ++i) A[i][j] = A[i][j] - A[i][k] * A[k][j];
  }
#pragma unroll
  for (int j = 0; j < 3; ++j)
#pragma unroll
    for (int i = j + 1; i < 3; ++i) x[i] = x[i] - x[j] * A[i][j];
#pragma unroll
  for (int j = 2; j >= 0; --j) {
    x[j] = x[j] / A[j][j];
#pragma unroll
    for (int i = 0; i < j; ++i) x[i] = x[i] - x[j] * A[i][j];
  }
  return true;
}

// Tournament selection for the next generation (oracle tournament_parents).
template <int T>
__device__ __forceinline__ void tournament(int P, int O_next, uint64_t seed, uint32_t sk, int gen,
                           const int* map_slot, int* out, unsigned long long* sortk,
                           int* perm, int* lds_out = nullptr) {
  const int tid = threadIdx.x;
  const int n_m = (O_next + 1) / 2;
  const int n_random = n_m * 4;
  const int n_perms = (n_random + P - 1) / P;
  const int n = n_perms * P;
  const Rng rng(seed, sk);
  int ib = 1;  // bits of the index field
  while ((1 << ib) < P) ++ib;
  const unsigned long long imask = (1ull << ib) - 1ull;
  // permutation q = argsort of its P keys (ties by index): rank of each (key, i) composite
  // among the P composites of its own permutation
  for (int idx = tid; idx < n; idx += T) {
    const int q = idx / P, i = idx - q * P;
    const unsigned key = rng.draw((uint32_t)idx, (uint32_t)gen, TAG_SEL_PERM).x;
    sortk[idx] = ((unsigned long long)key << ib) | (unsigned)i;
  }
  __syncthreads();
  for (int idx = tid; idx < n; idx += T) {
    const int q = idx / P;
    const unsigned long long kp = sortk[idx];
    const unsigned long long* kq = sortk + (size_t)q * P;
    int r = 0;
    for (int j = 0; j < P; ++j) r += kq[j] < kp ? 1 : 0;
    perm[q * P + r] = (int)(kp & imask);
  }
  __syncthreads();
  for (int t = tid; t < 2 * n_m; t += T) {
    const int a = perm[2 * t], b = perm[2 * t + 1];
    const unsigned bit = rng.draw((uint32_t)t, (uint32_t)gen, TAG_SEL_CHOICE).x & 1u;
    const int w = bit ? b : a;
    const int v = map_slot ? map_slot[MV_IDX(w, P, CK_SURV_PARENT)] : w;
    out[t] = v;
    if (lds_out) lds_out[t] = v;  // the sort keys are dead after the rank pass's barrier
  }
}

// The next generation's variation plan (engine.h VPlan) of state b, with every thread: (1)
// the matings' crossover draws (cx_sub, item 2 m + subset) into LDS cxs; (2) the mutations:
// four lanes per offspring row i (lanes 4 k + q of a wave; T is a multiple of 64, so a group
// never straddles waves), lane q taking draw q of the row's geometric-gap walk over the Vr
// genes (Philox index i * MUT_J + q, TAG_MUT_MASK) -- the same draws and positions as walking
// them one after another (prefix sums of the 1 + gap steps inside the group), in one round;
// a position maps to its stored gene (a fixed gene's draw is consumed, nothing is written)
// and the row's stored hits take the plan's slots in draw order.  A row whose fourth
// position is still inside the genes is finished by its lane 3, serially (2 % of the rows);
// more than PLAN_MUT stored mutations set the overflow flag.  par: the tournament's parents
// (LDS, 2 per mating); geo / cmap / ginfo: LDS.
// MV_PLAN_CAP (checks / test builds only): the stored mutations a plan row may hold before
// it is flagged as overflowing (default PLAN_MUT).  A small cap (`make planovf`: 1) sends most
// mutated rows through k_genc's overflow paths, which a PLAN_MUT of 8 reaches about once per
// million rows, so their bit-parity can be tested (tests/test_gpu_parity.py).
#ifndef MV_PLAN_CAP
#define MV_PLAN_CAP PLAN_MUT
#endif
static_assert(MV_PLAN_CAP >= 1 && MV_PLAN_CAP <= PLAN_MUT, "plan cap within the plan's slots");
template <int T>
__device__ __forceinline__ void variation_plan(const SurvArgs& a, const int b, const int gen,
                                               const int* par, int* cxs, const uint32_t* geo,
                                               const int* cmap, const int* ginfo) {
  static_assert(T % 64 == 0, "variation_plan: groups of four lanes inside a wave");
  const int n = a.O_next, nm = n / 2;
  const int tid = threadIdx.x, lane = tid & 63;
  const Rng rng(a.seed, state_stream(a.stream_key, a.state_keys, a.key0, b));
  for (int t = tid; t < 2 * nm; t += T) {
    int c = pack_cx(cx_sub(rng, gen, t >> 1, t & 1, (t & 1) ? a.n_sub1 : a.n_sub0, a.cx_prob));
    if (a.cx_sbx) c &= 1;
    cxs[t] = c;
  }
  __syncthreads();
  const int Vr = a.Vr;
  const float lq = __log2f(1.0f - 1.0f / (float)Vr);
  for (int t0 = 0; t0 < 4 * n; t0 += T) {  // uniform trip count
    const int t = t0 + tid;
    const bool live = t < 4 * n;
    const int i = live ? t >> 2 : 0, q = t & 3;
    const int m = i % nm, side = i / nm;
    int st = 0;
    double uq = 0.0;
    if (live) {
      const u32x4 w = rng.draw((uint32_t)(i * MUT_J + q), (uint32_t)gen, TAG_MUT_MASK);
      st = 1 + geo_gap(geo, Vr, w.x, lq);
      uq = u53(w.y, w.z);
    }
    {
      const int t1 = __shfl(st, (lane + 63) & 63);
      st += q >= 1 ? t1 : 0;
      const int t2 = __shfl(st, (lane + 62) & 63);
      st += q >= 2 ? t2 : 0;
    }
    const int pos = st - 1;  // position of draw q (increasing in q)
    const bool hit = live && pos < Vr;
    const int cq = hit ? cmap[pos] : -1;
    const bool stored = cq >= 0;
    const unsigned long long sm = __ballot(stored);
    const unsigned grp = (unsigned)((sm >> (lane & ~3)) & 0xFull);
    const int slot = __popc(grp & ((1u << q) - 1u));  // stored hits before this lane's
    const int c0 = cxs[2 * m], c1 = cxs[2 * m + 1];
    int* mw = a.plan_mw + ((size_t)b * n + i) * PLAN_MUT;
    double* mu = a.plan_mu + ((size_t)b * n + i) * PLAN_MUT;
    auto put = [&](int k, int g, double u) {
      const int gi = ginfo[MV_IDX(g, a.V, CK_GEN_MUTPOS)];
      const int oth = (!a.cx_sbx && swapped_packed(gi, c0, c1)) ? 1 : 0;
      mw[k] = g | (((gi & 3) == 0 ? 1 : 0) << 16) | (oth << 17);
      mu[k] = u;
    };
    if (stored) put(slot, cq, uq);
    if (live && q == 3) {  // the row's count (and the rare rest of its walk), then its header
      int cnt = __popc(grp), ovf = cnt > MV_PLAN_CAP ? 1 : 0;
      if (hit && !ovf) {
        int p = pos;
        for (int j = 4;; ++j) {
          const u32x4 w = rng.draw((uint32_t)(i * MUT_J + j), (uint32_t)gen, TAG_MUT_MASK);
          p += 1 + geo_gap(geo, Vr, w.x, lq);
          if (p >= Vr) break;
          const int g = cmap[p];
          if (g < 0) continue;
          if (cnt >= MV_PLAN_CAP) {
            ovf = 1;
            break;
          }
          put(cnt, g, u53(w.y, w.z));
          ++cnt;
        }
      }
      const int p0 = par[2 * m], p1 = par[2 * m + 1];
      const int pv = side ? (p1 | (p0 << 16)) : (p0 | (p1 << 16));
      a.plan_hdr[(size_t)b * n + i] = make_int4(pv, c0, c1, cnt | (ovf << 4));
    }
  }
}

// NWMAX: dominance words per individual held in registers (N <= 64 NWMAX); above
// SURV_NLDS the bitsets go to the HBM scratch a.dom_g instead of LDS.
// a: pointers and sizes (slot or dense mode); b: the state; N, gen, sel_gen and
// parents_out (NULL: no next tournament) vary per generation in the whole-attack kernel.
template <int NWMAX, int T>
__device__ __forceinline__ void survive_state(const SurvArgs& a, const int b, const int N,
                                              const int gen, const int sel_gen,
                                              int* const parents_out, unsigned char* smem) {
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int R = a.R, RN = R + 3;
  const int NW = (N + 63) / 64;
  const int n_m_next = parents_out ? (a.O_next + 1) / 2 : 0;
  const int pslots = parents_out ? ((n_m_next * 4 + a.n_survive - 1) / a.n_survive) * a.n_survive : 1;
  const bool plan = parents_out && a.plan_hdr;
  const SurvOff o = surv_offsets(N, R, pslots, a.plan_hdr ? plan_tab_words(a.Vr, a.V) : 0, T);
  SurvLds L;
  L.F = (double*)(smem + o.F);
  L.ref = a.ref;  // global (surv_offsets)
  L.U = (double*)(smem + o.U);
  L.Uf = (double4*)(smem + o.Uf);
  L.dist = (double*)(smem + o.dist);
  L.red = (double*)(smem + o.red);
  L.scal = (double*)(smem + o.scal);
  L.wsc = (double*)(smem + o.wsc);
  if (NWMAX * 64 > SURV_NLDS)
    L.dom = a.dom_g + (size_t)b * a.dom_stride;
  else
    L.dom = (unsigned long long*)(smem + o.dom);
  L.ranked = (unsigned long long*)(smem + o.ranked);
  L.cur = (unsigned long long*)(smem + o.cur);
  L.I = (int*)(smem + o.I);
  L.pos = (int*)(smem + o.pos);
  L.front_of = (int*)(smem + o.front_of);
  L.slot = (int*)(smem + o.slot);
  L.niche = (int*)(smem + o.niche);
  L.memb = (int*)(smem + o.memb);
  L.key = (int*)(smem + o.key);
  L.surv = (int*)(smem + o.surv);
  L.sel = (int*)(smem + o.sel);
  L.fstart = (int*)(smem + o.fstart);
  L.count = (int*)(smem + o.count);
  L.remain = (int*)(smem + o.remain);
  L.csr_off = (int*)(smem + o.csr_off);
  L.csr = (int*)(smem + o.csr);
  L.cand = (int*)(smem + o.cand);
  L.ckey = (int*)(smem + o.ckey);
  L.iscal = (int*)(smem + o.iscal);
  L.sortk = (unsigned long long*)(smem + o.sortk);
  L.perm = (int*)(smem + o.perm);
  L.dmin = (unsigned long long*)(smem + o.dmin);
  L.lround = (int*)(smem + o.lround);
  double* ideal = L.scal;
  double* worst = L.scal + 3;
  double* wpop = L.scal + 6;
  // the front's worst point, the nadir and the extremes: every wave computes the same bits
  // (below) into its OWN copy and reads only that one, so no two waves write one LDS word
  double* wfront = L.wsc + (tid >> 6) * 16;
  double* nadir = wfront + 3;
  double* ext = wfront + 6;  // 9
  double* pext = L.scal + 24;  // 9: the carried extremes, staged at entry
  const int has_ext = a.has_extreme[b] != 0;
  // carried ideal / worst, loaded at entry so their latency overlaps the F load
  const double pre_ideal = tid < 3 ? a.ideal[(size_t)b * 3 + tid] : 0.0;
  const double pre_worst = tid < 3 ? a.worst[(size_t)b * 3 + tid] : 0.0;
  const bool slot_mode = a.pop_slot != nullptr;
#define PHASE(k) \
  if (MV_CLOCKS && a.phase && tid == 0) a.phase[(size_t)b * 32 + (k)] = clock64();
  PHASE(0)

  // ---- load merged F, ref points
  for (int m = tid; m < N; m += T) {
    int s = m;
    const double* src;
    if (slot_mode) {
      s = m < a.P ? a.pop_slot[(size_t)b * a.P + m] : a.free_slot[(size_t)b * a.O + (m - a.P)];
      s = MV_IDX(s, a.S, CK_SURV_SLOT);
      src = a.F + ((size_t)b * a.S + s) * 3;
    } else {
      src = a.F + ((size_t)b * N + m) * 3;
    }
    const double f0 = src[0], f1 = src[1], f2 = src[2];
    L.F[m * 3 + 0] = f0;
    L.F[m * 3 + 1] = f1;
    L.F[m * 3 + 2] = f2;
    L.slot[m] = s;
    L.front_of[m] = -1;
    L.sel[m] = 0;
  }
  for (int m = N + tid; m < NW * 64; m += T) {  // padding rows: compare false both ways
    L.F[m * 3 + 0] = __builtin_nan("");
    L.F[m * 3 + 1] = __builtin_nan("");
    L.F[m * 3 + 2] = __builtin_nan("");
  }
  if (tid < 9) pext[tid] = a.extreme[(size_t)b * 9 + tid];
  if (tid == 0) L.iscal[14] = 0;  // dominance work counter
  for (int q = tid; q < NW; q += T) {
    L.ranked[q] = 0ull;
    L.cur[q] = 0ull;
  }
  __syncthreads();
  PHASE(1)

  // ---- ideal / worst (np.min/np.max over vstack(prev, F, ref)), worst of population: wave
  // 0, before it joins the dominance pass below (independent of it; its results are first
  // read after the pass's barrier).  min/max of these values do not depend on the reduction
  // order (NaN propagates either way; no -0.0 objective exists: f1 is a probability, f2 a
  // sqrt, f3 a sum starting at +0.0).
  if (wave == 0) {
    double mn[3], mx[3], wp[3];
    for (int k = 0; k < 3; ++k) {
      mn[k] = __builtin_inf();
      mx[k] = -__builtin_inf();
      wp[k] = -__builtin_inf();
    }
    for (int m = lane; m < N; m += 64)
      for (int k = 0; k < 3; ++k) {
        const double v = L.F[m * 3 + k];
        mn[k] = min_prop(mn[k], v);
        mx[k] = max_prop(mx[k], v);
        wp[k] = max_prop(wp[k], v);
      }
    for (int r = lane; r < R; r += 64)
      for (int k = 0; k < 3; ++k) {
        const double v = L.ref[r * 3 + k];
        mn[k] = min_prop(mn[k], v);
        mx[k] = max_prop(mx[k], v);
      }
    for (int k = 0; k < 3; ++k) {
      mn[k] = wred_min(mn[k]);
      mx[k] = wred_max(mx[k]);
      wp[k] = wred_max(wp[k]);
    }
    if (lane < 3) {
      const int k = lane;
      double vmn = mn[0], vmx = mx[0], vwp = wp[0];
      if (k == 1) {
        vmn = mn[1];
        vmx = mx[1];
        vwp = wp[1];
      } else if (k == 2) {
        vmn = mn[2];
        vmx = mx[2];
        vwp = wp[2];
      }
      ideal[k] = min_prop(pre_ideal, vmn);
      worst[k] = max_prop(pre_worst, vmx);
      wpop[k] = vwp;
    }
  }
  PHASE(11)

  // ---- dominance bitsets, word-major: bit i - 64 q of dom[q N + j]  <=>  i dominates j
  // (lanes j read and write consecutive words).  Work items are the unordered 64x64 block
  // pairs (qi <= qj) split into the four 16-row quarters of block qj, taken from an LDS
  // counter (wave 0 joins after ideal/worst).  Lane l holds row i = 64 qi + l;
  // the 16 rows j of the quarter are LDS broadcasts, fully unrolled (F is padded to whole
  // blocks with NaN rows, which compare false both ways: no bounds tests).  One pass of
  // the six compares per (i, j) gives both directions: lt && !gt -> i dominates j (the
  // ballot is word qi of dom[j], kept by lane u); gt && !lt -> j dominates
  // i, bit u of this lane's 16-bit quarter qq of word qj of dom[i] (off-diagonal pairs
  // only: the diagonal block is covered by its ballots).
  if (NWMAX * 64 > SURV_NLDS) {
    // HBM bitsets: whole 64 x 64 block pairs, so both directions leave as full words in
    // the word-major layout (dom[q N + j]): lane u's ballot word qi of dom[j0 + u] and lane
    // l's 64-bit word qj of dom[i] are 512 contiguous bytes each (the quarter items' 2-byte
    // stores to rows 128 B apart cost 28.8 GB of HBM traffic per configs[3] launch)
    const int n_b = NW * (NW + 1) / 2;
    for (;;) {
      int t = 0;
      if (lane == 0) t = atomicAdd(&L.iscal[14], 1);
      t = __builtin_amdgcn_readfirstlane(t);  // lane 0 is the first active lane
      if (t >= n_b) break;
      int qi = 0, rem = t;
      while (rem >= NW - qi) {
        rem -= NW - qi;
        ++qi;
      }
      const int qj = qi + rem;
      const int i = qi * 64 + lane;
      const double fi0 = L.F[i * 3 + 0], fi1 = L.F[i * 3 + 1], fi2 = L.F[i * 3 + 2];
      const int j0 = qj * 64;
      const double* fj = L.F + j0 * 3;
      unsigned mlo = 0u, mhi = 0u;
      unsigned long long acc = 0ull;
      DomRow<0, 64, unsigned long long>::run(fi0, fi1, fi2, fj, mlo, mhi, acc, lane);
      const unsigned long long mine = ((unsigned long long)mhi << 32) | mlo;
      if (j0 + lane < N) L.dom[(size_t)qi * N + j0 + lane] = mine;
      if (qi != qj && i < N) L.dom[(size_t)qj * N + i] = acc;
    }
  } else {
    unsigned short* dom16 = (unsigned short*)L.dom;
    const int n_q = NW * (NW + 1) * 2;  // block pairs x 4 quarters
    for (;;) {
      int t = 0;
      if (lane == 0) t = atomicAdd(&L.iscal[14], 1);
      t = __builtin_amdgcn_readfirstlane(t);  // lane 0 is the first active lane
      if (t >= n_q) break;
      const int qq = t & 3;
      int qi = 0, rem = t >> 2;
      while (rem >= NW - qi) {
        rem -= NW - qi;
        ++qi;
      }
      const int qj = qi + rem;
      const int i = qi * 64 + lane;
      const double fi0 = L.F[i * 3 + 0], fi1 = L.F[i * 3 + 1], fi2 = L.F[i * 3 + 2];
      const int j0 = qj * 64 + qq * 16;
      const double* fj = L.F + j0 * 3;
      unsigned mlo = 0u, mhi = 0u, acc = 0u;
      DomRow<0, 16, unsigned>::run(fi0, fi1, fi2, fj, mlo, mhi, acc, lane);
      const unsigned long long mine = ((unsigned long long)mhi << 32) | mlo;
      if (lane < 16 && j0 + lane < N)
        L.dom[(size_t)qi * N + j0 + lane] = mine;
      if (qi != qj && i < N) dom16[((size_t)qj * N + i) * 4 + qq] = (unsigned short)acc;
    }
  }
  __syncthreads();
  PHASE(2)

  // ---- fast non-dominated sort (discovery order), stop once >= n_survive ranked
  int* wsum = L.iscal + 16;  // one int per wave (iscal[15] is the association counter)
  int n0 = block_compact<T>(
      N,
      [&](int j) {
        for (int q = 0; q < NW; ++q)
          if (L.dom[(size_t)q * N + j]) return false;
        return true;
      },
      L.I, 0, wsum);
  for (int k = tid; k < n0; k += T) {
    const int j = L.I[k];
    L.pos[j] = k;
    L.front_of[j] = 0;
    atomicOr(&L.ranked[j >> 6], 1ull << (j & 63));
    atomicOr(&L.cur[j >> 6], 1ull << (j & 63));
  }
  if (tid == 0) {
    L.fstart[0] = 0;
    L.fstart[1] = n0;
  }
  __syncthreads();
  int cum = n0, nf = 1;
  while (cum < a.n_survive && cum < N) {
    const int nc = block_compact<T>(
        N,
        [&](int j) {
          if ((L.ranked[j >> 6] >> (j & 63)) & 1ull) return false;
          for (int q = 0; q < NW; ++q)
            if (L.dom[(size_t)q * N + j] & ~L.ranked[q]) return false;
          return true;
        },
        L.memb, 0, wsum);
    if (nc == 0) break;  // unreachable for an acyclic dominance relation
    for (int k = tid; k < nc; k += T) {
      const int j = L.memb[k];
      int mx = -1;
      for (int q = 0; q < NW; ++q) {
        unsigned long long bits = L.dom[(size_t)q * N + j] & L.cur[q];
        while (bits) {
          const int i = q * 64 + __ffsll((long long)bits) - 1;
          bits &= bits - 1ull;
          mx = L.pos[i] > mx ? L.pos[i] : mx;
        }
      }
      L.key[k] = mx * N + j;
    }
    __syncthreads();
    for (int k = tid; k < nc; k += T) {
      const int kk = L.key[k];
      int r = 0;
      for (int t = 0; t < nc; ++t) r += L.key[t] < kk;
      L.I[cum + r] = L.memb[k];
    }
    for (int q = tid; q < NW; q += T) L.cur[q] = 0ull;
    __syncthreads();
    for (int k = tid; k < nc; k += T) {
      const int j = L.I[cum + k];
      L.pos[j] = k;
      L.front_of[j] = nf;
      atomicOr(&L.ranked[j >> 6], 1ull << (j & 63));
      atomicOr(&L.cur[j >> 6], 1ull << (j & 63));
    }
    cum += nc;
    ++nf;
    if (tid == 0) L.fstart[nf] = cum;
    __syncthreads();
  }
  const int n_ranked = cum;
  PHASE(3)

  // ---- extreme points (ASF over prev extremes + front 0 + ref points), worst of front
  {
    const int ne = has_ext ? 3 : 0;
    const int ncand = ne + n0 + R;
    double bv[3];
    int bi[3];
    double wf[3];
    for (int k = 0; k < 3; ++k) {
      bv[k] = __builtin_inf();
      bi[k] = INT_MAX;
      wf[k] = -__builtin_inf();
    }
    for (int c = tid; c < ncand; c += T) {
      double row[3];
      if (c < ne) {
        for (int k = 0; k < 3; ++k) row[k] = pext[c * 3 + k];
      } else if (c < ne + n0) {
        const int m = L.I[c - ne];
        for (int k = 0; k < 3; ++k) {
          row[k] = L.F[m * 3 + k];
          wf[k] = max_prop(wf[k], row[k]);
        }
      } else {
        for (int k = 0; k < 3; ++k) row[k] = L.ref[(c - ne - n0) * 3 + k];
      }
      double d[3];
      for (int k = 0; k < 3; ++k) {
        d[k] = row[k] - ideal[k];
        if (d[k] < 1e-3) d[k] = 0.0;
      }
      for (int i = 0; i < 3; ++i) {
        double asf = -__builtin_inf();
        for (int k = 0; k < 3; ++k) asf = max_prop(asf, d[k] * (i == k ? 1.0 : 1e6));
        if (arg_better(asf, c, bv[i], bi[i])) {
          bv[i] = asf;
          bi[i] = c;
        }
      }
    }
    PHASE(21)
    // One packed reduction for the three argmins and the front's worst point, ONE barrier,
    // then every wave combines the eight waves' partials and solves the nadir itself (the
    // same bits in every wave), so no thread waits for a single-thread step.  The ASF values
    // are >= +0, +inf or NaN: np.argmin's order (first NaN, else smallest value, ties the
    // smallest index) is the lexicographic minimum of (NaN ? -1 : value, index), i.e. a
    // v_min_f64 reduction of the keys, then a min of the indices holding the minimum key.
    // The worst point: max over the non-NaN values, NaN if any value is NaN (max_prop).
    double kmin[3], wmx[3];
    int imin[3];
    unsigned nanw = 0u;
    for (int i = 0; i < 3; ++i) {
      const double key = bv[i] != bv[i] ? -1.0 : bv[i];
      kmin[i] = wave_reduce(key, [](double x, double y) { return __builtin_fmin(x, y); });
      int ix = key == kmin[i] ? bi[i] : INT_MAX;
      ix = min(ix, dpp_i32<0xB1>(ix));
      ix = min(ix, dpp_i32<0x4E>(ix));
      ix = min(ix, dpp_i32<0x141>(ix));
      ix = min(ix, dpp_i32<0x140>(ix));
      int i0, i1;
      swap_i32<16>(ix, i0, i1);
      ix = min(i0, i1);
      swap_i32<32>(ix, i0, i1);
      imin[i] = min(i0, i1);
      const bool wn = wf[i] != wf[i];
      nanw |= __ballot(wn) ? (1u << i) : 0u;
      wmx[i] = wave_reduce(wn ? -__builtin_inf() : wf[i],
                           [](double x, double y) { return __builtin_fmax(x, y); });
    }
    if (lane == 0)
      for (int i = 0; i < 3; ++i) {
        L.red[wave * 16 + i] = kmin[i];
        L.red[wave * 16 + 3 + i] = (double)imin[i];
        L.red[wave * 16 + 6 + i] = (nanw >> i) & 1u ? __builtin_nan("") : wmx[i];
      }
    __syncthreads();
    PHASE(22)
    // every wave: the same combination of the waves' partials (lane w holds wave w's; a
    // lexicographic (value, index) argmin and a NaN-propagating max, both independent of the
    // combination order, so every wave gets the same bits) and then, on lane 0, the
    // extremes and the nadir, written to the wave's own copy (wsc), which only that wave
    // reads (LDS is in order within a wave).
    double cw[3];
    int cix[3];
    {
      constexpr int NWV = T / 64;
      static_assert(NWV <= 16, "survival combine: at most 16 waves");
      const bool has = lane < NWV;
      for (int i = 0; i < 3; ++i) {
        double v = has ? L.red[lane * 16 + i] : __builtin_inf();
        int ix = has ? (int)L.red[lane * 16 + 3 + i] : INT_MAX;
        double w = has ? L.red[lane * 16 + 6 + i] : -__builtin_inf();
        // within the 16-lane row by DPP (quad xor 1, xor 2, half mirror, mirror: every lane
        // ends with the row's result, as in wave_reduce); ds_bpermute shuffles here cost
        // ~6 k cycles per state (MV_SURV_PHASES 22 -> 25)
#define MV_COMBINE_STEP(CTRL)                                                           \
  {                                                                                     \
    const double ov = dpp_f64<CTRL>(v);                                                 \
    const int oi = dpp_i32<CTRL>(ix);                                                   \
    const double ow = dpp_f64<CTRL>(w);                                                 \
    if (ov < v || (ov == v && oi < ix)) {                                               \
      v = ov;                                                                           \
      ix = oi;                                                                          \
    }                                                                                   \
    w = max_prop(w, ow);                                                                \
  }
        MV_COMBINE_STEP(0xB1)
        MV_COMBINE_STEP(0x4E)
        MV_COMBINE_STEP(0x141)
        MV_COMBINE_STEP(0x140)
#undef MV_COMBINE_STEP
        cix[i] = ix;
        cw[i] = w;
      }
    }
    if (lane == 0) {
      for (int i = 0; i < 3; ++i) {
        const int ix = cix[i];
        const double w = cw[i];
        wfront[i] = w;
        double row[3];
        if (ix < ne) {
          for (int k = 0; k < 3; ++k) row[k] = pext[ix * 3 + k];
        } else if (ix < ne + n0) {
          const int m = L.I[ix - ne];
          for (int k = 0; k < 3; ++k) row[k] = L.F[m * 3 + k];
        } else {
          for (int k = 0; k < 3; ++k) row[k] = L.ref[(ix - ne - n0) * 3 + k];
        }
        for (int k = 0; k < 3; ++k) ext[i * 3 + k] = row[k];
      }
    }
    wave_sync();
    PHASE(25)
    if (lane == 0) {
      // nadir (get_nadir_point with the call-site argument swap)
      double M[3][3], plane[3] = {1.0, 1.0, 1.0};
      for (int i = 0; i < 3; ++i)
        for (int k = 0; k < 3; ++k) M[i][k] = ext[i * 3 + k] - ideal[k];
      double Mc[3][3];
      for (int i = 0; i < 3; ++i)
        for (int k = 0; k < 3; ++k) Mc[i][k] = M[i][k];
      bool ok = lu_solve3(Mc, plane);
      double nd[3];
      if (ok) {
        double icp[3];
        for (int k = 0; k < 3; ++k) {
          icp[k] = 1.0 / plane[k];
          nd[k] = ideal[k] + icp[k];
        }
        bool close = true, small = false;
        for (int i = 0; i < 3; ++i) {
          const double mp = (M[i][0] * plane[0] + M[i][1] * plane[1]) + M[i][2] * plane[2];
          close = close && (fabs(mp - 1.0) <= 1e-8 + 1e-5 * 1.0);
          small = small || (icp[i] <= 1e-6);
        }
        if (!close || small) {
          ok = false;
        } else {
          for (int k = 0; k < 3; ++k)
            if (nd[k] > worst[k]) nd[k] = worst[k];
        }
      }
      if (!ok)
        for (int k = 0; k < 3; ++k) nd[k] = wpop[k];
      for (int k = 0; k < 3; ++k) {
        if (nd[k] - ideal[k] <= 1e-6) nd[k] = wfront[k];
        nadir[k] = nd[k];
      }
    }
    wave_sync();
    PHASE(26)
  }
  PHASE(4)

  // ---- aspiration reference directions (normalised), R points + 3 extreme axes
  {
    const double nv = 1.0 / sqrt(3.0);
    const double asp = a.mu * (1.0 / 3.0);
    for (int r = tid; r < RN; r += T) {
      double res[3];
      if (r < R) {
        double l[3];
        for (int k = 0; k < 3; ++k) l[k] = (L.ref[r * 3 + k] - ideal[k]) / (nadir[k] - ideal[k]);
        const double dot = (l[0] * nv + l[1] * nv) + l[2] * nv;
        double inter[3];
        if (fabs(dot) > 1e-6) {
          const double d = ((1.0 * nv + 0.0 * nv) + 0.0 * nv) / dot;
          for (int k = 0; k < 3; ++k) inter[k] = 0.0 + l[k] * d;
        } else {
          const double q0 = l[0] - 1.0, q1 = l[1] - 0.0, q2 = l[2] - 0.0;
          const double t = (q0 * nv + q1 * nv) + q2 * nv;
          for (int k = 0; k < 3; ++k) inter[k] = l[k] - t * nv;
        }
        for (int k = 0; k < 3; ++k) res[k] = asp + (inter[k] - asp);
        if (!(res[0] > 0.0 && res[1] > 0.0 && res[2] > 0.0)) {
          for (int k = 0; k < 3; ++k)
            if (res[k] < 0.0) res[k] = 0.0;
          const double s = (res[0] + res[1]) + res[2];
          for (int k = 0; k < 3; ++k) res[k] = res[k] / s;
        }
      } else {
        for (int k = 0; k < 3; ++k) res[k] = (k == r - R) ? 1.0 : 0.0;
      }
      const double nrm = sqrt((res[0] * res[0] + res[1] * res[1]) + res[2] * res[2]);
      for (int k = 0; k < 3; ++k) L.U[r * 3 + k] = res[k] / nrm;
      L.Uf[r] = make_double4(L.U[r * 3], L.U[r * 3 + 1], L.U[r * 3 + 2], 0.0);
    }
    if (tid == 0) L.iscal[15] = 0;
    __syncthreads();
  }
  PHASE(5)

  // ---- association of the ranked individuals (I order) to the nearest direction
  {
    double den[3];
    for (int k = 0; k < 3; ++k) {
      den[k] = nadir[k] - ideal[k];
      if (den[k] == 0.0) den[k] = 1e-12;
    }
    // Two adjacent lanes per individual, each sweeping half of the directions (N = P + O
    // individuals on 8 waves would otherwise leave 3 waves idle and double up one SIMD);
    // the halves combine with lane swaps: fp32 minimum (exact), then the fp64 candidate
    // minimum in np.argmin's order (arg_better is a total order, so the combination equals
    // the sequential scan).
    const int nh = RN >> 1;  // directions per half (wave-uniform loop counts); an odd RN's
                             // last direction goes to the second half's chain 0
    for (int v = tid; v < 2 * n_ranked; v += T) {
      const int p = v >> 1, hf = v & 1;
      const int jb = hf ? nh : 0;
      const bool odd = hf && (RN & 1);
      const int m = L.I[p];
      double Nn[3];
      for (int k = 0; k < 3; ++k) Nn[k] = (L.F[m * 3 + k] - ideal[k]) / den[k];
      if (Nn[0] == 0.0 && Nn[1] == 0.0 && Nn[2] == 0.0 && !signbit(Nn[0]) && !signbit(Nn[1]) &&
          !signbit(Nn[2])) {  // at the ideal point: every distance is exactly +0 (both lanes)
        if (!hf) {
          L.niche[p] = 0;
          L.dist[p] = 0.0;
        }
        continue;
      }
      // fp64 pre-filter of the squared perpendicular distances, |N|^2 - (N.u)^2 with FMAs on
      // the same unit directions as the exact pass.  Its error against the exact pass's
      // sqrt'ed value squared is below 20 u |N|^2 (u = 2^-53: the dot product 3 u |N|, its
      // square 6 u |N|^2, |N|^2 3 u |N|^2; the exact pass's own e = s u - N error 10 u |N| |e|),
      // so the exact minimum -- and every direction whose sqrt'ed distance ties it -- lies
      // within tol = 1e-14 (|N|^2 + best) > 40 u |N|^2 + 4.5e-16 best of the pre-filter's
      // minimum.  Unlike the fp32 filter's 3e-5 |N|^2 this separates crowded directions
      // (late botnet generations), so no refinement sweeps are needed; more than four hits
      // (near-duplicate directions) or a NaN / overflow go to the exact pass below.
      const double nn = fma(Nn[0], Nn[0], fma(Nn[1], Nn[1], Nn[2] * Nn[2]));
      const double4* Ud = L.Uf;
      auto d2f = [&](int j) {
        const double4 u = Ud[j];
        const double sp = fma(Nn[0], u.x, fma(Nn[1], u.y, Nn[2] * u.z));
        return fma(-sp, sp, nn);
      };
      double b0 = __builtin_inf(), b1 = b0, b2 = b0, b3 = b0;
      const int n4 = nh >> 2;
      if (nn < __builtin_inf()) {
#pragma unroll MV_ASSOC_UNROLL
        for (int k = 0; k < n4; ++k) {
          const int j = jb + 4 * k;
          b0 = __builtin_fmin(b0, d2f(j));
          b1 = __builtin_fmin(b1, d2f(j + 1));
          b2 = __builtin_fmin(b2, d2f(j + 2));
          b3 = __builtin_fmin(b3, d2f(j + 3));
        }
        for (int j = jb + 4 * n4; j < jb + nh; ++j) b0 = __builtin_fmin(b0, d2f(j));
        if (odd) b0 = __builtin_fmin(b0, d2f(RN - 1));
      }
      double best = __builtin_fmin(__builtin_fmin(b0, b1), __builtin_fmin(b2, b3));
      best = __builtin_fmin(best, dpp_f64<0xB1>(best));  // the pair's other lane (DPP xor 1)
      const double lim = best + 1e-14 * (nn + best);
      if (lim < __builtin_inf()) {  // false on NaN / inf (the same in both lanes)
        double bd = __builtin_inf();
        int bj = 0;
        auto cand = [&](int j) {  // exact fp64 distance, np.argmin order
          const double* u = &L.U[j * 3];
          const double s = (Nn[0] * u[0] + Nn[1] * u[1]) + Nn[2] * u[2];
          const double e0 = s * u[0] - Nn[0], e1 = s * u[1] - Nn[1], e2 = s * u[2] - Nn[2];
          const double dd = sqrt((e0 * e0 + e1 * e1) + e2 * e2);
          if (arg_better(dd, j, bd, bj)) {
            bd = dd;
            bj = j;
          }
        };
        const unsigned cm0 = (b0 <= lim ? 1u : 0u) | (b1 <= lim ? 2u : 0u) |
                             (b2 <= lim ? 4u : 0u) | (b3 <= lim ? 8u : 0u);
        int c0 = 0, c1 = 0, c2 = 0, c3 = 0, nc = 0;
        auto hit = [&](int jc) {
          c0 = nc == 0 ? jc : c0;
          c1 = nc == 1 ? jc : c1;
          c2 = nc == 2 ? jc : c2;
          c3 = nc == 3 ? jc : c3;
          ++nc;
        };
        unsigned cm = cm0;
        while (cm) {  // every direction of this half within lim, in chain order
          const int u = __builtin_ctz(cm);
          cm &= cm - 1u;
          int k = 0;
          for (; k + 4 <= n4; k += 4) {
            const int jc = jb + 4 * k + u;
            const double d0 = d2f(jc), d1 = d2f(jc + 4), d2 = d2f(jc + 8), d3 = d2f(jc + 12);
            if (d0 <= lim) hit(jc);
            if (d1 <= lim) hit(jc + 4);
            if (d2 <= lim) hit(jc + 8);
            if (d3 <= lim) hit(jc + 12);
          }
          for (; k < n4; ++k) {
            const int jc = jb + 4 * k + u;
            if (d2f(jc) <= lim) hit(jc);
          }
          if (u == 0) {
            for (int jc = jb + 4 * n4; jc < jb + nh; ++jc)
              if (d2f(jc) <= lim) hit(jc);
            if (odd && d2f(RN - 1) <= lim) hit(RN - 1);
          }
        }
        const bool ovf = nc > 4 || dpp_i32<0xB1>(nc) > 4;
        if (!ovf) {
          if (nc > 0) cand(c0);
          if (nc > 1) cand(c1);
          if (nc > 2) cand(c2);
          if (nc > 3) cand(c3);
        }
        const double od = dpp_f64<0xB1>(bd);
        const int oj = dpp_i32<0xB1>(bj);
        if (arg_better(od, oj, bd, bj)) {
          bd = od;
          bj = oj;
        }
        if (!hf) {
          if (ovf) {
            L.key[atomicAdd(&L.iscal[15], 1)] = p;
          } else {
            L.niche[p] = bj;
            L.dist[p] = bd;
          }
        }
      } else if (!hf) {
        L.key[atomicAdd(&L.iscal[15], 1)] = p;
      }
    }
    __syncthreads();
    PHASE(10)
    // exact np.argmin over sqrt'ed distances for the flagged individuals: one individual per
    // wave, the directions spread over the lanes (j = lane + 64 k), then the wave's argmin in
    // np.argmin's order (arg_better is a total order, so the split does not change the
    // result).  A thread-serial scan here cost 90 k cycles per state at botnet generation
    // 1000, where the aspiration directions crowd together and 72 of 303 individuals per
    // state have more pre-filter candidates than the fast pass keeps.
    const int n_flag = L.iscal[15];
    if (MV_CLOCKS && a.phase && tid == 0) a.phase[(size_t)b * 32 + 12] = n_flag;
    for (int t = wave; t < n_flag; t += T / 64) {
      const int p = L.key[t];
      const int m = L.I[p];
      double Nn[3];
      for (int k = 0; k < 3; ++k) Nn[k] = (L.F[m * 3 + k] - ideal[k]) / den[k];
      double bd = __builtin_inf();
      int bj = INT_MAX;
      for (int j = lane; j < RN; j += 64) {
        const double* u = &L.U[j * 3];
        const double s = (Nn[0] * u[0] + Nn[1] * u[1]) + Nn[2] * u[2];
        const double e0 = s * u[0] - Nn[0], e1 = s * u[1] - Nn[1], e2 = s * u[2] - Nn[2];
        const double dd = sqrt((e0 * e0 + e1 * e1) + e2 * e2);
        if (arg_better(dd, j, bd, bj)) {
          bd = dd;
          bj = j;
        }
      }
      wave_argbest(bd, bj, [](double v, int i1, double w, int i2) {
        return arg_better(v, i1, w, i2);
      });
      if (lane == 0) {
        L.niche[p] = bj;
        L.dist[p] = bd;
      }
    }
    __syncthreads();
  }
  PHASE(6)

  // ---- survivor selection: fronts until the last + niching on the last front
  int n_out;
  if (n_ranked > a.n_survive) {
    // Niching in closed form.  With member keys fixed per generation, niche n's picks
    // follow one order (min-dist member first when its until-front count c_n is 0, then
    // ascending (key, position)); its j-th pick happens at "level" c_n + j, the loop's
    // rounds visit the non-empty levels in ascending order, and within a round the
    // niches go in ascending (round key, niche).  So every pick's output position is a
    // prefix count over levels plus a rank inside its level: no sequential loop.
    const int fs = L.fstart[nf - 1];
    const int Lc = n_ranked - fs;
    const int n_rem = nf == 1 ? a.n_survive : a.n_survive - fs;
    const int until = nf == 1 ? 0 : fs;
    const Rng rng(a.seed, state_stream(a.stream_key, a.state_keys, a.key0, b));
    int* grank = L.memb;
    int* lev = L.csr;
    int* cnt = L.count;
    int* mcnt = L.remain;
    int* start = L.csr_off;
    int* bestkr = L.cand;
    const int* nich = L.niche + fs;
    const double* dst = L.dist + fs;
    const int nlev = N + Lc + 1;
    int* fill = L.ckey;  // [RN] fill counters of the niche member lists
    int* mem = L.key;    // [Lc] last-front members grouped by niche (order inside a niche
                         // is arbitrary: only counts are taken over it)
    for (int n = tid; n < RN; n += T) {
      cnt[n] = 0;
      mcnt[n] = 0;
      L.dmin[n] = ~0ull;
      bestkr[n] = INT_MAX;
      fill[n] = 0;
    }
    if (tid == 0) L.iscal[14] = 0;  // largest niche (the dominance counter is done)
    for (int l = tid; l < nlev; l += T) L.lround[l] = 0;
    // The counters above must be zero before ANY thread counts into them.  (Round 3 had no
    // barrier here: a thread of one wave could add its member to mcnt[n] / cnt[n] before the
    // thread of another wave that zeroes entry n ran, and the zeroing store erased the count.
    // With few crowded niches -- clone-heavy botnet generations: 2-7 niches for ~270
    // last-front members -- the member lists then overlapped and niching returned duplicate
    // survivors; found by the checks build, check 26, tests/golden/survival_botnet_clones.npz.)
    __syncthreads();
    unsigned long long* sk = L.sortk;
    for (int p = tid; p < until; p += T) atomicAdd(&cnt[L.niche[p]], 1);
    // member order inside each niche: ascending (niche, member key, position); grank = rank
    for (int p = tid; p < Lc; p += T) {
      const unsigned key = rng.draw((uint32_t)p, (uint32_t)gen, TAG_NICHE_MEMBER).x;
      const int m_n = atomicAdd(&mcnt[nich[p]], 1) + 1;
      if (NWMAX * 64 > SURV_NLDS && m_n > NICHE_SORT_MIN) atomicMax(&L.iscal[14], m_n);
      // (niche, member key, position); positions take 10 bits (N <= 1024)
      sk[p] = ((unsigned long long)nich[p] << 42) | ((unsigned long long)key << 10) | (unsigned)p;
    }
    __syncthreads();
    PHASE(16)
    for (int p = tid; p < Lc; p += T) {
      const int np_ = nich[p];
      if (cnt[np_] == 0)
        atomicMin(&L.dmin[np_], (unsigned long long)__double_as_longlong(dst[p]));
    }
    for (int n = tid; n < RN; n += T) start[n] = mcnt[n];
    __syncthreads();
    block_scan_excl<T>(start, RN, wsum);
    const bool by_sort = NWMAX * 64 > SURV_NLDS && L.iscal[14] > NICHE_SORT_MIN;  // uniform
    if (!by_sort) {
      for (int p = tid; p < Lc; p += T) {
        const int np_ = nich[p];
        mem[start[np_] + atomicAdd(&fill[np_], 1)] = p;
      }
    }
    __syncthreads();
    PHASE(17)
    // grank = rank of sk[p] among all keys = members of smaller niches (start) + rank inside
    // its own niche.  The keys are distinct and niche-major, so that is sk[p]'s position in
    // the sorted keys (by_sort), or counted over its niche's members only
    if (by_sort) {
      const int P2 = pow2_at_least(Lc);
      for (int q = Lc + tid; q < P2; q += T) sk[q] = ~0ull;  // padding sorts last
      __syncthreads();
      bitonic_sort_u64<T>(sk, P2);
      for (int r = tid; r < Lc; r += T) {
        const int p = (int)(sk[r] & 1023ull);
        const int np_ = nich[p];
        grank[p] = r;
        if (cnt[np_] == 0 && (unsigned long long)__double_as_longlong(dst[p]) == L.dmin[np_])
          atomicMin(&bestkr[np_], r - start[np_]);
      }
    } else
    for (int p = tid; p < Lc; p += T) {
      const int np_ = nich[p];
      const unsigned long long kp = sk[p];
      int r = 0, t = start[np_];
      const int te = t + mcnt[np_];
      for (; t + 4 <= te; t += 4) {  // crowded niches: four gathers in flight
        const int m0 = mem[t], m1 = mem[t + 1], m2 = mem[t + 2], m3 = mem[t + 3];
        r += (sk[m0] < kp ? 1 : 0) + (sk[m1] < kp ? 1 : 0) + (sk[m2] < kp ? 1 : 0) +
             (sk[m3] < kp ? 1 : 0);
      }
      for (; t < te; ++t) r += sk[mem[t]] < kp ? 1 : 0;
      grank[p] = start[np_] + r;
      if (cnt[np_] == 0 && (unsigned long long)__double_as_longlong(dst[p]) == L.dmin[np_])
        atomicMin(&bestkr[np_], r);
    }
    __syncthreads();
    PHASE(18)
    // level of each pick; per level its member count (high half-word) and non-empty flag
    // (bit 0), so ONE exclusive scan gives every level's first bucket position and its round
    // index (the number of non-empty levels before it)
    for (int p = tid; p < Lc; p += T) {
      const int np_ = nich[p];
      const int kr = grank[p] - start[np_];
      int j = kr;
      if (cnt[np_] == 0) j = kr == bestkr[np_] ? 0 : kr + (kr < bestkr[np_] ? 1 : 0);
      const int l = cnt[np_] + j;
      lev[p] = l;
      grank[p] = atomicAdd(&L.lround[l], 1 << 16) >> 16;  // position inside the level
      atomicOr(&L.lround[l], 1);
    }
    __syncthreads();
    PHASE(19)
    block_scan_excl<T>(L.lround, nlev, wsum);
    // output order: ascending (level, round key of the niche, niche); a niche picks at most
    // once per level, so a pick's rank is the members of lower levels plus its rank by
    // (round key, niche) inside its own level -- counted over that level's bucket only, and
    // only for levels that start below n_rem
    int* bucket = L.key;  // [Lc] last-front members grouped by level
    for (int p = tid; p < Lc; p += T) {
      const int l = lev[p];
      const int lr = L.lround[l];
      const unsigned kr = rng.draw((uint32_t)((lr & 0xFFFF) * RN + nich[p]), (uint32_t)gen,
                                   TAG_NICHE_PERM).x;
      sk[p] = ((unsigned long long)kr << 11) | (unsigned long long)nich[p];
      bucket[(lr >> 16) + grank[p]] = p;
    }
    __syncthreads();
    PHASE(20)
    for (int p = tid; p < Lc; p += T) {
      const int l = lev[p];
      const int b0 = L.lround[l] >> 16;
      if (b0 >= n_rem) continue;
      const int b1 = l + 1 < nlev ? (L.lround[l + 1] >> 16) : Lc;
      const unsigned long long kp = sk[p];
      int r = b0;
      int t = b0;
      for (; t + 4 <= b1; t += 4) {
        const int m0 = bucket[t], m1 = bucket[t + 1], m2 = bucket[t + 2], m3 = bucket[t + 3];
        r += (sk[m0] < kp ? 1 : 0) + (sk[m1] < kp ? 1 : 0) + (sk[m2] < kp ? 1 : 0) +
             (sk[m3] < kp ? 1 : 0);
      }
      for (; t < b1; ++t) r += sk[bucket[t]] < kp ? 1 : 0;
      if (r < n_rem) L.surv[until + r] = fs + p;
    }
    for (int p = tid; p < until; p += T) L.surv[p] = p;
    n_out = a.n_survive;
  } else {
    for (int p = tid; p < n_ranked; p += T) L.surv[p] = p;
    n_out = n_ranked;
  }
  __syncthreads();
  PHASE(7)
  // the variation plan's tables, into the (now dead) F rows: their loads overlap the outputs
  uint32_t* pgeo = (uint32_t*)(smem + o.ptab);
  int* pcmap = (int*)(pgeo + a.Vr + 1);
  int* pginfo = pcmap + a.Vr;
  if (plan) {
    const int nw = plan_tab_words(a.Vr, a.V);
    for (int k = tid; k < nw; k += T) {
      const int v = k <= a.Vr ? (int)a.geo[k]
                              : (k < 2 * a.Vr + 1 ? a.cmap[k - a.Vr - 1] : a.ginfo[k - 2 * a.Vr - 1]);
      pgeo[k] = (uint32_t)v;
    }
  }

  // ---- outputs
  for (int k = tid; k < N; k += T) L.memb[k] = 0;  // selected flags by merged index
  __syncthreads();
  for (int k = tid; k < n_out; k += T) {
    const int m = L.I[L.surv[k]];
    L.memb[m] = 1;
    L.sel[k] = L.slot[m];  // new population order -> slot (read by the tournament below)
    if (slot_mode)
      a.pop_slot_out[(size_t)b * a.n_survive + k] = L.slot[m];
    else
      a.survivors[(size_t)b * a.n_survive + k] = m;
  }
  if (!slot_mode)
    for (int k = n_out + tid; k < a.n_survive; k += T)
      a.survivors[(size_t)b * a.n_survive + k] = -1;
  if (a.rank)
    for (int m = tid; m < N; m += T) a.rank[(size_t)b * N + m] = L.front_of[m];
  if (a.order)
    for (int p = tid; p < N; p += T) a.order[(size_t)b * N + p] = p < n_ranked ? L.I[p] : -1;
  if (a.niche)
    for (int p = tid; p < N; p += T) a.niche[(size_t)b * N + p] = p < n_ranked ? L.niche[p] : -1;
  if (a.dist)
    for (int p = tid; p < N; p += T)
      a.dist[(size_t)b * N + p] = p < n_ranked ? L.dist[p] : 0.0;
  if (tid == 0) {
    if (a.n_ranked) a.n_ranked[b] = n_ranked;
    for (int k = 0; k < 3; ++k) {
      a.ideal[(size_t)b * 3 + k] = ideal[k];
      a.worst[(size_t)b * 3 + k] = worst[k];
      if (a.nadir) a.nadir[(size_t)b * 3 + k] = nadir[k];
    }
    for (int k = 0; k < 9; ++k) a.extreme[(size_t)b * 9 + k] = ext[k];
    a.has_extreme[b] = 1;
  }
  __syncthreads();
  if (slot_mode && N > a.n_survive) {
    const int nfree = block_compact<T>(N, [&](int m) { return L.memb[m] == 0; }, L.key, 0, wsum);
#ifdef MV_CHECKS
    if (nfree != N - n_out) {  // duplicate survivors: record, dump this state's inputs
      if (tid == 0) chk_fail(CK_SURV_DUP, (long long)gen * 4096 + b, nfree);
      __shared__ int s_own;
      if (tid == 0) s_own = atomicCAS(&g_surv_dump_owner, 0, 1) == 0;
      __syncthreads();
      if (s_own) {
        double* d = g_surv_dump;
        for (int m = tid; m < N; m += T)
          for (int k = 0; k < 3; ++k)
            d[SURV_DUMP_HEAD + m * 3 + k] = a.F[((size_t)b * a.S + L.slot[m]) * 3 + k];
        if (tid < 3) {
          d[4 + tid] = pre_ideal;
          d[7 + tid] = pre_worst;
        }
        if (tid < 9) d[10 + tid] = pext[tid];
        if (tid == 0) {
          d[1] = gen;
          d[2] = b;
          d[3] = N;
          d[19] = has_ext;
          d[20] = a.n_survive;
          d[21] = __longlong_as_double((long long)a.seed);
          d[0] = 1.0;
        }
      }
    }
#endif
    for (int k = tid; k < nfree; k += T)
      a.free_slot[(size_t)b * a.O + MV_IDX(k, a.O, CK_SURV_SLOT)] = L.slot[L.key[k]];
  }
  __syncthreads();
  PHASE(8)
  if (parents_out) {
    tournament<T>(a.n_survive, a.O_next, a.seed,
                  state_stream(a.stream_key, a.state_keys, a.key0, b), sel_gen, slot_mode ? L.sel : nullptr,
               parents_out + (size_t)b * n_m_next * 2, L.sortk, L.perm,
               plan ? (int*)L.sortk : nullptr);
  }
  __syncthreads();
  if (plan) {  // (clocks: slots 23 / 24 bracket the plan of the last generation that has one)
    PHASE(23)
    variation_plan<T>(a, b, sel_gen, (const int*)L.sortk, (int*)L.sortk + 2 * n_m_next, pgeo,
                      pcmap, pginfo);
    __syncthreads();
    PHASE(24)
  }
  PHASE(9)
#undef PHASE
}

}  // namespace mv
