// Device-side index checks (debug builds only: -DMV_CHECKS, `make checks`).
//
// MV_IDX(i, n, code) is `i` in the product build.  In a checks build it tests 0 <= i < n;
// a failing index is recorded (the first failure of the launch sequence wins: check code,
// workgroup, thread, value, bound; plus a failure count) and replaced by 0, so the access
// that would have faulted reads or writes a valid element instead and the host can report
// WHICH index was wrong (mv_debug_checks).  Every global row / slot / gene offset the row,
// classifier and survival kernels compute from data (parents, out_map, pop/free slots) or
// from a runtime index into a private array goes through it.
//
// The record is a per-translation-unit __device__ array (no relocatable device code), read
// by take_checks_<tu>() on the host.  Stores and atomics are ordinary vector-memory ops.
#pragma once
#include <hip/hip_runtime.h>

namespace mv {

// check codes (mv_debug_checks reports them; DESIGN.md §8 lists them)
enum : int {
  CK_GEN_STATE = 1,     // k_gen/k_genc: row chunk's state >= B
  CK_GEN_PARENT = 2,    // mating's parent slot outside [0, in_rows)
  CK_GEN_DST = 3,       // out_map destination outside [0, out_rows)
  CK_GEN_MUTPOS = 4,    // cached mutation position outside [0, V)
  CK_GEN_MUTROW = 5,    // mutated row's parent slot outside [0, in_rows)
  CK_GEN_APPLY = 6,     // applied mutation position outside [0, V)
  CK_GEN_ROW = 7,       // row index outside [0, n) or history row outside [0, hist_rows)
  CK_GEN_LANE = 8,      // readlane row k outside [0, min(nrw, 64))
  CK_CONS_DST = 9,      // k_cons / phase 2: source or destination row outside its range
  CK_CONS_OPND = 10,    // constraint operand feature outside [0, D)
  CK_CONS_COL = 11,     // constraint column outside [0, C)
  CK_MLP_ROW = 12,      // k_mlp2: gene row (state / out_map) outside its range
  CK_MLP_OUT = 13,      // k_mlp2: F / history row outside its range
  CK_SURV_SLOT = 14,    // k_survive: pool slot outside [0, S)
  CK_SURV_PARENT = 15,  // k_survive: tournament parent slot outside [0, S)
  CK_GEN_SBX = 16,      // SBX crossed gene outside [0, V)
  // final element offsets at the access (after any register spill / reload), k_genc
  CK_AT_PARENT = 17,    // parent gene load (load_parent_row) outside the state's pool
  CK_AT_MUTLOAD = 18,   // row_draws' crossed-parent gene load outside the state's pool
  CK_AT_CHILD = 19,     // child gene store outside the state's pool
  CK_AT_F2 = 20,        // f2 store outside the state's F rows
  CK_AT_HIST1 = 21,     // phase-1 history store outside the state's history
  CK_AT_SRC2 = 22,      // phase-2 gene load outside the state's pool
  CK_AT_F3 = 23,        // f3 store outside the state's F rows
  CK_AT_HIST2 = 24,     // phase-2 history / G-column store outside the state's history
  CK_AT_BOUNDS = 25,    // gl / gu load outside the state's bounds
  CK_SURV_DUP = 26,     // k_survive: the survivors are not n_out distinct individuals
                        // (value = gen * 4096 + state in its group, bound = free count);
                        // the first such state's inputs go to the survival dump
};
// survival dump (checks builds): [0] 1 = valid, [1] gen, [2] state in its group, [3] N,
// [4, 7) carried ideal, [7, 10) carried worst, [10, 19) carried extremes, [19] has_extreme,
// [20] n_survive, [21] seed (as double bits), [24, 24 + 3 N) merged F in merge order
constexpr int SURV_DUMP_HEAD = 24;
constexpr int SURV_DUMP_N = SURV_DUMP_HEAD + 3 * 1024;

#ifdef MV_CHECKS
static __device__ int g_chk[8];  // code, block, thread, value, bound, failures, -, -

__device__ __noinline__ static void chk_fail(int code, long long v, long long n) {
  atomicAdd(&g_chk[5], 1);
  if (atomicCAS(&g_chk[0], 0, code) == 0) {
    volatile int* r = g_chk;
    r[1] = (int)blockIdx.x;
    r[2] = (int)threadIdx.x;
    r[3] = (int)v;
    r[4] = (int)n;
  }
}
__device__ __forceinline__ long long chk_idx(long long i, long long n, int code) {
  if (i < 0 || i >= n) {
    chk_fail(code, i, n);
    return 0;
  }
  return i;
}
#define MV_IDX(i, n, code) ((decltype(i))::mv::chk_idx((long long)(i), (long long)(n), (code)))
// pointer p inside [lo, hi) (element units), else lo
template <class T>
__device__ __forceinline__ T* chk_ptr(T* p, const T* lo, const T* hi, int code) {
  if (p < lo || p >= hi) {
    chk_fail(code, (long long)(p - lo), (long long)(hi - lo));
    return const_cast<T*>(lo);
  }
  return p;
}
#define MV_PTR(p, lo, hi, code) ::mv::chk_ptr((p), (lo), (hi), (code))
#define MV_CHECKS_ON 1
// Reads and clears this translation unit's record (out[8]).
#define MV_DEFINE_TAKE_CHECKS(name)                                               \
  hipError_t name(int* out) {                                                     \
    hipError_t e = hipMemcpyFromSymbol(out, HIP_SYMBOL(g_chk), 8 * sizeof(int));  \
    if (e != hipSuccess) return e;                                                \
    const int z[8] = {0, 0, 0, 0, 0, 0, 0, 0};                                    \
    return hipMemcpyToSymbol(HIP_SYMBOL(g_chk), z, 8 * sizeof(int));              \
  }
#else
#define MV_IDX(i, n, code) (static_cast<void>(n), (i))
#define MV_PTR(p, lo, hi, code) (static_cast<void>(lo), static_cast<void>(hi), (p))
#define MV_CHECKS_ON 0
#define MV_DEFINE_TAKE_CHECKS(name)                  \
  hipError_t name(int* out) {                        \
    for (int k = 0; k < 8; ++k) out[k] = 0;          \
    return hipSuccess;                               \
  }
#endif

hipError_t take_checks_eval(int* out);
hipError_t take_checks_survive(int* out);
hipError_t take_survival_dump(double* out);  // [SURV_DUMP_N], cleared

}  // namespace mv
