// Wave-level building blocks shared by the kernels (gfx950, wave64).
#pragma once
#include <hip/hip_runtime.h>

namespace mv {

// Wave-wide reductions without LDS: DPP within rows of 16 lanes (quad_perm xor 1, xor 2,
// row_half_mirror, row_mirror), then gfx950 permlane16/32 swaps across rows.  Every step
// combines a lane's value with exactly one partner's (commutative), so all 64 lanes end
// with the same, deterministic total.
template <int CTRL>
__device__ __forceinline__ double dpp_f64(double v) {
  const int lo = __double2loint(v), hi = __double2hiint(v);
  return __hiloint2double(__builtin_amdgcn_update_dpp(0, hi, CTRL, 0xF, 0xF, false),
                          __builtin_amdgcn_update_dpp(0, lo, CTRL, 0xF, 0xF, false));
}

// (value of this lane's row-pair partner half, own half) across 16-lane rows (SWAP=16) or
// 32-lane halves (SWAP=32): returns {x_first, x_second} with x_first + x_second the pair.
template <int SWAP>
__device__ __forceinline__ void swap_f64(double v, double& d0, double& d1) {
  const int lo = __double2loint(v), hi = __double2hiint(v);
  if (SWAP == 16) {
    const auto a = __builtin_amdgcn_permlane16_swap(lo, lo, false, false);
    const auto b = __builtin_amdgcn_permlane16_swap(hi, hi, false, false);
    d0 = __hiloint2double(b[0], a[0]);
    d1 = __hiloint2double(b[1], a[1]);
  } else {
    const auto a = __builtin_amdgcn_permlane32_swap(lo, lo, false, false);
    const auto b = __builtin_amdgcn_permlane32_swap(hi, hi, false, false);
    d0 = __hiloint2double(b[0], a[0]);
    d1 = __hiloint2double(b[1], a[1]);
  }
}

__device__ __forceinline__ double wave_sum(double v) {
  v = v + dpp_f64<0xB1>(v);
  v = v + dpp_f64<0x4E>(v);
  v = v + dpp_f64<0x141>(v);
  v = v + dpp_f64<0x140>(v);
  double d0, d1;
  swap_f64<16>(v, d0, d1);
  v = d0 + d1;
  swap_f64<32>(v, d0, d1);
  return d0 + d1;
}

__device__ __forceinline__ double nanmax(double a, double b) {
  if (a != a) return a;
  if (b != b) return b;
  return b > a ? b : a;
}

// Four wave sums in one butterfly (k_genc's row: f2, the lane ops' f3 part and two
// ABS_SUMDIFF columns).  Each total is the same pairwise tree as wave_sum's -- blocks of 1, 2,
// 4, 8, 16, 32 lanes -- so its bits are wave_sum's (a + b == b + a; only which lane holds a
// block sum differs): level 1 keeps values 0, 1 on even lanes and 2, 3 on odd ones, level 2
// one value per lane (lane bits (0, 1) -> value 0, 1, 2, 3 on lanes 0, 2, 1, 3), levels 3 and
// 4 shift the higher block down the row (row_shl 4, 8: lanes 0-3 collect), levels 5 and 6
// are wave_sum's row swaps.  About 35 VALU instead of four wave_sums' 72.
__device__ __forceinline__ double rdl_f64(double v, int k) {
  const int lo = __builtin_amdgcn_readlane(__double2loint(v), k);
  const int hi = __builtin_amdgcn_readlane(__double2hiint(v), k);
  return __hiloint2double(hi, lo);
}
__device__ __forceinline__ void wave_sum4(double v0, double v1, double v2, double v3, int lane,
                                          double (&t)[4]) {
  const bool odd = (lane & 1) != 0, b1 = (lane & 2) != 0;
  const double k0 = odd ? v2 : v0, k1 = odd ? v3 : v1;  // kept
  const double s0 = odd ? v0 : v2, s1 = odd ? v1 : v3;  // the partner's values
  const double a0 = k0 + dpp_f64<0xB1>(s0);
  const double a1 = k1 + dpp_f64<0xB1>(s1);
  const double kk = b1 ? a1 : a0, ss = b1 ? a0 : a1;
  double w = kk + dpp_f64<0x4E>(ss);
  w = w + dpp_f64<0x104>(w);  // row_shl:4 -- lane i + 4's block
  w = w + dpp_f64<0x108>(w);  // row_shl:8
  double d0, d1;
  swap_f64<16>(w, d0, d1);
  w = d0 + d1;
  swap_f64<32>(w, d0, d1);
  w = d0 + d1;
  t[0] = rdl_f64(w, 0);
  t[1] = rdl_f64(w, 2);
  t[2] = rdl_f64(w, 1);
  t[3] = rdl_f64(w, 3);
}

// nanmax as selects (no exec-mask branches): the same value for every input
__device__ __forceinline__ double nanmax_sel(double a, double b) {
  double r = b > a ? b : a;
  r = b != b ? b : r;
  return a != a ? a : r;
}

template <class Op>
__device__ __forceinline__ double wave_reduce(double v, Op op) {
  v = op(v, dpp_f64<0xB1>(v));
  v = op(v, dpp_f64<0x4E>(v));
  v = op(v, dpp_f64<0x141>(v));
  v = op(v, dpp_f64<0x140>(v));
  double d0, d1;
  swap_f64<16>(v, d0, d1);
  v = op(d0, d1);
  swap_f64<32>(v, d0, d1);
  return op(d0, d1);
}

template <int CTRL>
__device__ __forceinline__ int dpp_i32(int v) {
  return __builtin_amdgcn_update_dpp(0, v, CTRL, 0xF, 0xF, false);
}

template <int SWAP>
__device__ __forceinline__ void swap_i32(int v, int& d0, int& d1) {
  if (SWAP == 16) {
    const auto a = __builtin_amdgcn_permlane16_swap(v, v, false, false);
    d0 = a[0];
    d1 = a[1];
  } else {
    const auto a = __builtin_amdgcn_permlane32_swap(v, v, false, false);
    d0 = a[0];
    d1 = a[1];
  }
}

// (value, index) reduction: better(v, i, bv, bi) must be a strict total order, so every lane
// ends with the same winner.
template <class Better>
__device__ __forceinline__ void wave_argbest(double& v, int& i, Better better) {
#define MV_ARG_STEP(CTRL)                                   \
  {                                                         \
    const double ov = dpp_f64<CTRL>(v);                     \
    const int oi = dpp_i32<CTRL>(i);                        \
    if (better(ov, oi, v, i)) {                             \
      v = ov;                                               \
      i = oi;                                               \
    }                                                       \
  }
  MV_ARG_STEP(0xB1)
  MV_ARG_STEP(0x4E)
  MV_ARG_STEP(0x141)
  MV_ARG_STEP(0x140)
#undef MV_ARG_STEP
  double d0, d1;
  int i0, i1;
  swap_f64<16>(v, d0, d1);
  swap_i32<16>(i, i0, i1);
  if (better(d1, i1, d0, i0)) {
    d0 = d1;
    i0 = i1;
  }
  swap_f64<32>(d0, v, d1);
  swap_i32<32>(i0, i, i1);
  if (better(d1, i1, v, i)) {
    v = d1;
    i = i1;
  }
}

__device__ __forceinline__ double wave_max(double v) {
  v = nanmax_sel(v, dpp_f64<0xB1>(v));
  v = nanmax_sel(v, dpp_f64<0x4E>(v));
  v = nanmax_sel(v, dpp_f64<0x141>(v));
  v = nanmax_sel(v, dpp_f64<0x140>(v));
  double d0, d1;
  swap_f64<16>(v, d0, d1);
  v = nanmax_sel(d0, d1);
  swap_f64<32>(v, d0, d1);
  return nanmax_sel(d0, d1);
}

// LDS byte addresses held in registers: lds_addr of a pointer into the kernel's LDS, and a
// double loaded straight from such an address (one ds_read_b64 on the register -- a
// generic base + offset made the compiler add the dynamic-LDS base, 0, to every address)
typedef const __attribute__((address_space(3))) double lds_double;
__device__ __forceinline__ unsigned lds_addr(const void* p) {
  return (unsigned)(uintptr_t)(const __attribute__((address_space(3))) void*)p;
}
__device__ __forceinline__ double lds_ld(unsigned a) { return *(lds_double*)(uintptr_t)a; }

// lanes set in the uniform mask m take b, the others a: one v_cndmask per half on the SGPR
// pair (no branch, no EXEC change -- a select the compiler cannot turn into a switch over
// register indices)
__device__ __forceinline__ double select_lanes_d(double a, double b, unsigned long long m) {
  unsigned lo, hi;
  asm("v_cndmask_b32_e64 %0, %1, %2, %3" : "=v"(lo) : "v"(__double2loint(a)), "v"(__double2loint(b)), "s"(m));
  asm("v_cndmask_b32_e64 %0, %1, %2, %3" : "=v"(hi) : "v"(__double2hiint(a)), "v"(__double2hiint(b)), "s"(m));
  return __hiloint2double((int)hi, (int)lo);
}

__device__ __forceinline__ void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

}  // namespace mv
