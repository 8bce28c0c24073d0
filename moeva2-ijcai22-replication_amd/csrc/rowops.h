// Device building blocks of the row kernels (variation, constraint program, Dense chain),
// shared by the per-phase kernels (eval.hip) and the whole-attack kernel (attack.hip).
#pragma once
#include "check.h"
#include "detmath.h"
#include "draws.h"
#include "engine.h"
#include "kernels.h"
#include "philox.h"
#include "wave.h"

namespace mv {

typedef float floatx4 __attribute__((ext_vector_type(4)));

// numpy float remainder (npy_divmod): result takes the divisor's sign
__device__ __forceinline__ double py_mod(double a, double b) {
  double m = fmod(a, b);
  if (m != 0.0) {
    if ((b < 0.0) != (m < 0.0)) m += b;
  } else {
    m = copysign(0.0, b);
  }
  return m;
}

__device__ __forceinline__ double month_of(double f) {
  return floor(f / 100.0) * 12.0 + py_mod(f, 100.0);
}

// Constraint-program tables (ops sorted by code, ABS_SUMDIFF last): global memory
// (k_constraints) or the LDS copy of the problem blob (k_vary).
struct OpTab {
  const int* code;      // [C]
  const int4* arg;      // [C]
  const double2* k;     // [C]
  const int* col;       // [C] original constraint column
  const int* pool;      // [n_pool]
  int C, n_lane;        // ops [0, n_lane) lane-parallel, [n_lane, C) ABS_SUMDIFF
  double tol;
  const double* hlo = nullptr;  // checks builds: the state's history / G range [hlo, hhi)
  const double* hhi = nullptr;
  // slim program (k_genc phase 2, region S): k as fp64 [C], the ABS_SUMDIFF args [C - n_lane]
  const double* k1 = nullptr;
  const int4* sd = nullptr;
};

__device__ __forceinline__ OpTab global_tab(const DProblem& p) {
  OpTab t;
  t.code = p.op_code;
  t.arg = (const int4*)p.op_arg;
  t.k = (const double2*)p.op_k;
  t.col = p.op_col;
  t.pool = p.idx_pool;
  t.C = p.C;
  t.n_lane = p.C - p.n_sumdiff;
  t.tol = p.tol;
  return t;
}

// One constraint column on the ML row x (LDS).  FULL adds the LCLD financial identities;
// ABS_SUMDIFF columns are evaluated wave-parallel (sumdiff_wave) by the caller.
// XR: the row accessor -- a pointer to the LDS row, or any type with operator[](int) (the
// narrow-row kernel's lane-strided row, narrow.h).
template <bool FULL, class XR>
__device__ __forceinline__ double eval_op(const OpTab& t, int c, const XR& x) {
  const int code = t.code[c];
  const int4 ar = t.arg[c];
  switch (code) {
    case 1:  // MV_OP_DIFF (botnet_constraints.py:283-285)
      return x[ar.x] - x[ar.y];
    case 2: {  // MV_OP_RATIO_SAFE (botnet_constraints.py:304-306)
      const double a = x[ar.x], b = x[ar.y];
      return (b != 0.0 ? a / b : 0.0) - t.k[c].x;
    }
    case 9: {  // MV_OP_XOR_AUG (examples/utils.py:7-29)
      const double2 k = t.k[c];
      const bool b1 = x[ar.y] >= k.x;
      const bool b2 = x[ar.z] >= k.y;
      return fabs(x[ar.x] - ((b1 != b2) ? 1.0 : 0.0));
    }
    default:
      break;
  }
  if (FULL) {
    switch (code) {
      case 4: {  // MV_OP_LCLD_INSTALL (lcld_constraints.py:174-177), numpy evaluation order
        const double x0 = x[ar.x], x1 = x[ar.y], x2 = x[ar.z], x3 = x[ar.w];
        const double r = x2 / 1200.0;
        const double base = 1.0 + x2 / 1200.0;
        const double num = (x0 * r) * pow(base, x1);
        const double den = pow(base, x1) - 1.0;
        return fabs(x3 - num / den) - t.k[c].x;
      }
      case 5: {  // MV_OP_LCLD_TERM (:186)
        const double v = x[ar.x];
        return fabs((36.0 - v) * (60.0 - v));
      }
      case 6:  // MV_OP_ABS_RATIO (:189-207)
        return fabs(x[ar.x] - x[ar.y] / x[ar.z]);
      case 7:  // MV_OP_MONTHDIFF (:195-201)
        return fabs(x[ar.x] - (month_of(x[ar.y]) - month_of(x[ar.z])));
      case 8: {  // MV_OP_RATIO_MASKED (:210-216)
        const double den = x[ar.z];
        double ratio = -1.0;
        if (den != 0.0) {
          ratio = x[ar.y] / den;
          if (ratio == __builtin_inf() || ratio != ratio) ratio = -1.0;
        }
        return fabs(x[ar.x] - ratio);
      }
      default:
        break;
    }
  }
  return __builtin_nan("");
}

// The slim program's operand view (k_genc phase 2): slot s < dm is stored mutable feature s,
// held in the wave's row buffer; slot dm + f is feature f of the state's x_init (region X,
// shared by the waves).  The row buffer is then dm doubles instead of D.
struct SlotRow {
  const double* row;
  const double* xi;
  int dm;
  __device__ __forceinline__ double operator[](int s) const {
    return s < dm ? row[s] : xi[s - dm];
  }
};

// |sum(pool[a0:a1]) - sum(pool[a1:a2])| with all 64 lanes, one reduction of the per-lane
// differences (exact for the integer-valued features of every shipped program; the
// summation order differs from numpy otherwise).
template <class XR>
__device__ __forceinline__ double sumdiff_wave(const OpTab& t, int c, const XR& x, int lane) {
  const int4 ar = t.sd ? t.sd[c - t.n_lane] : t.arg[c];
  double s = 0.0;
  for (int q = ar.x + lane; q < ar.y; q += 64) s += x[t.pool[q]];
  for (int q = ar.y + lane; q < ar.z; q += 64) s -= x[t.pool[q]];
  return fabs(wave_sum(s));
}

// Constraint row -> G columns (+ history columns); returns the wave-uniform f3 = sum(G).
// Values <= tol -> 0 (Constraints.evaluate); with clamp, G * (G > 0) (default_problem.py:93-97).
template <bool FULL>
__device__ __forceinline__ double constraints_row(const OpTab& t, const double* xrow, int lane,
                                                  double* grow, double* hcols,
                                                  bool clamp_positive) {
  double acc3 = 0.0;
  for (int c = lane; c < t.n_lane; c += 64) {
    double v = eval_op<FULL>(t, c, xrow);
    if (v <= t.tol) v = 0.0;
    const double g = clamp_positive ? v * (v > 0.0 ? 1.0 : 0.0) : v;
    if (grow) grow[t.col[c]] = g;
    if (hcols) hcols[t.col[c]] = g;
    acc3 += g;
  }
  for (int c = t.n_lane; c < t.C; ++c) {
    double v = sumdiff_wave(t, c, xrow, lane);
    if (v <= t.tol) v = 0.0;
    const double g = clamp_positive ? v * (v > 0.0 ? 1.0 : 0.0) : v;
    if (lane == 0) {
      if (grow) grow[t.col[c]] = g;
      if (hcols) hcols[t.col[c]] = g;
      acc3 += g;
    }
  }
  return wave_sum(acc3);
}

// k_vary's constraint evaluation: each lane keeps its (at most OPS_REG) lane-parallel ops
// packed in registers -- code (4 bits) | a0 (14) | a1 (14) -- so a row's operand reads are
// independent LDS loads issued back to back.  DIFF and RATIO_SAFE (the botnet program) are
// evaluated inline; other codes, and ops beyond OPS_REG per lane, go through eval_op.
constexpr int OPS_REG = 6;

__device__ __forceinline__ unsigned pack_op(const OpTab& t, int c) {
  const int4 ar = t.arg[c];
  return (unsigned)t.code[c] | ((unsigned)ar.x << 4) | ((unsigned)ar.y << 18);
}

// (The slim program has its own straight-line form, constraints_slim below.)
template <bool FULL, class XR>
__device__ __forceinline__ double constraints_regs(const OpTab& t, const unsigned* opw, int kops,
                                                   const XR& xrow, int lane, double* grow,
                                                   double* hcols) {
  double va[OPS_REG], vb[OPS_REG];
#pragma unroll
  for (int k = 0; k < OPS_REG; ++k) {
    if (k < kops) {
      va[k] = xrow[(opw[k] >> 4) & 0x3FFF];
      vb[k] = xrow[opw[k] >> 18];
    }
  }
  double acc3 = 0.0;
#pragma unroll
  for (int k = 0; k < OPS_REG; ++k) {
    const int c = lane + 64 * k;
    if (k < kops && c < t.n_lane) {
      const int code = opw[k] & 15;
      double v;
      if (code == 1)
        v = va[k] - vb[k];
      else if (code == 2)
        v = (vb[k] != 0.0 ? va[k] / vb[k] : 0.0) - t.k[c].x;
      else
        v = eval_op<FULL>(t, c, xrow);
      if (v <= t.tol) v = 0.0;
      const double g = v * (v > 0.0 ? 1.0 : 0.0);
      const int col = MV_IDX(t.col[c], t.C, CK_CONS_COL);
      if (grow) grow[col] = g;
      if (hcols) *MV_PTR(hcols + col, t.hlo, t.hhi, CK_AT_HIST2) = g;
      acc3 += g;
    }
  }
  for (int c = lane + 64 * OPS_REG; c < t.n_lane; c += 64) {
    double v = eval_op<FULL>(t, c, xrow);
    if (v <= t.tol) v = 0.0;
    const double g = v * (v > 0.0 ? 1.0 : 0.0);
    if (grow) grow[t.col[c]] = g;
    if (hcols) *MV_PTR(hcols + MV_IDX(t.col[c], t.C, CK_CONS_COL), t.hlo, t.hhi, CK_AT_HIST2) = g;
    acc3 += g;
  }
  double sdsum = 0.0;  // ABS_SUMDIFF columns (wave-uniform values)
  for (int c = t.n_lane; c < t.C; ++c) {
    double v = sumdiff_wave(t, c, xrow, lane);
    if (v <= t.tol) v = 0.0;
    const double g = v * (v > 0.0 ? 1.0 : 0.0);
    if (lane == 0) {
      if (grow) grow[t.col[c]] = g;
      if (hcols)
        *MV_PTR(hcols + MV_IDX(t.col[c], t.C, CK_CONS_COL), t.hlo, t.hhi, CK_AT_HIST2) = g;
    }
    sdsum += g;
  }
  return wave_sum(acc3) + sdsum;
}

// The slim program's operands as LDS byte addresses in registers (k_genc; DProblem.slim),
// set up once per workgroup by slim_ops: lane op k of this lane reads oa[k] and ob[k] -- the
// SlotRow slot's place in the wave's row buffer (row_at) or region X (xi_at) -- and an unused
// op slot reads the 0.0 of region S (zero_at) twice, so its column value is 0 - 0 = 0 with no
// validity test.  rbits: the lane's RATIO_SAFE ops (bit k); rg: the op groups k with any
// RATIO_SAFE lane (wave-uniform: the others never enter the quotient branch).  sd_reg
// (DProblem.sd_reg): lane l's term of either side of ABS_SUMDIFF op j in sdl / sdr, the zero
// slot past a side's end.
constexpr int SD_REG = 2;
struct SlimOps {
  unsigned oa[OPS_REG], ob[OPS_REG];
  unsigned rbits;
  int rg;
  bool sd_reg;
  unsigned sdl[SD_REG], sdr[SD_REG];
};
__device__ __forceinline__ void slim_ops(const OpTab& t, const unsigned* opw, int kops,
                                         bool sd_reg, const void* row, const void* xi,
                                         const void* zero, int dm, int lane, SlimOps& so) {
  const unsigned row_at = lds_addr(row), xi_at = lds_addr(xi), zero_at = lds_addr(zero);
  auto slot_at = [&](int s) { return s < dm ? row_at + 8u * s : xi_at + 8u * (s - dm); };
  so.rbits = 0;
  so.rg = 0;
#pragma unroll
  for (int k = 0; k < OPS_REG; ++k) {
    const unsigned w = opw[k];
    const bool live = k < kops && lane + 64 * k < t.n_lane;
    so.oa[k] = live ? slot_at((w >> 4) & 0x3FFF) : zero_at;
    so.ob[k] = live ? slot_at(w >> 18) : zero_at;
    const bool ratio = live && (w & 15) == 2;
    so.rbits |= ratio ? 1u << k : 0u;
    so.rg |= __ballot(ratio) ? 1 << k : 0;
  }
  so.sd_reg = sd_reg;
  auto at = [&](int q, int end) { return q < end ? slot_at(t.pool[q]) : zero_at; };
#pragma unroll
  for (int j = 0; j < SD_REG; ++j) {
    so.sdl[j] = zero_at;
    so.sdr[j] = zero_at;
    if (sd_reg && j < t.C - t.n_lane) {
      const int4 ar = t.sd[j];
      so.sdl[j] = at(ar.x + lane, ar.y);
      so.sdr[j] = at(ar.y + lane, ar.z);
    }
  }
}

// constraints_regs for the slim program (every lane op DIFF or RATIO_SAFE, tol >= 0),
// straight-line: every lane takes its op's difference, the RATIO_SAFE lanes of a group in rg
// replace it with the quotient, and the clamp is  g = v <= tol ? 0 : v  -- the value of
// constraints_regs's (v <= tol -> 0; v * (v > 0)) once tol >= 0: a v above tol is positive.
// The unused slots' g = 0 leave the column sum bit-identical (it is never -0).  sd_reg:
// (0 + l) - r  with the zero slot for an absent term is bit-identical to sumdiff_wave's
// conditional += / -= (s - +0 == s); otherwise sumdiff_wave on the SlotRow view.
template <class XR>
__device__ __forceinline__ double constraints_slim(const OpTab& t, const SlimOps& so,
                                                   const XR& xrow, int lane, double* grow,
                                                   double* hcols) {
  double va[OPS_REG], vb[OPS_REG];
#pragma unroll
  for (int k = 0; k < OPS_REG; ++k) {
    va[k] = lds_ld(so.oa[k]);
    vb[k] = lds_ld(so.ob[k]);
  }
  const double tol = t.tol;
  double acc3 = 0.0;
  // the columns' stores (G, history) in their own copy of the loop: a per-op store test
  // kept a lane mask per op live across the row loop
  auto lane_ops = [&](auto st) __attribute__((always_inline)) {
#pragma unroll
    for (int k = 0; k < OPS_REG; ++k) {
      const int c = lane + 64 * k;
      double v = va[k] - vb[k];
      if ((so.rg >> k) & 1)
        if ((so.rbits >> k) & 1) v = (vb[k] != 0.0 ? va[k] / vb[k] : 0.0) - t.k1[c];
      const double g = v <= tol ? 0.0 : v;
      if (decltype(st)::value && c < t.n_lane) {
        const int col = MV_IDX(t.col[c], t.C, CK_CONS_COL);
        if (grow) grow[col] = g;
        if (hcols) *MV_PTR(hcols + col, t.hlo, t.hhi, CK_AT_HIST2) = g;
      }
      acc3 += g;
    }
  };
  if (grow || hcols)
    lane_ops(std::true_type{});
  else
    lane_ops(std::false_type{});
  double sdsum = 0.0;  // ABS_SUMDIFF columns (wave-uniform values)
  auto sd_col = [&](int c, double v) {
    const double g = v <= tol ? 0.0 : v;
    if (lane == 0) {
      if (grow) grow[t.col[c]] = g;
      if (hcols) *MV_PTR(hcols + MV_IDX(t.col[c], t.C, CK_CONS_COL), t.hlo, t.hhi, CK_AT_HIST2) = g;
    }
    sdsum += g;
  };
  const int nsd = t.C - t.n_lane;
  if (so.sd_reg) {
#pragma unroll
    for (int j = 0; j < SD_REG; ++j) {
      if (j < nsd) {
        const double l = lds_ld(so.sdl[j]);
        const double r = lds_ld(so.sdr[j]);
        sd_col(t.n_lane + j, fabs(wave_sum((0.0 + l) - r)));
      }
    }
  } else {
    for (int c = t.n_lane; c < t.C; ++c) sd_col(c, sumdiff_wave(t, c, xrow, lane));
  }
  return wave_sum(acc3) + sdsum;
}

// constraints_slim in two halves around a batched reduction (k_genc, so.sd_reg): the lane
// ops' partial f3 (acc3) and each ABS_SUMDIFF column's lane value ((0 + l) - r, 0 past the
// program's columns) -- then, from their wave totals, the sum-diff columns' stores and f3,
// in constraints_slim's order.
__device__ __forceinline__ void constraints_slim_parts(const OpTab& t, const SlimOps& so, int lane,
                                                       double* grow, double* hcols, double& acc3,
                                                       double (&sdv)[SD_REG]) {
  double va[OPS_REG], vb[OPS_REG];
#pragma unroll
  for (int k = 0; k < OPS_REG; ++k) {
    va[k] = lds_ld(so.oa[k]);
    vb[k] = lds_ld(so.ob[k]);
  }
  const double tol = t.tol;
  acc3 = 0.0;
  auto lane_ops = [&](auto st) __attribute__((always_inline)) {
#pragma unroll
    for (int k = 0; k < OPS_REG; ++k) {
      const int c = lane + 64 * k;
      double v = va[k] - vb[k];
      if ((so.rg >> k) & 1)
        if ((so.rbits >> k) & 1) v = (vb[k] != 0.0 ? va[k] / vb[k] : 0.0) - t.k1[c];
      const double g = v <= tol ? 0.0 : v;
      if (decltype(st)::value && c < t.n_lane) {
        const int col = MV_IDX(t.col[c], t.C, CK_CONS_COL);
        if (grow) grow[col] = g;
        if (hcols) *MV_PTR(hcols + col, t.hlo, t.hhi, CK_AT_HIST2) = g;
      }
      acc3 += g;
    }
  };
  if (grow || hcols)
    lane_ops(std::true_type{});
  else
    lane_ops(std::false_type{});
  const int nsd = t.C - t.n_lane;
#pragma unroll
  for (int j = 0; j < SD_REG; ++j) {
    const double l = lds_ld(so.sdl[j]);
    const double r = lds_ld(so.sdr[j]);
    sdv[j] = j < nsd ? (0.0 + l) - r : 0.0;
  }
}
__device__ __forceinline__ double constraints_slim_finish(const OpTab& t, int lane, double* grow,
                                                          double* hcols, double acc3_total,
                                                          const double (&sd_total)[SD_REG]) {
  const double tol = t.tol;
  double sdsum = 0.0;
  const int nsd = t.C - t.n_lane;
#pragma unroll
  for (int j = 0; j < SD_REG; ++j) {
    if (j < nsd) {
      const int c = t.n_lane + j;
      const double v = fabs(sd_total[j]);
      const double g = v <= tol ? 0.0 : v;
      if (lane == 0) {
        if (grow) grow[t.col[c]] = g;
        if (hcols) *MV_PTR(hcols + MV_IDX(t.col[c], t.C, CK_CONS_COL), t.hlo, t.hhi, CK_AT_HIST2) = g;
      }
      sdsum += g;
    }
  }
  return acc3_total + sdsum;
}

// pymoo PolynomialMutation for one gene (softmax_mutation.py:77-103), no FMA contraction,
// det_pow (detmath.h; its bit-identical FMA-product form) for np.power.
__device__ __forceinline__ double poly_mut(double x, double xl, double xu, double u, double eta) {
  const double d1 = (x - xl) / (xu - xl);
  const double d2 = (xu - x) / (xu - xl);
  const double mp = 1.0 / (eta + 1.0);
  double dq;
  if (u <= 0.5) {
    const double xy = 1.0 - d1;
    const double val = 2.0 * u + (1.0 - 2.0 * u) * det_pow<true>(xy, eta + 1.0);
    dq = det_pow<true>(val, mp) - 1.0;
  } else {
    const double xy = 1.0 - d2;
    const double val = 2.0 * (1.0 - u) + 2.0 * (u - 0.5) * det_pow<true>(xy, eta + 1.0);
    dq = 1.0 - det_pow<true>(val, mp);
  }
  double y = x + dq * (xu - xl);
  if (y < xl) y = xl;
  if (y > xu) y = xu;
  return y;
}


__device__ __forceinline__ void scatter_gene(const DProblem& p, double* __restrict__ xrow,
                                             int info, double x) {
  const int kind = info & 3;
  const int feat = (info >> 17) & 0x7FFF;
  if (kind != 2) {
    xrow[feat] = x;
  } else {
    const int o0 = p.ohe_off[feat], o1 = p.ohe_off[feat + 1];
    for (int k = o0; k < o1; ++k) xrow[p.ohe_feat[k]] = (x == (double)(k - o0)) ? 1.0 : 0.0;
  }
}

// scatter_gene with the one-hot tables in LDS (region B)
__device__ __forceinline__ void scatter_gene_tab(const int* __restrict__ ooff,
                                                 const int* __restrict__ ofeat,
                                                 double* __restrict__ xrow, int info, double x) {
  const int kind = info & 3;
  const int feat = (info >> 17) & 0x7FFF;
  if (kind != 2) {
    xrow[feat] = x;
  } else {
    const int o0 = ooff[feat], o1 = ooff[feat + 1];
    for (int k = o0; k < o1; ++k) xrow[ofeat[k]] = (x == (double)(k - o0)) ? 1.0 : 0.0;
  }
}

__device__ __forceinline__ int rdl(int v, int k) { return __builtin_amdgcn_readlane(v, k); }


// pymoo 0.4.2.2 SimulatedBinaryCrossover._do for one gene of one mating [pymoo-recall;
// SURVEY.md §7 "north_star says SBX"]: the child of `side` (0: c[0], 1: c[1]) from parents
// p0 = X[0], p1 = X[1] with bounds [xl, xu] (widened for integer genes by the caller), the
// uniform `rand` of calc_betaq and the swap draw; numpy's evaluation order, no FMA.
__device__ __forceinline__ double sbx_child(double p0, double p1, double xl, double xu,
                                            double rand, bool swap, int side, double eta) {
  const double y1 = p0 < p1 ? p0 : p1;
  const double y2 = p0 < p1 ? p1 : p0;
  double delta = y2 - y1;
  if (delta < 1.0e-10) delta = 1.0e-10;
  // c[0] takes c1 (lower side) unless swapped; c[1] the other one
  const bool low = (side == 0) != swap;
  const double beta = low ? 1.0 + (2.0 * (y1 - xl) / delta) : 1.0 + (2.0 * (xu - y2) / delta);
  const double alpha = 2.0 - det_pow<true>(beta, -(eta + 1.0));
  const double ex = 1.0 / (eta + 1.0);
  const double betaq =
      rand <= (1.0 / alpha) ? det_pow<true>((rand * alpha), ex)
                            : det_pow<true>((1.0 / (2.0 - rand * alpha)), ex);
  double c = low ? 0.5 * ((y1 + y2) - betaq * delta) : 0.5 * ((y1 + y2) + betaq * delta);
  if (c < xl) c = xl;  // set_to_bounds_if_outside_by_problem
  if (c > xu) c = xu;
  return c;
}

// MixedVariableMutation of one gene (moeva2.py:104-111): real_pm, or int_pm =
// IntegerFromFloatMutation (bounds widened by 0.5 - 1e-16, np.round half-to-even, clamp).
__device__ __forceinline__ double mutate_gene(double x, double xl, double xu, bool is_real,
                                              double u, double eta) {
  const double y = poly_mut(x, is_real ? xl : xl - INT_WIDEN, is_real ? xu : xu + INT_WIDEN, u,
                            eta);
  if (is_real) return y;
  double yi = rint(y);
  if (yi < xl) yi = xl;
  if (yi > xu) yi = xu;
  return yi;
}

constexpr int MUT_CAP = 4;     // mutations per row precomputed in the prologue (registers)

// SBX option of the mixed-variable crossover (real_sbx / int_sbx = IntegerFromFloat-
// Crossover(SBX): widened bounds, np.round, then the build's clamp to [xl, xu]) for one row
// whose genes lane + 64 t hold the row's own parent.  Mating m's draws per gene g: one
// Philox word (index m * MUT_J + g, TAG_SBX): bit 0 = 0 -> the variable crosses
// (prob_per_variable 0.5), bit 1 -> swap c1/c2, words y, z -> calc_betaq's uniform.  The
// mating-level draw (prob 0.9) of each subset comes from TAG_CX as for two-point.
// The crossed genes' children are computed spread over the wave's lanes: pass 1 finds the
// genes that cross (each lane its genes lane + 64 t) and appends their indices to the wave's
// LDS list sdesc in (t, lane) order; pass 2 gives item s of the list to lane s % 64 in round
// s / 64, which recomputes the gene's draw and inputs and writes the child to sres[s]; pass
// 3 hands each child back.  With the children computed in place (one t at a time) every lane
// paid for all NT slots' two det_pow chains whenever any lane of the slot crossed; spread,
// a row costs ceil(crossed / 64) rounds.  Same draws, same arithmetic: bit-identical.
template <int NT>
__device__ __forceinline__ void sbx_row(double* x, const int* ginf, const double* gown,
                                        const double* goth, const double* gl, const double* gu,
                                        int V, const int* fidx, int m, int side, int on0, int on1,
                                        const Rng& rng,
                                        int gen, double eta, int lane, int* sdesc,
                                        double* sres) {
  int slot[NT];
  int cnt = 0;  // wave-uniform
#pragma unroll
  for (int t = 0; t < NT; ++t) {
    const int g = lane + 64 * t;
    bool need = false;
    if (g < V) {
      const bool real = (ginf[t] & 3) == 0;
      if (real ? on0 : on1) {
        const double own = x[t], oth = goth[g];
        const u32x4 w = rng.draw((uint32_t)(m * MUT_J + fidx[g]), (uint32_t)gen, TAG_SBX);
        need = !(w.x & 1u) && fabs(own - oth) > 1.0e-14;
      }
    }
    const unsigned long long mask = __ballot(need);
    const int s = cnt + (int)__builtin_amdgcn_mbcnt_hi((unsigned)(mask >> 32),
                                                        __builtin_amdgcn_mbcnt_lo((unsigned)mask, 0u));
    slot[t] = need ? s : -1;
    if (need) sdesc[s] = g | (((ginf[t] & 3) == 0 ? 1 : 0) << 16);
    cnt += __popcll(mask);
  }
  for (int r = 0; r < cnt; r += 64) {
    const int s = r + lane;
    if (s < cnt) {
      const int d = sdesc[s];
      const int g = MV_IDX(d & 0xFFFF, V, CK_GEN_SBX);
      const bool real = (d >> 16) != 0;
      const double own = gown[g], oth = goth[g];
      const double p0 = side == 0 ? own : oth, p1 = side == 0 ? oth : own;
      const u32x4 w = rng.draw((uint32_t)(m * MUT_J + fidx[g]), (uint32_t)gen, TAG_SBX);
      const double lo = gl[g], hi = gu[g];
      double c = sbx_child(p0, p1, real ? lo : lo - INT_WIDEN, real ? hi : hi + INT_WIDEN,
                           u53(w.y, w.z), (w.x & 2u) != 0u, side, eta);
      if (!real) {
        c = rint(c);
        if (c < lo) c = lo;
        if (c > hi) c = hi;
      }
      sres[s] = c;
    }
  }
#pragma unroll
  for (int t = 0; t < NT; ++t)
    if (slot[t] >= 0) x[t] = sres[slot[t]];
}

// Every mutation of row i (the whole geometric-gap draw sequence of mutation_draws over the
// Vr genes, no register cache): the SBX rows take this path since their crossed values exist
// only in the row loop.  Positions map to stored genes through cmap (-1: a fixed gene of the
// compact layout, whose mutation is the identity).
template <int NT>
__device__ __forceinline__ void mutate_row_full(double* x, const uint32_t* s_geo,
                                                const int* s_ginfo, const int* s_cmap,
                                                const double* gl, const double* gu, int Vr, int i,
                                                const Rng& rng, int gen, double eta, int lane) {
  const float lq = __log2f(1.0f - 1.0f / (float)Vr);
  int pos = -1;
  for (int j = 0;; ++j) {
    const u32x4 w = rng.draw((uint32_t)(i * MUT_J + j), (uint32_t)gen, TAG_MUT_MASK);
    pos += 1 + geo_gap(s_geo, Vr, w.x, lq);
    if (pos >= Vr) break;
    const int cp = s_cmap[pos];
    if (cp >= 0 && (cp & 63) == lane) {
      double xv = 0.0;
#pragma unroll
      for (int t = 0; t < NT; ++t)
        if (cp == lane + 64 * t) xv = x[t];
      xv = mutate_gene(xv, gl[cp], gu[cp], (s_ginfo[cp] & 3) == 0, u53(w.y, w.z), eta);
#pragma unroll
      for (int t = 0; t < NT; ++t)
        if (cp == lane + 64 * t) x[t] = xv;
    }
  }
}

__device__ __forceinline__ bool gene_swapped(int info, int on0, int lo0, int hi0, int on1,
                                             int lo1, int hi1) {
  const int sub = (info >> 2) & 0x7FFF;
  return (info & 3) == 0 ? (on0 && sub >= lo0 && sub < hi0) : (on1 && sub >= lo1 && sub < hi1);
}


__device__ __forceinline__ double rdl_d(double v, int k) {
  const int lo = __builtin_amdgcn_readlane(__double2loint(v), k);
  const int hi = __builtin_amdgcn_readlane(__double2hiint(v), k);
  return __hiloint2double(hi, lo);
}

// Softmax of the fp32 logits z[0..nout) (held as fp64, max mx) as Keras computes it in fp32
// (tf.nn.softmax; classifier.py:23-29): h_k = z_k - max in fp32, e_k = exp(h_k) rounded to
// fp32, den = the class-order fp32 sum of e_k, p_c = e_c / den in fp32.  Only exp is taken
// in fp64 and rounded once (the correctly rounded fp32 exp, independent of any expf
// implementation, so oracle/device_order.py reproduces it bit for bit); every other step is
// Keras's fp32 arithmetic.  This matters beyond the last bit: near f1 = 1 the fp32 sum
// 1 + e saturates -- f1 is exactly 1.0 for margins above ~16.6 and moves in 2^-24 steps --
// and those plateaus shape the attack's early search.  A softmax computed in fp64 and rounded
// once resolves that region twice as finely and measurably changes the end result: botnet
// rq1 o4 85 % over 64 seeds vs 91 % with this arithmetic, 92 % for the numpy (Keras-order)
// oracle.
// Fully unrolled over the at most 8 classes (a runtime-indexed array would live in scratch).
__device__ __forceinline__ void softmax_e(const double (&z)[8], int nout, double mx,
                                          float (&e)[8], float& den) {
  const float m = (float)mx;
  den = 0.f;
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    e[k] = 0.f;
    if (k < nout) {
      const float h = (float)z[k] - m;
      e[k] = (float)exp((double)h);
      den = den + e[k];
    }
  }
}
__device__ __forceinline__ double softmax_pick(const double (&z)[8], int nout, double mx, int c) {
  float e[8], den;
  softmax_e(z, nout, mx, e, den);
  float pc = 0.f;
#pragma unroll
  for (int k = 0; k < 8; ++k) pc = k == c ? e[k] : pc;
  return (double)(pc / den);
}
__device__ __forceinline__ void softmax_all(const double (&z)[8], int nout, double mx,
                                            float (&prob)[8]) {
  float e[8], den;
  softmax_e(z, nout, mx, e, den);
#pragma unroll
  for (int k = 0; k < 8; ++k) prob[k] = e[k] / den;
}

// Async global -> LDS copy of nbytes (a 1-KiB multiple): 16 B per lane, 1 KiB per wave
// instruction, the workgroup's waves interleaved.
template <int T = VARY_T>
__device__ __forceinline__ void glds_copy(unsigned char* lds, const unsigned char* g,
                                          unsigned nbytes, int wave, int lane) {
  for (unsigned off = wave * 1024u; off < nbytes; off += T * 16u)
    __builtin_amdgcn_global_load_lds(g + off + lane * 16, lds + off, 16, 0, 0);
}

// Rows of one k_gen / k_cons workgroup: a chunk of one state's rows; wave w takes rows
// i0 + w + 4k (k < nrw).
struct RowChunk {
  int b, i0, i1, nrw;
};
// XCD-aware order: the dispatcher deals workgroup i to XCD i mod 8, so logical chunk ids
// are renumbered to keep consecutive ones -- the chunks of one state, which read the same
// parents and state blob -- on one XCD and its L2.
__device__ __forceinline__ int xcd_local_id() {
  constexpr int NX = 8;
  const int G = gridDim.x, i = blockIdx.x;
  const int q = G / NX, r = G % NX, x = i % NX, k = i / NX;
  return x < r ? x * (q + 1) + k : r * (q + 1) + (x - r) * q + k;
}
template <int W = VARY_W>
__device__ __forceinline__ RowChunk row_chunk(int n, int rows_wg, int wave) {
  RowChunk r;
  const int nchunk = (n + rows_wg - 1) / rows_wg;
  const int id = xcd_local_id();
  r.b = id / nchunk;
  r.i0 = (id - r.b * nchunk) * rows_wg;
  r.i1 = min(n, r.i0 + rows_wg);
  const int span = r.i1 - r.i0 - wave;
  r.nrw = span > 0 ? (span + W - 1) / W : 0;
  return r;
}


constexpr int M2_ROWS = 64;
constexpr int M2_ALD = 72;  // layer-0 chunk row stride (floats): 8 mod 64 makes the MFMA A-operand
                            // ds_read_b128 groups conflict-free (68 was 2-way in half the groups)

__host__ __device__ inline int mlp2_hmax(const DProblem& p) {
  int h = 16;
  for (int l = 1; l < p.n_layers; ++l) h = p.dims[l] > h ? p.dims[l] : h;
  return h;
}
// head: row states (256 B), the final layer's weights and bias, the hidden layers' biases
__host__ __device__ inline int mlp2_hidden_bias_floats(const DProblem& p) {
  int n = 0;
  for (int l = 1; l + 1 < p.n_layers; ++l) n += p.dims[l + 1];
  return n;
}
__host__ __device__ inline size_t mlp2_head(const DProblem& p) {
  const int nl = p.n_layers;
  return 256 + (((size_t)(p.dims[nl - 1] * p.dims[nl] + p.dims[nl] + mlp2_hidden_bias_floats(p)) *
                     4 + 15) & ~(size_t)15);
}
// The hidden ping-pong H aliases the layer-0 chunk buffers (free once layer 0 is done), so
// four workgroups fit a CU's LDS.
__host__ __device__ inline int mlp2_region_floats(const DProblem& p) {
  const int a0 = 2 * M2_ROWS * M2_ALD, h = 2 * M2_ROWS * (mlp2_hmax(p) + 4);
  return a0 > h ? a0 : h;
}
// The final layer's per-wave partial sums [4][M2_ROWS][n_out] go to the free half of the
// ping-pong when they fit there, else after the region.
__host__ __device__ inline bool mlp2_part_inplace(const DProblem& p) {
  return 4 * p.dims[p.n_layers] <= mlp2_hmax(p) + 4;
}
// xml_direct: the ML scaler at the mutable features (mlS, mlM: Dm4 doubles each) staged in
// LDS after the tile buffers
__host__ __device__ inline size_t mlp2_sc_off(const DProblem& p) {
  return mlp2_head(p) + (size_t)mlp2_region_floats(p) * 4 +
         (mlp2_part_inplace(p) ? 0 : (size_t)4 * M2_ROWS * p.dims[p.n_layers] * 4);
}
__host__ __device__ inline size_t mlp2_lds(const DProblem& p) {
  return mlp2_sc_off(p) + (p.xml_direct ? (size_t)2 * p.Dm4 * 8 : 0);
}

// A wave's share of a layer's (column tile, row tile) grid: column tiles cb + 4cj over all
// four row tiles when the layer has >= 3 column tiles, else the waves also split the row
// tiles (N = 32: two waves per column tile, N = 16: one row tile per wave).
struct TileMap {
  int cb, rt0, nrt;
};
__device__ __forceinline__ TileMap tile_map(int nct, int wave) {
  const int cw = nct >= 3 ? 4 : nct;
  return TileMap{wave % cw, (wave / cw) * cw, cw};
}

// One k-group's 16 fp32 MFMAs per (column tile cj, row tile rt) accumulator: k-step s
// (the float4 component) is the OUTER loop, so consecutive MFMAs write different
// accumulators and never wait for each other's result (a dependent v_mfma_f32_16x16x4f32
// waits out its predecessor's full latency: the rt-outer order ran the layer-0 chunk at ~3x
// its MFMA issue time).  Every accumulator still sums its k in the order x, y, z, w, so
// the result is bit-identical to the rt-outer order.
__device__ __forceinline__ float f4c(const float4& v, int s) {
  return s == 0 ? v.x : s == 1 ? v.y : s == 2 ? v.z : v.w;
}
template <int CJ>
__device__ __forceinline__ void mfma_k4(const float4 (&af)[4], const float4 (&bf)[CJ],
                                        floatx4 (&acc)[CJ][4], int cb, int nct, int nrt) {
  if (nrt == 4) {
#pragma unroll
    for (int s = 0; s < 4; ++s)
#pragma unroll
      for (int cj = 0; cj < CJ; ++cj)
        if (cb + 4 * cj < nct)
#pragma unroll
          for (int rt = 0; rt < 4; ++rt)
            acc[cj][rt] = __builtin_amdgcn_mfma_f32_16x16x4f32(f4c(af[rt], s), f4c(bf[cj], s),
                                                               acc[cj][rt], 0, 0, 0);
  } else {
#pragma unroll
    for (int s = 0; s < 4; ++s)
#pragma unroll
      for (int cj = 0; cj < CJ; ++cj)
        if (cb + 4 * cj < nct)
#pragma unroll
          for (int rt = 0; rt < 4; ++rt)
            if (rt < nrt)
              acc[cj][rt] = __builtin_amdgcn_mfma_f32_16x16x4f32(f4c(af[rt], s), f4c(bf[cj], s),
                                                                 acc[cj][rt], 0, 0, 0);
  }
}

template <int CJ>
__device__ __forceinline__ void mlp2_layer(const float* __restrict__ A, int lda,
                                           const float* __restrict__ Wp, int nkg, int N,
                                           floatx4 (&acc)[CJ][4], TileMap m, int il, int ka) {
  const int nct = N >> 4;
  const int wave = m.cb;
  // loads are unconditional with clamped indices (a conditional load makes hipcc branch and
  // wait vmcnt(0), which would drain the next group's prefetch every step)
  auto load_b = [&](int kg, float4 (&bf)[CJ]) {
    const int kgc = kg < nkg ? kg : nkg - 1;
#pragma unroll
    for (int cj = 0; cj < CJ; ++cj) {
      const int ct = wave + 4 * cj < nct ? wave + 4 * cj : nct - 1;
      bf[cj] = *(const float4*)(Wp + ((size_t)kgc * N + ct * 16 + il) * 16 + 4 * ka);
    }
  };
  auto load_a = [&](int kg, float4 (&af)[4]) {
    const int kgc = kg < nkg ? kg : nkg - 1;
#pragma unroll
    for (int rt = 0; rt < 4; ++rt) {
      const int r = m.rt0 + (rt < m.nrt ? rt : 0);
      af[rt] = *(const float4*)(A + (r * 16 + il) * lda + kgc * 16 + 4 * ka);
    }
  };
  float4 bf[CJ], af[4];
  load_b(0, bf);
  load_a(0, af);
  for (int kg = 0; kg < nkg; ++kg) {
    float4 bn[CJ], an[4];
    load_b(kg + 1, bn);  // next group's weights (L2) while this group's MFMAs run
    load_a(kg + 1, an);
    mfma_k4<CJ>(af, bf, acc, wave, nct, m.nrt);
#pragma unroll
    for (int cj = 0; cj < CJ; ++cj) bf[cj] = bn[cj];
#pragma unroll
    for (int rt = 0; rt < 4; ++rt) af[rt] = an[rt];
  }
}

// Parent genes of one child row (k_gen / k_genc): lane l loads genes l + 64 t from the own or
// the other parent through a buffer resource over the state's pool: the byte offset is the
// chosen parent's row offset plus 8 l (one select per gene between two per-row values), and
// 512 t rides in the load's immediate offset.  Genes past V (the last register's padding
// lanes, never stored) may read past the row; past the pool the buffer's range check returns
// 0 instead of faulting.  Crossover test per gene: pkey = the gene's position in its subset,
// + 0x10000 in the second (integer) subset, so an unsigned compare against each subset's
// segment [lo, lo + n) -- n = 0 when the subset's crossover is off -- decides it with no
// per-gene selects (a gene of one subset is never inside the other's shifted segment).
struct PoolRsrc {
  __amdgpu_buffer_rsrc_t r;
};
__device__ __forceinline__ PoolRsrc pool_rsrc(const double* base, size_t elems) {
  const size_t bytes = elems * 8;
  return PoolRsrc{__builtin_amdgcn_make_buffer_rsrc(
      (void*)base, (short)0, (int)(bytes < 0x7FFFFFFFull ? bytes : 0x7FFFFFFFull), 0x00020000)};
}
__device__ __forceinline__ unsigned parent_key(int ginf) {
  return (unsigned)((ginf >> 2) & 0x7FFF) + ((ginf & 3) == 0 ? 0u : 0x10000u);
}
template <int NT>
__device__ __forceinline__ void load_parent_row(const PoolRsrc& pool, int V, int pr, int cx0,
                                                int cx1, const unsigned (&pkey)[NT], int lane,
                                                double* x, long long pool_elems = 0) {
  typedef unsigned u32x2 __attribute__((ext_vector_type(2)));
  unsigned own8 = (unsigned)(pr & 0xFFFF) * (unsigned)V * 8u;
  unsigned oth8 = (unsigned)(pr >> 16) * (unsigned)V * 8u;
  // opaque, so the compiler selects these two offsets instead of the two row indices (which
  // it then multiplied per gene: a quarter-rate v_mul_lo_u32 each)
  asm("" : "+s"(own8), "+s"(oth8));
  own8 += 8u * (unsigned)lane;
  oth8 += 8u * (unsigned)lane;
  asm("" : "+v"(own8), "+v"(oth8));  // and 512 t stays the loads' immediate offset
  const int s0 = (cx0 >> 1) & 0x7FFF, s1 = (cx1 >> 1) & 0x7FFF;
  const unsigned lo0 = (unsigned)s0, lo1 = (unsigned)s1 + 0x10000u;
  const unsigned n0 = (cx0 & 1) ? (unsigned)((cx0 >> 16) - s0) : 0u;
  const unsigned n1 = (cx1 & 1) ? (unsigned)((cx1 >> 16) - s1) : 0u;
#pragma unroll
  for (int t = 0; t < NT; ++t) {
    const bool cross = pkey[t] - lo0 < n0 || pkey[t] - lo1 < n1;
    const unsigned off = cross ? oth8 : own8;
    if (MV_CHECKS_ON && lane + 64 * t < V)
      (void)MV_IDX((long long)(off / 8 + 64 * t), pool_elems, CK_AT_PARENT);
    const u32x2 w = __builtin_amdgcn_raw_buffer_load_b64(pool.r, off + 512u * t, 0, 0);
    x[t] = __hiloint2double((int)w.y, (int)w.x);
  }
}

// The cached mutations of row k (position / value q held by lane 4 k + q, row_draws): each
// position is wave-uniform, so register t = pos / 64 takes the value on lane pos % 64 through
// a lane-mask select on every register (a scalar branch on t made the compiler select a
// pointer into x, which kept the caller's row buffers in scratch, or copy every register).
template <int NT, int CAP>
__device__ __forceinline__ void apply_row_mutations(double* x, int nmut, int mposv, double mvalv,
                                                    int k, int lane) {
#pragma unroll
  for (int q = 0; q < CAP; ++q) {
    if (q >= nmut) break;  // (uniform: no readlane for the absent slots)
    const int pr = rdl(mposv, CAP * k + q);  // stored gene; -1: a fixed gene (compact layout)
    if (pr >= 0) {
      const int pos = MV_IDX(pr, 64 * NT, CK_GEN_APPLY);
      const double y = rdl_d(mvalv, CAP * k + q);
      const int tt = pos >> 6;
      const unsigned long long m = 1ull << (pos & 63);
#pragma unroll
      for (int t = 0; t < NT; ++t) x[t] = select_lanes_d(x[t], y, t == tt ? m : 0ull);
    }
  }
}

// The planned mutations of an SBX row k (lane PLAN_MUT k + q: mw word, PM uniform), applied
// to the row's SBX children: the gene's lane mutates it (the order of distinct positions does
// not matter).
template <int NT>
__device__ __forceinline__ void plan_mutate_row(double* x, int nmut, int mwv, double muv, int k,
                                                int lane, const double* gl, const double* gu,
                                                int V, double eta) {
  for (int q = 0; q < nmut; ++q) {
    const int w = rdl(mwv, PLAN_MUT * k + q);
    const double u = rdl_d(muv, PLAN_MUT * k + q);
    const int cq = MV_IDX(w & 0xFFFF, V, CK_GEN_APPLY);
    const int tt = cq >> 6;
    if (lane == (cq & 63)) {
      double xv = 0.0;
#pragma unroll
      for (int t = 0; t < NT; ++t)
        if (t == tt) xv = x[t];
      xv = mutate_gene(xv, gl[cq], gu[cq], ((w >> 16) & 1) != 0, u, eta);
#pragma unroll
      for (int t = 0; t < NT; ++t)
        if (t == tt) x[t] = xv;
    }
  }
}

// bf16 perf mode ------------------------------------------------------------------------
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

// Eight fp32 activations (two float4) rounded to bf16 (v_cvt_pk_bf16_f32, RNE); zeros when
// the lane's k lies past the layer's K (the LDS there is not part of the operand).
__device__ __forceinline__ bf16x8 to_bf16x8(float4 lo, float4 hi, bool on) {
  bf16x8 r;
  r[0] = (__bf16)(on ? lo.x : 0.f);
  r[1] = (__bf16)(on ? lo.y : 0.f);
  r[2] = (__bf16)(on ? lo.z : 0.f);
  r[3] = (__bf16)(on ? lo.w : 0.f);
  r[4] = (__bf16)(on ? hi.x : 0.f);
  r[5] = (__bf16)(on ? hi.y : 0.f);
  r[6] = (__bf16)(on ? hi.z : 0.f);
  r[7] = (__bf16)(on ? hi.w : 0.f);
  return r;
}

// mlp2_layer in the bf16 mode: k-steps of 32 on v_mfma_f32_16x16x32_bf16.  Lane (il, ka)
// holds k = 32 s + 8 ka + j (j < 8) of step s: its A operand is two ds_read_b128 of its row
// (rounded to bf16), its B operand one dwordx4 of Wb[kg0 + s][n][32].  K (a multiple of 16)
// is the number of k of A processed here; lanes whose 8 k lie past K contribute zeros.
template <int CJ>
__device__ __forceinline__ void mlp2_layer_bf(const float* __restrict__ A, int lda, int K,
                                              const unsigned short* __restrict__ Wb, int kg0,
                                              int N, floatx4 (&acc)[CJ][4], TileMap m, int il,
                                              int ka) {
  const int nct = N >> 4;
  const int wave = m.cb;
  const int nst = (K + 31) >> 5;
  const __bf16* W = (const __bf16*)Wb;
  auto load_b = [&](int s, bf16x8 (&bf)[CJ]) {
    const int sc = s < nst ? s : nst - 1;
#pragma unroll
    for (int cj = 0; cj < CJ; ++cj) {
      const int ct = wave + 4 * cj < nct ? wave + 4 * cj : nct - 1;
      bf[cj] = *(const bf16x8*)(W + ((size_t)(kg0 + sc) * N + ct * 16 + il) * 32 + 8 * ka);
    }
  };
  bf16x8 bf[CJ];
  load_b(0, bf);
  for (int s = 0; s < nst; ++s) {
    bf16x8 bn[CJ];
    load_b(s + 1, bn);  // next step's weights (L2) while this step's MFMAs run
    const int k = 32 * s + 8 * ka;
    const bool on = k < K;
    const int kc = on ? k : 0;
    bf16x8 af[4];
#pragma unroll
    for (int rt = 0; rt < 4; ++rt) {
      const int r = m.rt0 + (rt < m.nrt ? rt : 0);
      const float* ar = A + (r * 16 + il) * lda + kc;
      af[rt] = to_bf16x8(*(const float4*)ar, *(const float4*)(ar + 4), on);
    }
#pragma unroll
    for (int cj = 0; cj < CJ; ++cj) {
      if (wave + 4 * cj < nct) {
#pragma unroll
        for (int rt = 0; rt < 4; ++rt) {
          if (rt >= m.nrt) continue;
          acc[cj][rt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[rt], bf[cj], acc[cj][rt], 0, 0, 0);
        }
      }
    }
#pragma unroll
    for (int cj = 0; cj < CJ; ++cj) bf[cj] = bn[cj];
  }
}

}  // namespace mv
