// Deterministic pow for the variation operators: the same sequence of IEEE double
// operations (+ - * /, frexp/ldexp/floor, no FMA: the library is built with
// -ffp-contract=off) as oracle/device_order.py:det_pow, so the engine's mutated and SBX genes
// are bit-identical to the oracle's wherever the oracle uses it.
//
// Why: numpy's np.power (C library pow) and the device library's pow are both within about
// an ulp of the true value but do not agree bit for bit; one differing last bit in one
// mutated gene makes a state's whole GA trajectory part from the oracle's (the first such
// generation was found with tools/traj_diff.py).  The reference's operators
// (softmax_mutation.py:77-103, pymoo SBX calc_betaq) are the same formulas with this pow.
//
// General exponents: exp(y ln x) with ln x as a double-double (fdlibm e_log.c's
// reduction and polynomial), y ln x as a double-double (Dekker product, no FMA) and fdlibm
// e_exp.c's reduction taking the low word.  Integer exponents up to 64 in magnitude:
// binary powering in double-double.  Measured against np.power (tests/test_detpow_cpu.py):
// at most 1 ulp apart on the operators' argument ranges.  Identity with the oracle is the
// point, not the last bit of np.power.
//
// det_pow<true> (the device's variation operators) takes each exact product from an FMA,
// p = a b, e = fma(a, b, -p), where Dekker's split-based product is exact too: both then
// return the one representable error a b - p, so the result is bit-identical to det_pow<>
// (and to the oracle) at a fraction of the operations.  Dekker is exact unless a partial
// product underflows: y ln x (|y| >= 2^-10, |ln x| >= 2^-53 for x != 1) and the reciprocal
// correction (q rh ~ 1) never do; the binary powering's products do only for x < 1, so
// there the split is kept.
#pragma once
#include <hip/hip_runtime.h>

namespace mv {

// Dekker's exact product without FMA (|a|, |b| < 2^996) and Knuth's two-sum.
__host__ __device__ inline void det_split(double a, double& hi, double& lo) {
  const double t = 134217729.0 * a;  // 2^27 + 1
  hi = t - (t - a);
  lo = a - hi;
}
__host__ __device__ inline void det_two_prod(double a, double b, double& p, double& e) {
  double ah, al, bh, bl;
  det_split(a, ah, al);
  det_split(b, bh, bl);
  p = a * b;
  e = ((ah * bh - p) + ah * bl + al * bh) + al * bl;
}
__host__ __device__ inline void det_two_sum(double a, double b, double& s, double& e) {
  s = a + b;
  const double bb = s - a;
  e = (a - (s - bb)) + (b - bb);
}
template <bool FMA>
__host__ __device__ inline void det_two_prod_x(double a, double b, double& p, double& e) {
  if (FMA) {
    p = a * b;
    e = fma(a, b, -p);
  } else {
    det_two_prod(a, b, p, e);
  }
}
__host__ __device__ inline void det_fast_two_sum(double a, double b, double& s, double& e) {
  s = a + b;
  e = b - (s - a);
}
// double-double product (hi, lo normalised)
template <bool FMA = false>
__host__ __device__ inline void det_dd_mul(double ah, double al, double bh, double bl, double& h,
                                           double& l) {
  double p, e;
  det_two_prod_x<FMA>(ah, bh, p, e);
  e = e + (ah * bl + al * bh);
  det_fast_two_sum(p, e, h, l);
}

// ln x as hi + lo (x > 0 finite): fdlibm e_log.c's reduction x = 2^k (1 + f),
// s = f / (2 + f) and polynomial, the k ln2_hi + f sum kept exact.
__host__ __device__ inline void det_log2(double x, double& hi, double& lo) {
  const double ln2_hi = 6.93147180369123816490e-01, ln2_lo = 1.90821492927058770002e-10;
  const double Lg1 = 6.666666666666735130e-01, Lg2 = 3.999999999940941908e-01,
               Lg3 = 2.857142874366239149e-01, Lg4 = 2.222219843214978396e-01,
               Lg5 = 1.818357216161805012e-01, Lg6 = 1.531383769920937332e-01,
               Lg7 = 1.479819860511658591e-01;
  int e = 0;
  double m = frexp(x, &e);  // x = m 2^e, m in [0.5, 1)
  if (m < 0.7071067811865476) {
    m = m * 2.0;
    e = e - 1;
  }
  const double f = m - 1.0;  // exact (Sterbenz)
  const double k = (double)e;
  const double s = f / (2.0 + f);
  const double z = s * s;
  const double w = z * z;
  const double t1 = w * (Lg2 + w * (Lg4 + w * Lg6));
  const double t2 = z * (Lg1 + w * (Lg3 + w * (Lg5 + w * Lg7)));
  const double R = t2 + t1;
  const double hfsq = 0.5 * f * f;
  double e1;
  det_two_sum(k * ln2_hi, f, hi, e1);  // k ln2_hi is exact (21 trailing zero bits)
  lo = ((k * ln2_lo - hfsq) + s * (hfsq + R)) + e1;
}

// exp(th + tl) (|tl| << |th|): fdlibm e_exp.c's reduction and rational form with the
// low part of the argument folded into the reduction's low word.
__host__ __device__ inline double det_exp2(double th, double tl) {
  const double ln2HI = 6.93147180369123816490e-01, ln2LO = 1.90821492927058770002e-10,
               invln2 = 1.44269504088896338700e+00;
  const double P1 = 1.66666666666666019037e-01, P2 = -2.77777777770155933842e-03,
               P3 = 6.61375632143793436117e-05, P4 = -1.65339022054652515390e-06,
               P5 = 4.13813679705723846039e-08;
  if (th != th) return th;
  if (th > 7.09782712893383973096e+02) return __builtin_inf();
  if (th < -7.45133219101941108420e+02) return 0.0;
  const double kd = floor(invln2 * th + 0.5);
  const double hi = th - kd * ln2HI;
  const double lo = kd * ln2LO - tl;
  const double r = hi - lo;
  const double q = r * r;
  const double c = r - q * (P1 + q * (P2 + q * (P3 + q * (P4 + q * P5))));
  const double y = 1.0 - ((lo - (r * c) / (2.0 - c)) - hi);
  return ldexp(y, (int)kd);
}

template <bool FMA = false>
__host__ __device__ inline double det_pow(double x, double y) {
  if (x != x || y != y) return x + y;  // NaN
  if (y == 0.0 || x == 1.0) return 1.0;
  if (x < 0.0) return __builtin_nan("");  // not reached by the variation operators
  if (x == 0.0) return y > 0.0 ? 0.0 : __builtin_inf();
  if (x == __builtin_inf()) return y > 0.0 ? __builtin_inf() : 0.0;
  if (y == floor(y) && fabs(y) <= 64.0) {  // binary powering, low bit first
    const int n0 = (int)fabs(y);
    int ex = 0;
    (void)frexp(x, &ex);
    int n = n0;
    if ((ex < 0 ? -ex : ex) * n0 > 900) {  // result near or past the double range
      double r = 1.0, b = x;
      while (n) {
        if (n & 1) r = r * b;
        n >>= 1;
        if (n) b = b * b;
      }
      return y < 0.0 ? 1.0 / r : r;
    }
    double rh = 1.0, rl = 0.0, bh = x, bl = 0.0;  // double-double
    if (FMA && x >= 1.0) {  // every product >= 1: no partial product underflows
      while (n) {
        if (n & 1) det_dd_mul<true>(rh, rl, bh, bl, rh, rl);
        n >>= 1;
        if (n) det_dd_mul<true>(bh, bl, bh, bl, bh, bl);
      }
    } else {
      while (n) {
        if (n & 1) det_dd_mul(rh, rl, bh, bl, rh, rl);
        n >>= 1;
        if (n) det_dd_mul(bh, bl, bh, bl, bh, bl);
      }
    }
    if (y > 0.0) return rh;
    const double q = 1.0 / rh;  // 1 / (rh + rl), one correction step
    double p, pe;
    det_two_prod_x<FMA>(q, rh, p, pe);
    const double rem = ((1.0 - p) - pe) - q * rl;
    return q + rem / rh;
  }
  double lh, ll, th, tl0;
  det_log2(x, lh, ll);
  det_two_prod_x<FMA>(y, lh, th, tl0);
  double tl = tl0 + y * ll;
  det_fast_two_sum(th, tl, th, tl);
  return det_exp2(th, tl);
}

}  // namespace mv
