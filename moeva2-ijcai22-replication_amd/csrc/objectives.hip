// Success scoring of final attack populations: ObjectiveCalculator._calculate_objective
// (src/attacks/moeva2/objective_calculator.py:44-84) batched over B states x n candidates.
//
//   k_obj_mlscale : x_ml = ml_scaler.transform(x)           (objective_calculator.py:61-63)
//   [k_constraints]: G = constraints.evaluate(x)             (:47-51, engine's program)
//   [k_predict]    : proba = classifier.predict_proba(x_ml)  (:64)
//   k_objectives  : CV = sum (G | ohe)*(>0)                  (:47-57, utils.py:43-54)
//                   f1 = proba[:, minimize_class]
//                   f2 = ||mm(x_init) - mm(x)||_{2|inf}      (:70-82)
//                   range flag for the [0-1e-4, 1+1e-4] scaling asserts (:72-76)
//
// All of it is HBM-bound streaming over the D-wide ML rows: one wave per row, lanes over
// features (coalesced fp64), wave reductions through DPP.
#include <hip/hip_runtime.h>

#include "engine.h"
#include "kernels.h"
#include "wave.h"

namespace mv {

// sklearn MinMaxScaler.transform: X *= scale_; X += min_ (two roundings, no FMA)
__global__ __launch_bounds__(256) void k_obj_mlscale(long total, int D, const double* __restrict__ x,
                                                     const double* __restrict__ s,
                                                     const double* __restrict__ m,
                                                     double* __restrict__ out) {
  const long stride = (long)gridDim.x * blockDim.x;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += stride) {
    const int j = (int)(i % D);
    double v = x[i] * s[j];
    out[i] = v + m[j];
  }
}

__global__ __launch_bounds__(256) void k_objectives(ObjArgs a) {
  const int lane = threadIdx.x & 63;
  const long row = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= a.total) return;
  const int st = (int)(row / a.n);
  const double* __restrict__ xr = a.x + row * a.D;
  const double* __restrict__ xi = a.x_init + (long)st * a.D;
  // distance on the min_max_scaler space
  double acc = 0.0;
  int bad = 0;
  for (int j = lane; j < a.D; j += 64) {
    double vs = xr[j] * a.mm_scale[j];
    vs = vs + a.mm_min[j];
    double v0 = xi[j] * a.mm_scale[j];
    v0 = v0 + a.mm_min[j];
    // written as "not inside" so a NaN fails the range like the reference's np.all asserts
    bad |= !((vs >= -1e-4) & (vs <= 1.0 + 1e-4) & (v0 >= -1e-4) & (v0 <= 1.0 + 1e-4));
    const double d = v0 - vs;
    if (a.norm == 2)
      acc = acc + d * d;
    else
      acc = nanmax(acc, fabs(d));
  }
  const double f2 = a.norm == 2 ? sqrt(wave_sum(acc)) : wave_max(acc);
  // one-hot groups of the full type mask: sum_g |1 - sum(x[group g])|
  double oh = 0.0;
  for (int g = lane; g < a.n_ohe; g += 64) {
    double s = 0.0;
    for (int k = a.ohe_off[g]; k < a.ohe_off[g + 1]; ++k) s = s + xr[a.ohe_feat[k]];
    oh = oh + fabs(1.0 - s);
  }
  oh = wave_sum(oh);
  // Problem.calc_constraint_violation over [G | ohe]: sum(G * (G > 0)); a NaN column keeps
  // the sum NaN (NaN * False = NaN), so such a row never counts as constraint-respecting
  double cv = 0.0;
  const double* __restrict__ gr = a.G + row * a.C;
  for (int c = lane; c < a.C; c += 64) {
    const double v = gr[c];
    cv = cv + (v > 0.0 || v != v ? v : 0.0);
  }
  cv = wave_sum(cv) + (oh > 0.0 || oh != oh ? oh : 0.0);
  const unsigned long long anybad = __ballot(bad);
  if (lane == 0) {
    a.obj[row * 3 + 0] = cv;
    // Classifier.predict_proba: a 1-column model means [1 - p, p] (classifier.py:27-28)
    const double p = a.proba[row * a.n_out + (a.n_out == 1 ? 0 : a.cls)];
    a.obj[row * 3 + 1] = a.n_out == 1 && a.cls == 0 ? 1.0 - p : p;
    a.obj[row * 3 + 2] = f2;
    a.range_bad[row] = anybad != 0ull;
  }
}

hipError_t launch_obj_mlscale(long total, int D, const double* x, const double* s,
                              const double* m, double* out, hipStream_t stream) {
  if (total <= 0) return hipSuccess;
  long blocks = (total + 255) / 256;
  if (blocks > 8192) blocks = 8192;
  hipLaunchKernelGGL(k_obj_mlscale, dim3((unsigned)blocks), dim3(256), 0, stream, total, D, x, s,
                     m, out);
  return hipGetLastError();
}

hipError_t launch_objectives(const ObjArgs& a, hipStream_t stream) {
  if (a.total <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_objectives, dim3((unsigned)((a.total + 3) / 4)), dim3(256), 0, stream, a);
  return hipGetLastError();
}

}  // namespace mv
