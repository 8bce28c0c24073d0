// Fitness evaluation and variation kernels (gfx950).
//
// One generation's candidate rows go through two kernels:
//  k_vary (one wave per row, small LDS, high occupancy):
//     [mode 1] two-point crossover + polynomial mutation of the row's parents
//              (moeva2.py:90-111 -> softmax_crossover.py:17-38 / softmax_mutation.py:20-67
//              semantics, Philox draws), child written to the population pool;
//     decode genes -> ML row x_f in LDS (feature_encoder.py:91-124);
//     encoder MinMax distance f2 (default_problem.py:80-91, utils.py:11-22);
//     constraint program -> G, f3 (default_problem.py:93-97,128-129);
//     ML-scaled fp32 row (default_problem.py:119-121) -> scratch xml[row][Dm4].
//  k_mlp (32-row tiles): the Dense-ReLU chain on MFMA (v_mfma_f32_16x16x4_f32, exact fp32
//     products), layer 1 over the mutable columns only (immutable columns folded into a
//     per-state bias), final Dense + softmax on the VALU with its weights in LDS
//     (classifier.py:23-29) -> f1.
// k_predict: Classifier.predict_proba on ML rows.   k_setup_states: per-state constants.
//
// Launch arguments live in constant memory: a ring of RowsArgs slots per device (c_rows),
// written stream-ordered from pinned host copies.  As by-value kernel arguments the
// several-hundred-byte structs spilled SGPRs into VGPRs; from a plain global buffer the
// pointers they hold lose their address space (every access became a flat op); pointers
// loaded from the constant address space are known to be global.  Only the
// per-generation scalars (slot, gen, first history row) are passed by value.
#include <mutex>

#include "engine.h"
#include "kernels.h"
#include "philox.h"

namespace mv {

__constant__ RowsArgs c_rows[ARG_SLOTS];

namespace {
struct ArgRing {
  bool ready = false;
  RowsArgs* host = nullptr;  // pinned [ARG_SLOTS]
  hipEvent_t ev[ARG_SLOTS] = {};
  int next = 0;
};
constexpr int MAX_DEVICES = 64;
ArgRing g_rings[MAX_DEVICES];
std::mutex g_ring_mu;
}  // namespace

hipError_t stage_rows(const RowsArgs& a, hipStream_t stream, int* slot) {
  int dev = 0;
  hipError_t e = hipGetDevice(&dev);
  if (e != hipSuccess) return e;
  if (dev < 0 || dev >= MAX_DEVICES) return hipErrorInvalidDevice;
  std::lock_guard<std::mutex> lock(g_ring_mu);
  ArgRing& r = g_rings[dev];
  if (!r.ready) {
    e = hipHostMalloc((void**)&r.host, ARG_SLOTS * sizeof(RowsArgs));
    for (int i = 0; i < ARG_SLOTS && e == hipSuccess; ++i)
      e = hipEventCreateWithFlags(&r.ev[i], hipEventDisableTiming);
    if (e != hipSuccess) return e;
    r.ready = true;
  }
  const int k = r.next;
  r.next = (r.next + 1) % ARG_SLOTS;
  e = hipEventSynchronize(r.ev[k]);  // the slot's previous launches have finished
  if (e != hipSuccess) return e;
  r.host[k] = a;
  e = hipMemcpyToSymbolAsync(HIP_SYMBOL(c_rows), r.host + k, sizeof(RowsArgs),
                             (size_t)k * sizeof(RowsArgs), hipMemcpyHostToDevice, stream);
  if (e == hipSuccess) *slot = k;
  return e;
}

hipError_t release_rows(int slot, hipStream_t stream) {
  int dev = 0;
  hipError_t e = hipGetDevice(&dev);
  if (e != hipSuccess) return e;
  std::lock_guard<std::mutex> lock(g_ring_mu);
  return hipEventRecord(g_rings[dev].ev[slot], stream);
}

typedef float floatx4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

__device__ __forceinline__ double nanmax(double a, double b) {
  if (a != a) return a;
  if (b != b) return b;
  return b > a ? b : a;
}

__device__ __forceinline__ double wave_max(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = nanmax(v, __shfl_xor(v, o, 64));
  return v;
}

__device__ __forceinline__ void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

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

// One constraint column on the ML row x (LDS).  FULL adds the LCLD financial identities;
// ABS_SUMDIFF columns are evaluated wave-parallel (sumdiff_wave) by the caller.
template <bool FULL>
__device__ __forceinline__ double eval_op(const DProblem& p, int c, const double* __restrict__ x) {
  const int code = p.op_code[c];
  const int4 ar = *(const int4*)(p.op_arg + 4 * c);
  switch (code) {
    case 1:  // MV_OP_DIFF (botnet_constraints.py:283-285)
      return x[ar.x] - x[ar.y];
    case 2: {  // MV_OP_RATIO_SAFE (botnet_constraints.py:304-306)
      const double a = x[ar.x], b = x[ar.y];
      return (b != 0.0 ? a / b : 0.0) - p.op_k[2 * c];
    }
    case 9: {  // MV_OP_XOR_AUG (examples/utils.py:7-29)
      const double2 k = *(const double2*)(p.op_k + 2 * c);
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
        return fabs(x3 - num / den) - p.op_k[2 * c];
      }
      case 5: {  // MV_OP_LCLD_TERM (:186)
        const double t = x[ar.x];
        return fabs((36.0 - t) * (60.0 - t));
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

// |sum(pool[a0:a1]) - sum(pool[a1:a2])| with all 64 lanes (exact for the integer-valued
// features of every shipped program; summation order differs from numpy otherwise).
__device__ __forceinline__ double sumdiff_wave(const DProblem& p, int c, const double* x,
                                               int lane) {
  const int4 ar = *(const int4*)(p.op_arg + 4 * c);
  double s0 = 0.0, s1 = 0.0;
  for (int q = ar.x + lane; q < ar.y; q += 64) s0 += x[p.idx_pool[q]];
  for (int q = ar.y + lane; q < ar.z; q += 64) s1 += x[p.idx_pool[q]];
  s0 = wave_sum(s0);
  s1 = wave_sum(s1);
  return fabs(s0 - s1);
}

// Constraint row -> G columns (+ history columns); returns the wave-uniform f3 = sum(G).
// Values <= tol -> 0 (Constraints.evaluate); with clamp, G * (G > 0) (default_problem.py:93-97).
template <bool FULL>
__device__ __forceinline__ double constraints_row(const DProblem& p, const double* xrow,
                                                  int lane, double* grow, double* hcols,
                                                  bool clamp_positive) {
  double acc3 = 0.0;
  for (int c = lane; c < p.C; c += 64) {
    if (p.op_code[c] == 3) continue;
    double v = eval_op<FULL>(p, c, xrow);
    if (v <= p.tol) v = 0.0;
    const double g = clamp_positive ? v * (v > 0.0 ? 1.0 : 0.0) : v;
    if (grow) grow[c] = g;
    if (hcols) hcols[c] = g;
    acc3 += g;
  }
  for (int k = 0; k < p.n_sumdiff; ++k) {
    const int c = p.sumdiff_ops[k];
    double v = sumdiff_wave(p, c, xrow, lane);
    if (v <= p.tol) v = 0.0;
    const double g = clamp_positive ? v * (v > 0.0 ? 1.0 : 0.0) : v;
    if (lane == 0) {
      if (grow) grow[c] = g;
      if (hcols) hcols[c] = g;
      acc3 += g;
    }
  }
  return wave_sum(acc3);
}

// pymoo PolynomialMutation for one gene (softmax_mutation.py:77-103), no FMA contraction.
__device__ __forceinline__ double poly_mut(double x, double xl, double xu, double u, double eta) {
  const double d1 = (x - xl) / (xu - xl);
  const double d2 = (xu - x) / (xu - xl);
  const double mp = 1.0 / (eta + 1.0);
  double dq;
  if (u <= 0.5) {
    const double xy = 1.0 - d1;
    const double val = 2.0 * u + (1.0 - 2.0 * u) * pow(xy, eta + 1.0);
    dq = pow(val, mp) - 1.0;
  } else {
    const double xy = 1.0 - d2;
    const double val = 2.0 * (1.0 - u) + 2.0 * (u - 0.5) * pow(xy, eta + 1.0);
    dq = 1.0 - pow(val, mp);
  }
  double y = x + dq * (xu - xl);
  if (y < xl) y = xl;
  if (y > xu) y = xu;
  return y;
}

struct Cx {
  int on[2];
  int lo[2];
  int hi[2];
};

// Crossover draws of mating m for both variable-type subsets (oracle crossover_draws).
__device__ __forceinline__ Cx cx_draws(const Rng& rng, int gen, int m, const int n_sub[2],
                                       double prob) {
  Cx c;
#pragma unroll
  for (int s = 0; s < 2; ++s) {
    const int n = n_sub[s];
    c.on[s] = 0;
    c.lo[s] = 0;
    c.hi[s] = 0;
    if (n <= 0) continue;
    const u32x4 w = rng.draw((uint32_t)(m * 2 + s), (uint32_t)gen, TAG_CX);
    c.on[s] = u53(w.x, w.y) < prob;
    if (n - 1 <= 0) continue;
    const int a = 1 + (int)(((uint64_t)w.z * (uint64_t)(n - 1)) >> 32);
    if (n - 1 == 1) {
      c.lo[s] = a;
      c.hi[s] = n;
    } else {
      int b = 1 + (int)(((uint64_t)w.w * (uint64_t)(n - 2)) >> 32);
      if (b >= a) ++b;
      c.lo[s] = a < b ? a : b;
      c.hi[s] = a < b ? b : a;
    }
  }
  return c;
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

// Generate (mode 1) or load (mode 0) the genes of row (b, i); lane-parallel, 4 genes/lane.
// gene_info packs kind (2 bits) | subset index << 2 | feature (or OHE group) << 17.
__device__ __forceinline__ void row_genes(const RowsArgs& a, int gen, int b, int i, int lane,
                                          double* xrow) {
  const DProblem& p = a.p;
  const int V = p.V;
  double* gout = nullptr;
  if (a.genes_out) {
    const int orow = a.out_map ? a.out_map[(size_t)b * a.n + i] : i;
    gout = a.genes_out + ((size_t)b * a.out_rows + orow) * V;
  }
  if (a.mode == 0) {
    const double* gin = a.genes_in + ((size_t)b * a.in_rows + i) * V;
    for (int g = lane; g < V; g += 64) {
      const double x = gin[g];
      if (gout) gout[g] = x;
      if (xrow) scatter_gene(p, xrow, p.gene_info[g], x);
    }
    return;
  }
  const Rng rng(a.seed, a.stream_key);
  const int nm = a.n / 2;
  const int m = i % nm;
  const int side = i / nm;
  const int* par = a.parents + ((size_t)b * nm + m) * 2;
  const int own = side ? par[1] : par[0];
  const int oth = side ? par[0] : par[1];
  const double* gown = a.genes_in + ((size_t)b * a.in_rows + own) * V;
  const double* goth = a.genes_in + ((size_t)b * a.in_rows + oth) * V;
  const Cx cx = cx_draws(rng, gen, m, p.n_sub, a.cx_prob);
  const int nq = (V + 3) >> 2;
  const double* gl = a.s.gl + (size_t)b * V;
  const double* gu = a.s.gu + (size_t)b * V;
  for (int g0 = lane * 4; g0 < V; g0 += 256) {
    const int4 inf4 = *(const int4*)(p.gene_info + g0);  // padded to a multiple of 4
    const u32x4 w = rng.draw((uint32_t)(i * nq + (g0 >> 2)), (uint32_t)gen, TAG_MUT_MASK);
    const int infs[4] = {inf4.x, inf4.y, inf4.z, inf4.w};
    const uint32_t words[4] = {w.x, w.y, w.z, w.w};
    double xv[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int info = infs[j];
      const int ss = (info & 3) == 0 ? 0 : 1;
      const int sub = (info >> 2) & 0x7FFF;
      const bool swap = cx.on[ss] && sub >= cx.lo[ss] && sub < cx.hi[ss];
      xv[j] = (g0 + j < V) ? (swap ? goth : gown)[g0 + j] : 0.0;
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int g = g0 + j;
      if (g < V) {
        double x = xv[j];
        if (words[j] < a.mut_thr) {  // prob 1/V: one lane per row on average
          const bool is_real = (infs[j] & 3) == 0;
          const u32x4 wu = rng.draw((uint32_t)(i * V + g), (uint32_t)gen, TAG_MUT_U);
          const double xl = gl[g], xu = gu[g];
          const double y = poly_mut(x, is_real ? xl : xl - INT_WIDEN,
                                    is_real ? xu : xu + INT_WIDEN, u53(wu.x, wu.y), a.eta);
          if (is_real) {
            x = y;
          } else {  // IntegerFromFloatMutation: np.round (half to even), then clamp
            double yi = rint(y);
            if (yi < xl) yi = xl;
            if (yi > xu) yi = xu;
            x = yi;
          }
        }
        if (gout) gout[g] = x;
        if (xrow) scatter_gene(p, xrow, infs[j], x);
      }
    }
  }
}

// Variation (mode 1) / gene load (mode 0) + decode + f2 + constraints/f3 + fp32 ML row.
// One wave per row, 4 rows per workgroup; LDS = 4 ML rows (fp64).
template <bool FULL>
__global__ __launch_bounds__(256) void k_vary(int slot, int gen,
                                              int hist_row0) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const RowsArgs& a = c_rows[slot];
  const DProblem& p = a.p;
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int r = blockIdx.x * 4 + wave;
  if (r >= a.total) return;
  const int b = r / a.n;
  const int i = r - b * a.n;
  if (!a.do_eval) {
    row_genes(a, gen, b, i, lane, nullptr);
    return;
  }
  const int D = p.D;
  double* xrow = (double*)smem + (size_t)wave * D;
  const double* xi = a.s.x_init + (size_t)b * D;
  for (int f = lane; f < D; f += 64) xrow[f] = xi[f];
  wave_sync();
  row_genes(a, gen, b, i, lane, xrow);
  wave_sync();
  // fp32 ML row (scratch) + encoder MinMax distance over the mutable features
  const int Dm = p.Dm, Dm4 = p.Dm4;
  const double* es = a.s.enc_scale + (size_t)b * Dm;
  const double* em = a.s.enc_min + (size_t)b * Dm;
  const double* x0 = a.s.x0_mm + (size_t)b * Dm;
  float* xo = a.xml + (size_t)r * Dm4;
  const bool l2 = p.norm == 2;
  double acc = 0.0;
  for (int j = lane; j < Dm4; j += 64) {
    float v = 0.f;
    if (j < Dm) {
      const double xf = xrow[p.mut_feat[j]];
      v = (float)(xf * p.mlS[j] + p.mlM[j]);
      const double d = (xf * es[j] + em[j]) - x0[j];
      acc = l2 ? acc + d * d : nanmax(acc, fabs(d));
    }
    xo[j] = v;
  }
  acc = l2 ? wave_sum(acc) : wave_max(acc);
  double f2 = l2 ? sqrt(acc) : acc;
  if (p.scale_obj) f2 = f2 * p.f2_scale + 0.0;
  double* grow = a.G ? a.G + ((size_t)b * a.n + i) * p.C : nullptr;
  double* hrow = a.hist ? a.hist + ((size_t)b * a.hist_rows + hist_row0 + i) * a.hist_w : nullptr;
  const double f3 = constraints_row<FULL>(p, xrow, lane, grow,
                                          (hrow && a.hist_w > 3) ? hrow + 3 : nullptr, true);
  if (lane == 0) {
    if (a.F) {
      const int orow = a.out_map ? a.out_map[(size_t)b * a.n + i] : i;
      double* fr = a.F + ((size_t)b * a.out_rows + orow) * 3;
      fr[1] = f2;
      fr[2] = f3;
    }
    if (hrow) {
      hrow[1] = f2;
      hrow[2] = f3;
    }
  }
}

// ---------------------------------------------------------------------------------------
// Dense layer on MFMA: out[32][N] = relu(in[32][K] . W[K][N] + bias), K % 4 == 0, N % 16 == 0.
// Software-pipelined: U k-steps of A (LDS) and B (global/L2) fragments are loaded before
// their 2*U MFMAs so the B-load latency is paid once per U steps.
template <int MAXCT>
__device__ __forceinline__ void dense_mfma(const float* __restrict__ in, int ldi, int K,
                           const float* __restrict__ W, int N, const float* __restrict__ bias,
                           const float* __restrict__ bias_state, const int* row_state,
                           float* __restrict__ out, int ldo, int wave, int lane) {
  constexpr int U = MAXCT >= 4 ? 4 : 8;
  const int nct = N >> 4;
  floatx4 acc[2][MAXCT];
#pragma unroll
  for (int c = 0; c < MAXCT; ++c) {
    acc[0][c] = floatx4{0.f, 0.f, 0.f, 0.f};
    acc[1][c] = floatx4{0.f, 0.f, 0.f, 0.f};
  }
  const int ka = lane >> 4;
  const int il = lane & 15;
  const float* in0 = in + il * ldi + ka;
  const float* in1 = in + (il + 16) * ldi + ka;
  const float* wb = W + (size_t)ka * N + il;
  for (int k0 = 0; k0 < K; k0 += 4 * U) {
    float a0[U], a1[U], bf[U][MAXCT];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int kk = k0 + 4 * u;
      const bool ok = kk < K;
      a0[u] = ok ? in0[kk] : 0.f;
      a1[u] = ok ? in1[kk] : 0.f;
#pragma unroll
      for (int c = 0; c < MAXCT; ++c) {
        const int ct = wave + c * 4;
        bf[u][c] = (ok && ct < nct) ? wb[(size_t)kk * N + ct * 16] : 0.f;
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
#pragma unroll
      for (int c = 0; c < MAXCT; ++c) {
        if (wave + c * 4 < nct) {
          acc[0][c] = __builtin_amdgcn_mfma_f32_16x16x4f32(a0[u], bf[u][c], acc[0][c], 0, 0, 0);
          acc[1][c] = __builtin_amdgcn_mfma_f32_16x16x4f32(a1[u], bf[u][c], acc[1][c], 0, 0, 0);
        }
      }
    }
  }
#pragma unroll
  for (int c = 0; c < MAXCT; ++c) {
    const int ct = wave + c * 4;
    if (ct < nct) {
      const int col = ct * 16 + il;
#pragma unroll
      for (int rt = 0; rt < 2; ++rt) {
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int row = rt * 16 + ka * 4 + j;
          float bv;
          if (bias_state) {
            const int st = row_state[row] < 0 ? 0 : row_state[row];
            bv = bias_state[(size_t)st * N + col];
          } else {
            bv = bias[col];
          }
          const float v = acc[rt][c][j] + bv;
          out[row * ldo + col] = v > 0.f ? v : 0.f;
        }
      }
    }
  }
}

// Final Dense + softmax for row t (one thread), weights staged in LDS: ws[k*nout + c], wsb[c].
__device__ __forceinline__ void last_layer_softmax(const float* in, int ldi, int K, int nout,
                                                   const float* ws, const float* wsb, int t,
                                                   float* prob) {
  float mx = -__builtin_inff();
  for (int c = 0; c < nout; ++c) {
    float s = 0.f;
#pragma unroll 8
    for (int k = 0; k < K; ++k) s = fmaf(in[t * ldi + k], ws[k * nout + c], s);
    prob[c] = s + wsb[c];
    mx = prob[c] > mx ? prob[c] : mx;
  }
  float den = 0.f;
  for (int c = 0; c < nout; ++c) {
    prob[c] = expf(prob[c] - mx);
    den += prob[c];
  }
  for (int c = 0; c < nout; ++c) prob[c] = prob[c] / den;
}

__host__ __device__ inline int max_hidden(const int* dims, int n_layers) {
  int h = 16;
  for (int l = 1; l < n_layers; ++l) h = dims[l] > h ? dims[l] : h;
  return h;
}

// Dense chain over 32-row tiles of the fp32 ML rows -> f1.
template <int MAXCT>
__global__ __launch_bounds__(EVAL_T) void k_mlp(int slot, int hist_row0) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const RowsArgs& a = c_rows[slot];
  const DProblem& p = a.p;
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int Dm4 = p.Dm4;
  const int lda = Dm4 + 1;
  const int nl = p.n_layers;
  const int hmax = max_hidden(p.dims, nl);
  const int Klast = p.dims[nl - 1];
  const int nout = p.dims[nl];
  int* row_state = (int*)smem;  // [32]
  float* ws = (float*)(smem + 128);
  float* wsb = ws + Klast * nout;
  const size_t head = mlp_head_bytes(Klast, nout);
  float* R1 = (float*)(smem + head);
  float* R2 = (float*)(smem + head + eval_region1_bytes(Dm4, hmax));
  const int r0 = blockIdx.x * EVAL_TR;
  if (tid < EVAL_TR) row_state[tid] = (r0 + tid < a.total) ? (r0 + tid) / a.n : -1;
  for (int q = tid; q < Klast * nout; q += EVAL_T) ws[q] = p.W[nl - 1][q];
  if (tid < nout) wsb[tid] = p.bias[nl - 1][tid];
  const int nq = Dm4 >> 2;
  for (int idx = tid; idx < EVAL_TR * nq; idx += EVAL_T) {
    const int t = idx / nq, q = idx - t * nq;
    const int r = r0 + t;
    float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
    if (r < a.total) v = *(const float4*)(a.xml + (size_t)r * Dm4 + 4 * q);
    float* d = R1 + t * lda + 4 * q;
    d[0] = v.x;
    d[1] = v.y;
    d[2] = v.z;
    d[3] = v.w;
  }
  __syncthreads();
  const float* in = R1;
  int ldi = lda;
  int K = Dm4;
  float* outb = R2;
  float* other = R1;
  for (int l = 0; l + 1 < nl; ++l) {
    const int N = p.dims[l + 1];
    dense_mfma<MAXCT>(in, ldi, K, p.W[l], N, p.bias[l], l == 0 ? a.s.bias1 : nullptr, row_state,
                      outb, N + 1, wave, lane);
    __syncthreads();
    in = outb;
    ldi = N + 1;
    K = N;
    float* tmp = outb;
    outb = other;
    other = tmp;
  }
  if (tid < EVAL_TR) {
    const int st = row_state[tid];
    if (st >= 0) {
      float prob[8];
      last_layer_softmax(in, ldi, K, nout, ws, wsb, tid, prob);
      const double f1 = (double)prob[a.s.min_class[st]];
      const int i = (r0 + tid) - st * a.n;
      if (a.F) {
        const int orow = a.out_map ? a.out_map[(size_t)st * a.n + i] : i;
        a.F[((size_t)st * a.out_rows + orow) * 3] = f1;
      }
      if (a.hist) a.hist[((size_t)st * a.hist_rows + hist_row0 + i) * a.hist_w] = f1;
    }
  }
}

// Classifier.predict_proba: 32 rows per workgroup, full-width first layer.
template <int MAXCT>
__global__ __launch_bounds__(EVAL_T) void k_predict(MlpArgs a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int nl = a.n_layers;
  const int hmax = max_hidden(a.dims, nl);
  const int Klast = a.dims[nl - 1];
  const int nout = a.dims[nl];
  const int lda = a.D4 + 1;
  float* ws = (float*)(smem + 128);
  float* wsb = ws + Klast * nout;
  const size_t head = mlp_head_bytes(Klast, nout);
  float* R1 = (float*)(smem + head);
  float* R2 = (float*)(smem + head + eval_region1_bytes(a.D4, hmax));
  const int D = a.dims[0];
  const int r0 = blockIdx.x * EVAL_TR;
  for (int q = tid; q < Klast * nout; q += EVAL_T) ws[q] = a.W[nl - 1][q];
  if (tid < nout) wsb[tid] = a.bias[nl - 1][tid];
  for (int idx = tid; idx < EVAL_TR * a.D4; idx += EVAL_T) {
    const int t = idx / a.D4, j = idx - t * a.D4;
    const int r = r0 + t;
    R1[t * lda + j] = (r < a.n && j < D) ? (float)a.x[(size_t)r * D + j] : 0.f;
  }
  __syncthreads();
  const float* in = R1;
  int ldi = lda, K = a.D4;
  float* outb = R2;
  float* other = R1;
  for (int l = 0; l + 1 < nl; ++l) {
    const int N = a.dims[l + 1];
    dense_mfma<MAXCT>(in, ldi, K, a.W[l], N, a.bias[l], nullptr, nullptr, outb, N + 1, wave,
                      lane);
    __syncthreads();
    in = outb;
    ldi = N + 1;
    K = N;
    float* tmp = outb;
    outb = other;
    other = tmp;
  }
  if (tid < EVAL_TR && r0 + tid < a.n) {
    float prob[8];
    last_layer_softmax(in, ldi, K, nout, ws, wsb, tid, prob);
    for (int c = 0; c < nout; ++c) a.proba[(size_t)(r0 + tid) * nout + c] = (double)prob[c];
  }
}

// Constraints only (Constraints.evaluate numpy path): one wave per ML-space row.
template <bool FULL>
__global__ __launch_bounds__(256) void k_constraints(int slot, int n,
                                                     const double* x, double* G) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const DProblem& p = c_rows[slot].p;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int r = blockIdx.x * 4 + wave;
  if (r >= n) return;
  double* xrow = (double*)smem + (size_t)wave * p.D;
  for (int f = lane; f < p.D; f += 64) xrow[f] = x[(size_t)r * p.D + f];
  wave_sync();
  constraints_row<FULL>(p, xrow, lane, G + (size_t)r * p.C, nullptr, false);
}

// Per-state constants: one workgroup per state.
__global__ __launch_bounds__(256) void k_setup_states(int slot,
                                                      const double* x_init, const double* xl,
                                                      const double* xu, const float* W1full,
                                                      const float* b1, double* gl, double* gu,
                                                      double* enc_scale, double* enc_min,
                                                      double* x0_mm, float* bias1,
                                                      double* genes0) {
  const DProblem& p = c_rows[slot].p;
  const int b = blockIdx.x;
  const int tid = threadIdx.x;
  const double* xi = x_init + (size_t)b * p.D;
  const double* lo = xl + (size_t)b * p.D;
  const double* hi = xu + (size_t)b * p.D;
  for (int g = tid; g < p.V; g += blockDim.x) {
    const int kind = p.gene_kind[g];
    double l, u, x0;
    if (kind != 2) {
      const int f = p.gene_feat[g];
      l = lo[f];
      u = hi[f];
      x0 = xi[f];
      if (kind != 0) x0 = rint(x0);  // sampling.py:74-76
    } else {
      const int q = p.gene_feat[g];
      const int o0 = p.ohe_off[q], o1 = p.ohe_off[q + 1];
      l = 0.0;
      u = (double)(o1 - o0 - 1);
      int best = 0;
      double bv = xi[p.ohe_feat[o0]];
      for (int k = o0 + 1; k < o1; ++k) {  // OneHotEncoder.inverse_transform = argmax
        const double v = xi[p.ohe_feat[k]];
        if (v > bv) {
          bv = v;
          best = k - o0;
        }
      }
      x0 = (double)best;
    }
    gl[(size_t)b * p.V + g] = l;
    gu[(size_t)b * p.V + g] = u;
    genes0[(size_t)b * p.V + g] = x0;
  }
  for (int j = tid; j < p.Dm; j += blockDim.x) {
    const int f = p.mut_feat[j];
    const double a0 = lo[f], a1 = hi[f];
    const double mn = a0 < a1 ? a0 : a1;
    const double mx = a0 < a1 ? a1 : a0;
    double rng = mx - mn;
    if (rng == 0.0) rng = 1.0;
    const double sc = 1.0 / rng;
    const double mi = 0.0 - mn * sc;
    enc_scale[(size_t)b * p.Dm + j] = sc;
    enc_min[(size_t)b * p.Dm + j] = mi;
    x0_mm[(size_t)b * p.Dm + j] = xi[f] * sc + mi;
  }
  // layer-1 bias fold over the immutable features (fp32, Keras casts inputs to float32)
  const int H1 = p.dims[1];
  for (int h = tid; h < H1; h += blockDim.x) {
    float s = 0.f;
    int jm = 0;
    for (int f = 0; f < p.D; ++f) {
      if (jm < p.Dm && p.mut_feat[jm] == f) {
        ++jm;
        continue;
      }
      const float xv = (float)(xi[f] * p.ml_scale[f] + p.ml_min[f]);
      s = fmaf(xv, W1full[(size_t)f * H1 + h], s);
    }
    bias1[(size_t)b * H1 + h] = b1[h] + s;
  }
}

// ---------------------------------------------------------------------------------------
// Allow up to the full 160 KiB of LDS per workgroup for the dynamic-LDS kernels.
static void configure_lds_once() {
  static bool done = false;
  if (done) return;
  const int lim = 160 * 1024;
  const void* fns[] = {(const void*)k_mlp<1>,          (const void*)k_mlp<2>,
                       (const void*)k_mlp<4>,          (const void*)k_mlp<8>,
                       (const void*)k_vary<false>,     (const void*)k_vary<true>,
                       (const void*)k_predict<1>,      (const void*)k_predict<2>,
                       (const void*)k_predict<4>,      (const void*)k_predict<8>,
                       (const void*)k_constraints<false>, (const void*)k_constraints<true>};
  for (const void* f : fns)
    (void)hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, lim);
  (void)hipGetLastError();
  done = true;
}

hipError_t launch_vary(const RowsArgs& a, int slot, int gen, int hist_row0,
                       hipStream_t stream) {
  if (a.total <= 0) return hipSuccess;
  configure_lds_once();
  const size_t lds = a.do_eval ? (size_t)4 * a.p.D * sizeof(double) : 0;
  const dim3 grid((a.total + 3) / 4);
  if (a.p.full_ops)
    hipLaunchKernelGGL(k_vary<true>, grid, dim3(256), lds, stream, slot, gen, hist_row0);
  else
    hipLaunchKernelGGL(k_vary<false>, grid, dim3(256), lds, stream, slot, gen, hist_row0);
  return hipGetLastError();
}

hipError_t launch_mlp(const RowsArgs& a, int slot, int hist_row0, hipStream_t stream) {
  if (a.total <= 0) return hipSuccess;
  configure_lds_once();
  const int nl = a.p.n_layers;
  const int hmax = max_hidden(a.p.dims, nl);
  const size_t lds = mlp_lds_bytes(a.p.Dm4, hmax, a.p.dims[nl - 1], a.p.dims[nl]);
  const dim3 grid((a.total + EVAL_TR - 1) / EVAL_TR);
  const int nct = hmax / 16;
  if (nct <= 4)
    hipLaunchKernelGGL(k_mlp<1>, grid, dim3(EVAL_T), lds, stream, slot, hist_row0);
  else if (nct <= 8)
    hipLaunchKernelGGL(k_mlp<2>, grid, dim3(EVAL_T), lds, stream, slot, hist_row0);
  else if (nct <= 16)
    hipLaunchKernelGGL(k_mlp<4>, grid, dim3(EVAL_T), lds, stream, slot, hist_row0);
  else
    hipLaunchKernelGGL(k_mlp<8>, grid, dim3(EVAL_T), lds, stream, slot, hist_row0);
  return hipGetLastError();
}

hipError_t launch_rows(const RowsArgs& a, int slot, int gen, int hist_row0,
                       hipStream_t stream) {
  hipError_t e = launch_vary(a, slot, gen, hist_row0, stream);
  if (e != hipSuccess || !a.do_eval) return e;
  return launch_mlp(a, slot, hist_row0, stream);
}

hipError_t launch_predict(const MlpArgs& a, hipStream_t stream) {
  if (a.n <= 0) return hipSuccess;
  configure_lds_once();
  const int nl = a.n_layers;
  const int hmax = max_hidden(a.dims, nl);
  const size_t lds = mlp_lds_bytes(a.D4, hmax, a.dims[nl - 1], a.dims[nl]);
  const dim3 grid((a.n + EVAL_TR - 1) / EVAL_TR);
  const int nct = hmax / 16;
  if (nct <= 4)
    hipLaunchKernelGGL(k_predict<1>, grid, dim3(EVAL_T), lds, stream, a);
  else if (nct <= 8)
    hipLaunchKernelGGL(k_predict<2>, grid, dim3(EVAL_T), lds, stream, a);
  else if (nct <= 16)
    hipLaunchKernelGGL(k_predict<4>, grid, dim3(EVAL_T), lds, stream, a);
  else
    hipLaunchKernelGGL(k_predict<8>, grid, dim3(EVAL_T), lds, stream, a);
  return hipGetLastError();
}

hipError_t launch_constraints(const DProblem& hp, int slot, int n, const double* x,
                              double* G, hipStream_t stream) {
  if (n <= 0) return hipSuccess;
  configure_lds_once();
  const size_t lds = (size_t)4 * hp.D * sizeof(double);
  const dim3 grid((n + 3) / 4);
  if (hp.full_ops)
    hipLaunchKernelGGL(k_constraints<true>, grid, dim3(256), lds, stream, slot, n, x, G);
  else
    hipLaunchKernelGGL(k_constraints<false>, grid, dim3(256), lds, stream, slot, n, x, G);
  return hipGetLastError();
}

hipError_t launch_setup_states(int slot, int B, const double* x_init, const double* xl,
                               const double* xu, const float* W1full, const float* b1, double* gl,
                               double* gu, double* enc_scale, double* enc_min, double* x0_mm,
                               float* bias1, double* genes0, hipStream_t stream) {
  if (B <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_setup_states, dim3(B), dim3(256), 0, stream, slot, x_init, xl, xu, W1full,
                     b1, gl, gu, enc_scale, enc_min, x0_mm, bias1, genes0);
  return hipGetLastError();
}

}  // namespace mv
