// k_narrow: the row kernel for narrow problems (LCLD: V = 15 / 25 genes, D = 47 / 57
// features, C = 10 / 20 constraint ops) -- one LANE per candidate row instead of one wave.
//
// The wave-per-row kernels (k_gen, k_cons) were shaped for botnet's 432 genes / 360 ops;
// on LCLD rows 60-85 % of their lanes idle and every row pays two wave barriers and a
// wave reduction.  Here a lane runs its row's whole chain:
//   crossover + mutation (the same Philox draws, no per-row mutation cap) -> child genes
//   (registers, NV per lane) -> pool; decode into the wave's LDS row block [Dm][64] (one
//   8-byte column per lane: conflict-free); fp32 ML row -> xml for k_mlp2; f2; the
//   constraint program (uniform op stream, operands from the lane's LDS column or, for
//   immutable features, the state's x_init) -> G / history columns, f3.
// k_gen + k_cons in one launch, all lanes busy.
//
// Results are bit-identical to k_gen + k_cons: the wave reductions of those kernels (lane j
// holds term j, then the DPP/permlane butterfly = a balanced pairwise tree over the 64 lanes
// in lane order, wave.h) are restated per lane as the same tree over the same leaves
// (tree_sum: leaves in order, zero leaves up to 64).
#pragma once
#include "rowops.h"

namespace mv {

constexpr int NARROW_T = 128;    // threads per k_narrow workgroup (2 waves, 128 rows)
constexpr int NARROW_MAXV = 32;  // genes per row held in registers
constexpr int NARROW_MAXF = 64;  // mutable features (Dm4) and constraint ops

// LDS: regions A (op program), B (gene tables), C (ML scaler), the feature -> mutable-slot
// map, then per wave the mutable features of its 64 rows as [Dm][64] doubles.
struct NarrowLds {
  unsigned a_at, b_at, c_at, m_at, rows_at, total;
};
__host__ __device__ inline NarrowLds narrow_lds(const VaryOff& o, const DProblem& p) {
  NarrowLds l{};
  unsigned at = 0;
  l.a_at = at;
  at += o.a_end;
  l.b_at = at;
  at += o.b_end - o.b_at;
  l.c_at = at;
  at += o.c_end - o.c_at;
  l.m_at = at;
  at += ((unsigned)p.D * 4 + 15) & ~15u;
  l.rows_at = at;
  at += (NARROW_T / 64) * (unsigned)p.Dm * 64 * 8;
  l.total = at;
  return l;
}

__host__ __device__ inline bool narrow_ok(const DProblem& p) {
  return p.V <= NARROW_MAXV && p.Dm4 <= NARROW_MAXF && p.C <= NARROW_MAXF &&
         p.n_sumdiff == 0 && p.Dm >= 1;
}

// A lane's row: mutable features from its LDS column, immutable ones from x_init.
struct NarrowRow {
  const double* xs;    // wave block [Dm][64], offset by the lane
  const int* mslot;    // [D]: mutable slot or -1
  const double* xi;    // the state's x_init [D]
  __device__ __forceinline__ double operator[](int f) const {
    const int m = mslot[f];
    return m >= 0 ? xs[m * 64] : xi[f];
  }
};

// The wave butterfly's balanced tree restated on one lane (leaf j = what lane j of the wave
// kernel holds; leaves past the pushed ones are +0.0): a binary-counter stack whose levels
// are static registers; the leaf index is wave-uniform, so every branch is uniform.  The
// tree over all 64 leaves equals the tree over the first power of two P2 >= n leaves plus
// one "+ 0.0" (the all-zero subtrees above it) when P2 < 64.
template <bool MAX>
struct LaneTree {
  double st[7];
  int j = 0;
  __device__ __forceinline__ static double comb(double a, double b) {
    return MAX ? nanmax(a, b) : a + b;
  }
  __device__ __forceinline__ void push(double v) {
    bool carry = true;
#pragma unroll
    for (int L = 0; L < 7; ++L) {
      const bool bit = (j >> L) & 1;
      if (carry && bit) v = comb(st[L], v);
      if (carry && !bit) {
        st[L] = v;
        carry = false;
      }
    }
    ++j;
  }
  __device__ __forceinline__ double finish() {
    if (j == 0) return 0.0;
    int lg = 0;
    while ((1 << lg) < j) ++lg;
    while (j < (1 << lg)) push(0.0);
    double r = 0.0;
#pragma unroll
    for (int L = 0; L < 7; ++L) r = L == lg ? st[L] : r;
    return lg < 6 ? comb(r, 0.0) : r;
  }
};

// The body of k_narrow (eval.hip): workgroup blockIdx.x takes rows [128 x, 128 x + 128) of
// the launch's B x n rows, lane = row.
template <int NV, bool FULL>
__device__ __forceinline__ void narrow_rows(const RowsArgs& a, int gen, int hist_row0,
                                            unsigned char* smem) {
  const DProblem& p = a.p;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int V = p.V, Dm = p.Dm, Dm4 = p.Dm4;
  const VaryOff o = vary_offsets(p);
  const NarrowLds L = narrow_lds(o, p);
  glds_copy<NARROW_T>(smem + L.a_at, p.vblob, o.a_end, wave, lane);
  glds_copy<NARROW_T>(smem + L.b_at, p.vblob + o.b_at, o.b_end - o.b_at, wave, lane);
  glds_copy<NARROW_T>(smem + L.c_at, p.vblob + o.c_at, o.c_end - o.c_at, wave, lane);
  int* mslot = (int*)(smem + L.m_at);
  for (int f = tid; f < p.D; f += NARROW_T) mslot[f] = -1;
  __builtin_amdgcn_s_waitcnt(0);
  __syncthreads();
  const int* s_ginfo = (const int*)(smem + L.b_at + (o.ginfo - o.b_at));
  const uint32_t* s_geo = (const uint32_t*)(smem + L.b_at + (o.geo - o.b_at));
  const int* s_mutf = (const int*)(smem + L.b_at + (o.mutf - o.b_at));
  const int* s_ooff = (const int*)(smem + L.b_at + (o.ooff - o.b_at));
  const int* s_ofeat = (const int*)(smem + L.b_at + (o.ofeat - o.b_at));
  const double* s_mlS = (const double*)(smem + L.c_at + (o.mlS - o.c_at));
  const double* s_mlM = (const double*)(smem + L.c_at + (o.mlM - o.c_at));
  for (int j = tid; j < Dm; j += NARROW_T) mslot[s_mutf[j]] = j;
  __syncthreads();

  // this lane's row (dead lanes of the last workgroup run state 0 row 0, store nothing)
  const long r = (long)blockIdx.x * NARROW_T + tid;
  const bool live = r < a.total;
  const int b = live ? (int)(r / a.n) : 0;
  const int i = live ? (int)(r - (long)b * a.n) : 0;
  const int orow = a.out_map ? a.out_map[(size_t)b * a.n + i] : i;
  const unsigned char* sblob = a.s.sblob + (size_t)b * o.sb;
  const double* gin = a.genes_in + (size_t)b * a.in_rows * V;

  // child genes (registers; mutations are patched in after the decode, below)
  double x[NV];
  const double* go = gin + (size_t)i * V;  // own parent (mode 0: the row itself)
  const double* gt = go;                   // other parent
  CxSub c0{0, 0, 0}, c1{0, 0, 0};
  int m = 0;
  const Rng rng(a.seed, state_stream(a.stream_key, a.state_keys, a.key0, b));
  if (a.mode == 1) {  // two-point crossover of the mating's subsets (k_gen load_row)
    const int nm = a.n / 2;
    m = i % nm;
    const int side = i / nm;
    const int2 pr = *(const int2*)(a.parents + ((size_t)b * nm + m) * 2);
    go = gin + (size_t)(side ? pr.y : pr.x) * V;
    gt = gin + (size_t)(side ? pr.x : pr.y) * V;
    c0 = cx_sub(rng, gen, m, 0, p.n_sub[0], a.cx_prob);
    c1 = cx_sub(rng, gen, m, 1, p.n_sub[1], a.cx_prob);
  }
#pragma unroll
  for (int g = 0; g < NV; ++g) {
    x[g] = 0.0;
    if (g < V) {
      const bool sw = gene_swapped(s_ginfo[g], c0.on, c0.lo, c0.hi, c1.on, c1.lo, c1.hi);
      x[g] = (sw ? gt : go)[g];
    }
  }
  double* gout =
      (live && a.genes_out) ? a.genes_out + ((size_t)b * a.out_rows + orow) * V : nullptr;
  if (gout) {
#pragma unroll
    for (int g = 0; g < NV; ++g)
      if (g < V) gout[g] = x[g];
  }

  // decode (feature_encoder.py:91-124) into the lane's column of the wave block
  double* xs = (double*)(smem + L.rows_at) + (size_t)wave * Dm * 64 + lane;
  const double* xi = (const double*)(sblob + o.xi);
  for (int j = 0; j < Dm; ++j) xs[j * 64] = xi[s_mutf[j]];
  auto put = [&](int info, double v) {
    const int feat = (info >> 17) & 0x7FFF;
    if ((info & 3) != 2) {
      xs[mslot[feat] * 64] = v;
    } else {
      const int o0 = s_ooff[feat], o1 = s_ooff[feat + 1];
      for (int k = o0; k < o1; ++k) xs[mslot[s_ofeat[k]] * 64] = (v == (double)(k - o0)) ? 1.0 : 0.0;
    }
  };
#pragma unroll
  for (int g = 0; g < NV; ++g)
    if (g < V) put(s_ginfo[g], x[g]);

  // every mutation of the row's geometric-gap sequence (mutation_draws), in position order:
  // positions are distinct, so each mutates the crossed value (re-read from its parent) and
  // overwrites that gene in the pool row and its features in the LDS column
  if (a.mode == 1) {
    const double* gl = a.s.gl + (size_t)b * V;
    const double* gu = a.s.gu + (size_t)b * V;
    const float lq = __log2f(1.0f - 1.0f / (float)V);
    int pos = -1;
    for (int j = 0;; ++j) {
      const u32x4 w = rng.draw((uint32_t)(i * MUT_J + j), (uint32_t)gen, TAG_MUT_MASK);
      pos += 1 + geo_gap(s_geo, V, w.x, lq);
      if (pos >= V) break;
      const int info = s_ginfo[pos];
      const bool sw = gene_swapped(info, c0.on, c0.lo, c0.hi, c1.on, c1.lo, c1.hi);
      const double xv = mutate_gene((sw ? gt : go)[pos], gl[pos], gu[pos], (info & 3) == 0,
                                    u53(w.y, w.z), a.eta);
      if (gout) gout[pos] = xv;
      put(info, xv);
    }
  }

  // fp32 ML row for k_mlp2 (default_problem.py:119-121) and f2 (default_problem.py:80-91)
  const double* s_es = (const double*)(sblob + o.es);
  const double* s_em = (const double*)(sblob + o.em);
  const double* s_x0 = (const double*)(sblob + o.x0);
  const bool l2 = p.norm == 2;
  float* xo = a.xml + ((size_t)b * a.n + i) * Dm4;
  LaneTree<false> t2s;
  LaneTree<true> t2m;
  for (int j = 0; j < Dm4; j += 4) {
    float v[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      v[q] = 0.f;
      if (j + q < Dm) {
        const int jq = j + q;
        const double xf = xs[jq * 64];
        v[q] = (float)(xf * s_mlS[jq] + s_mlM[jq]);
        const double d = (xf * s_es[jq] + s_em[jq]) - s_x0[jq];
        if (l2)
          t2s.push(0.0 + d * d);
        else
          t2m.push(nanmax(0.0, fabs(d)));
      }
    }
    if (live) *(float4*)(xo + j) = make_float4(v[0], v[1], v[2], v[3]);
  }
  double f2 = l2 ? sqrt(t2s.finish()) : t2m.finish();
  if (p.scale_obj) f2 = f2 * p.f2_scale + 0.0;

  // constraint program (Constraints.evaluate numpy path + default_problem.py:93-97,128-129)
  OpTab tab;
  tab.code = (const int*)(smem + L.a_at + o.opc);
  tab.arg = (const int4*)(smem + L.a_at + o.opa);
  tab.k = (const double2*)(smem + L.a_at + o.opk);
  tab.col = (const int*)(smem + L.a_at + o.ocol);
  tab.pool = (const int*)(smem + L.a_at + o.pool);
  tab.C = p.C;
  tab.n_lane = p.C;
  tab.tol = p.tol;
  const NarrowRow xr{xs, mslot, xi};
  double* grow = (live && a.G) ? a.G + ((size_t)b * a.n + i) * p.C : nullptr;
  double* hrow =
      (live && a.hist) ? a.hist + ((size_t)b * a.hist_rows + hist_row0 + i) * a.hist_w : nullptr;
  double* hcols = (hrow && a.hist_w > 3) ? hrow + 3 : nullptr;
  LaneTree<false> t3;
  for (int c = 0; c < p.C; ++c) {
    double v = eval_op<FULL>(tab, c, xr);
    if (v <= tab.tol) v = 0.0;
    const double g = v * (v > 0.0 ? 1.0 : 0.0);
    if (grow) grow[tab.col[c]] = g;
    if (hcols) hcols[tab.col[c]] = g;
    t3.push(0.0 + g);
  }
  const double f3 = t3.finish() + 0.0;
  if (live) {
    if (a.F) {
      a.F[((size_t)b * a.out_rows + orow) * 3 + 1] = f2;
      a.F[((size_t)b * a.out_rows + orow) * 3 + 2] = f3;
    }
    if (hrow) {
      hrow[1] = f2;
      hrow[2] = f3;
    }
  }
}

}  // namespace mv
