// Launch wrappers shared by the C-ABI layer (api.cpp) and the kernel files.
#pragma once
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>

#include "engine.h"

namespace mv {

// Kernel-exact profiling (mv_set_profiling): api.cpp sets a start / stop event pair before a
// profiled launch; the next MV_LAUNCH hands them to hipExtLaunchKernelGGL, which stamps the
// kernel's own start and end (events recorded around the launch would include the dispatch
// gap: ~8 us per k_genc launch, so the bench's per-kernel times now agree with rocprofv3's),
// and clears them.  Unset, MV_LAUNCH is hipLaunchKernelGGL.
extern thread_local hipEvent_t g_ev_start, g_ev_stop;
#define MV_LAUNCH(K, GRID, BLOCK, LDS, STREAM, ...)                                          \
  do {                                                                                       \
    if (::mv::g_ev_start) {                                                                  \
      hipExtLaunchKernelGGL(K, GRID, BLOCK, LDS, STREAM, ::mv::g_ev_start, ::mv::g_ev_stop,  \
                            0, __VA_ARGS__);                                                 \
      ::mv::g_ev_start = nullptr;                                                            \
      ::mv::g_ev_stop = nullptr;                                                             \
    } else {                                                                                 \
      hipLaunchKernelGGL(K, GRID, BLOCK, LDS, STREAM, __VA_ARGS__);                          \
    }                                                                                        \
  } while (0)

// LDS of k_mlp / k_predict: head (32 row states + final-layer weights and bias) + R1 (A tile
// / ping) + R2 (pong).
__host__ __device__ inline size_t eval_region1_bytes(int Dm4, int hmax) {
  const size_t a = (size_t)EVAL_TR * (Dm4 + 1) * sizeof(float);
  const size_t h = (size_t)EVAL_TR * (hmax + 1) * sizeof(float);
  const size_t r = a > h ? a : h;
  return (r + 15) & ~(size_t)15;
}
__host__ __device__ inline size_t mlp_head_bytes(int Klast, int nout) {
  const size_t w = (size_t)(Klast * nout + nout) * sizeof(float);
  return 128 + ((w + 15) & ~(size_t)15);
}
__host__ __device__ inline size_t mlp_lds_bytes(int Dm4, int hmax, int Klast, int nout) {
  return mlp_head_bytes(Klast, nout) + eval_region1_bytes(Dm4, hmax) +
         (size_t)EVAL_TR * (hmax + 1) * sizeof(float);
}

// Problem and per-state blobs: HBM images of LDS regions, each region 1-KiB aligned so a
// workgroup stages the regions it needs with 16-B-per-lane global_load_lds copies.
//   problem blob  A: constraint program (opa, opk, opc, ocol, pool)       -> k_cons
//                 B: mutation gap table, gene table, mutable features,
//                    one-hot group offsets / features, cmap [Vr] (gene -> stored gene or
//                    -1, fixed) and fidx [V] (stored gene -> gene)        -> k_gen
//                 C: ML scaler at the mutable features (mlS, mlM)         -> k_gen
//                 S: the slim program of k_genc's phase 2 (DIFF / RATIO_SAFE lane ops and
//                    ABS_SUMDIFF only): k (fp64), col, pool, sum-diff args, 0.0 -> LDS; the
//                    ops' packed words (code | a0 << 4 | a1 << 18) read from HBM
//   state blob    X: x_init                                               -> k_cons (k_gen OHE)
//                 E: encoder MinMax at the mutable features (es, em, x0)  -> k_gen
struct VaryOff {
  unsigned opa, opk, opc, ocol, pool, a_end;      // region A at 0
  unsigned geo, ginfo, mutf, ooff, ofeat, cmap, fidx, b_at, b_end;  // region B at b_at
  unsigned mlS, mlM, c_at, c_end;                 // region C at c_at
  unsigned s_k, s_col, s_pool, s_sd, s_zero, s_at, s_end;  // region S (staged part) at s_at
  unsigned s_opw, vb;                             // S packed op words; vb = blob bytes
  unsigned xi, x_end;                             // region X at 0
  unsigned es, em, x0, e_at, sb;                  // region E at e_at; sb = blob bytes
  unsigned rb;                                    // ML row buffer bytes
  unsigned rbs;                                   // slim row buffer bytes (Dm doubles, padded to 64)
};
__host__ __device__ inline VaryOff vary_offsets(const DProblem& p) {
  VaryOff o{};
  size_t off = 0;
  auto take = [&](size_t bytes) {
    const unsigned at = (unsigned)off;
    off = (off + bytes + 15) & ~(size_t)15;
    return at;
  };
  auto kb = [](size_t x) { return (unsigned)((x + 1023) & ~(size_t)1023); };
  const size_t C = p.C, Dm4 = p.Dm4;
  o.opa = take(C * 16);
  o.opk = take(C * 16);
  o.opc = take(C * 4);
  o.ocol = take(C * 4);
  o.pool = take((size_t)p.n_pool * 4);
  o.a_end = kb(off);
  o.b_at = o.a_end;
  off = o.b_at;
  o.geo = take((size_t)(p.Vr + 1) * 4);
  o.ginfo = take((size_t)((p.V + 3) & ~3) * 4);
  o.mutf = take(Dm4 * 4);
  o.ooff = take((size_t)(p.n_ohe + 1) * 4);
  o.ofeat = take((size_t)(p.n_ohe_feat > 0 ? p.n_ohe_feat : 1) * 4);
  o.cmap = take((size_t)p.Vr * 4);
  o.fidx = take((size_t)p.V * 4);
  o.b_end = kb(off);
  o.c_at = o.b_end;
  off = o.c_at;
  o.mlS = take(Dm4 * 8);
  o.mlM = take(Dm4 * 8);
  o.c_end = kb(off);
  o.s_at = o.c_end;
  off = o.s_at;
  o.s_k = take(C * 8);
  o.s_col = take(C * 4);
  o.s_pool = take((size_t)p.n_pool * 4);
  o.s_sd = take((size_t)(p.n_sumdiff > 0 ? p.n_sumdiff : 1) * 16);
  o.s_zero = take(16);  // a 0.0 (constraints_slim's absent sum-diff terms read it)
  o.s_end = kb(off);
  off = o.s_end;
  o.s_opw = take(C * 4);
  o.vb = kb(off);
  off = 0;
  o.xi = take((size_t)p.D * 8);
  o.x_end = kb(off);
  o.e_at = o.x_end;
  off = o.e_at;
  o.es = take(Dm4 * 8);
  o.em = take(Dm4 * 8);
  o.x0 = take(Dm4 * 8);
  o.sb = kb(off);
  o.rb = (unsigned)(((size_t)p.D * 8 + 15) & ~(size_t)15);
  // whole 64-gene registers: k_genc writes every lane of its row registers unconditionally
  o.rbs = (unsigned)(((size_t)p.Dm + 63) / 64 * 64 * 8);
  return o;
}
// k_gen keeps the ML-scaler / encoder coefficients of its genes in registers for IDENT
// problems with at most 8 genes per lane (no LDS staging of regions C and E then).
constexpr bool GEN_REGC = false;  // k_gen: coefficients in registers (true) or LDS (false)
__host__ __device__ inline bool gen_regc(const DProblem& p, int nt) {
  return GEN_REGC && p.ident && nt <= 8;
}
// k_gen LDS: region B [, C, E] [, X + one row per wave for one-hot decoding]
struct GenLds {
  unsigned b_at, c_at, e_at, x_at, rows_at, total;
};
__host__ __device__ inline GenLds gen_lds(const VaryOff& o, bool regc, bool ident, bool eval) {
  GenLds l{};
  unsigned at = 0;
  l.b_at = at;
  at += o.b_end - o.b_at;
  if (eval && !regc) {
    l.c_at = at;
    at += o.c_end - o.c_at;
    l.e_at = at;
    at += o.sb - o.e_at;
  }
  if (eval && !ident) {
    l.x_at = at;
    at += o.x_end;
    l.rows_at = at;
    at += (VARY_T / 64) * o.rb;
  }
  l.total = at;
  return l;
}
// k_genc's two-point slim instance (EARLY): everything is staged at its start and the
// constraint program runs inside phase 1's row loop on the child genes still in registers --
// no second row loop, no re-read of the children, no phase barrier (round 5: k_genc PMC
// 343 -> 250 MB per launch).  Phase 1 reads its gene tables from the problem blob (the
// variation plan leaves only the gene info there).  LDS: [S][X][E (and C)][one row per wave].
__host__ __device__ inline GenLds genc_fused_lds(const VaryOff& o, const DProblem& p) {
  GenLds l{};
  const unsigned ssz = o.s_end - o.s_at;
  const unsigned e_sz = o.sb - o.e_at;
  l.b_at = 0;
  l.x_at = ssz;
  l.e_at = ssz + o.x_end;
  l.c_at = l.e_at + e_sz;
  l.rows_at = l.c_at + (p.xml_direct ? 0u : (o.c_end - o.c_at));
  l.total = l.rows_at + CONS_W * o.rbs;
  return l;
}
// SBX rows: a per-wave list of the crossed genes (int) and their children (double) after the
// k_gen layout (rowops.h sbx_row)
__host__ __device__ inline unsigned gen_sbx_at(const GenLds& l) { return (l.total + 15u) & ~15u; }
__host__ __device__ inline unsigned gen_sbx_wave_bytes(int nt) { return 64u * (unsigned)nt * 12u; }
__host__ __device__ inline unsigned gen_lds_sbx(const GenLds& l, int nt) {
  return gen_sbx_at(l) + VARY_W * gen_sbx_wave_bytes(nt);
}
// k_cons LDS: region A, region X, one row per wave
__host__ __device__ inline unsigned cons_lds_total(const VaryOff& o) {
  return o.a_end + o.x_end + CONS_W * o.rb;
}
// k_genc's phase 2 with the slim program (DProblem.slim): region S, region X, one row of the
// stored mutable features per wave (the operands are SlotRow slots)
__host__ __device__ inline unsigned cons_lds_slim(const VaryOff& o) {
  return (o.s_end - o.s_at) + o.x_end + CONS_W * o.rbs;
}

// k_predict: TR-row tiles (32, or 16 for inputs too wide for a 32-row tile)
__host__ __device__ inline size_t predict_region1_bytes(int D4, int hmax, int TR) {
  const size_t a = (size_t)TR * (D4 + 1) * sizeof(float);
  const size_t h = (size_t)TR * (hmax + 1) * sizeof(float);
  const size_t r = a > h ? a : h;
  return (r + 15) & ~(size_t)15;
}
__host__ __device__ inline size_t predict_lds_bytes(int D4, int hmax, int Klast, int nout, int TR) {
  return mlp_head_bytes(Klast, nout) + predict_region1_bytes(D4, hmax, TR) +
         (size_t)TR * (hmax + 1) * sizeof(float);
}

// Development sensitivity knob: MV_LDS_PAD_<KERNEL> extra bytes of dynamic LDS requested
// by a launch (GENC, MLP, SURV), to measure how the chain's throughput depends on each
// kernel's LDS footprint (co-residency on a CU).  0 when unset.
size_t lds_pad(const char* env);

hipError_t launch_predict(const MlpArgs& a, hipStream_t stream);
hipError_t launch_decode(const DProblem& p, const DStates& s, int B, int n, const double* genes,
                         double* x, hipStream_t stream);

// Launch-argument ring (constant memory, per device): stage a copy on `stream`, launch with
// the returned slot, then release it on the same stream after the slot's last launch.
hipError_t stage_rows(const RowsArgs& a, hipStream_t stream, int* slot);
hipError_t release_rows(int slot, hipStream_t stream);
size_t surv_lds_bytes(int N, int R, int P, int ptab_words = 0, int threads = 0);

hipError_t launch_gen(const RowsArgs& a, int slot, int gen, int hist_row0, hipStream_t stream);
// Which kernels launch_gen / launch_cons run for these rows: 0 k_gen + k_cons, 1 k_narrow
// (launch_cons is empty), 2 k_genc (launch_cons is empty)
int row_kernel_kind(const RowsArgs& a);
int mlp_kernel_kind(const DProblem& p);
hipError_t launch_cons(const RowsArgs& a, int slot, int hist_row0, hipStream_t stream);
hipError_t launch_vary(const RowsArgs& a, int slot, int gen, int hist_row0,
                       hipStream_t stream);
hipError_t launch_mlp(const RowsArgs& a, int slot, int hist_row0, hipStream_t stream);
hipError_t launch_rows(const RowsArgs& a, int slot, int gen, int hist_row0,
                       hipStream_t stream);
hipError_t launch_constraints(const DProblem& hp, int slot, int n, const double* x,
                              double* G, hipStream_t stream);
hipError_t launch_setup_states(int slot, int B, const double* x_init, const double* xl,
                               const double* xu, const float* W1full, const float* b1, double* gl,
                               double* gu, unsigned char* sblob, float* bias1, double* genes0,
                               hipStream_t stream);
hipError_t launch_survive(const SurvArgs& a, int B, hipStream_t stream);
hipError_t launch_select(int B, int P, int O, uint64_t seed, uint32_t stream_key, int gen,
                         const int* pop_slot, int* parents, hipStream_t stream);
hipError_t launch_init_pool(int B, int P, int O, int V, int S, const double* genes0,
                            double* pool, int* pop_slot, int* free_slot, hipStream_t stream);
hipError_t launch_obj_mlscale(long total, int D, const double* x, const double* s,
                              const double* m, double* out, hipStream_t stream);
hipError_t launch_objectives(const ObjArgs& a, hipStream_t stream);
// pool rows (V stored genes) -> population genes [B][P][Vr]: a fixed gene (cmap < 0, compact
// layout) is its state's bound glr[b][g] (the full layout's genetic lower bound)
hipError_t launch_gather_pop(int B, int P, int V, int Vr, int S, const int* cmap,
                             const double* glr, const int* pop_slot, const double* pool,
                             const double* poolF, double* genes, double* F, hipStream_t stream);
// final population -> non-dominated mask front [B][P], row offsets [B+1], and (optional) the
// members' genes X [rows][Vr] / objectives Fx [rows][3] packed in state and population order
hipError_t launch_front(int B, int P, int V, int Vr, int S, const int* cmap, const double* glr,
                        const int* pop_slot, const double* pool, const double* poolF,
                        unsigned char* front, int* offsets, double* X, double* Fx,
                        hipStream_t stream);

}  // namespace mv
