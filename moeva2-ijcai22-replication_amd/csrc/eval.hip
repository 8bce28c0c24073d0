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
#include <cstdlib>
#include <mutex>

#include "check.h"
#include "engine.h"
#include "kernels.h"
#include "narrow.h"
#include "philox.h"
#include "rowops.h"
#include "wave.h"

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

size_t lds_pad(const char* env) {
  const char* v = std::getenv(env);
  return v ? (size_t)std::atol(v) : 0;
}

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

// The draws of one offspring row: packed parents (own | oth << 16) and the two crossover
// subsets' draws on the row's lane k; its mutations on lanes 4 k + q (a wave holds <= 16
// rows): lane 4 k + q takes the q-th draw of row k's geometric-gap process (Philox index
// row * MUT_J + q, TAG_MUT_MASK), the gaps' prefix sum over the row's four lanes gives the
// positions -- the same draws and positions as walking them one after another, computed in
// one parallel round -- and the lane mutates its position's crossed parent value
// (mutate_gene).  mut_v (row lane k): count | overflow << 3; a row with more than CAP
// mutations (its 5th draw is still inside the genes, checked on lane 4 k + 3) is redone by
// the caller with every mutation.  mposv / mvalv (lane 4 k + q): the stored gene (-1: a
// fixed gene of the compact layout, whose mutation is the identity) and its new value.
// (A separate one-row-per-lane kernel computing these ahead of k_gen was measured slower:
// its serial Philox / pow chains sit on the generation's critical path.)
// `preload` runs once the mating is known, before the mutation draws: the caller issues the
// first rows' parent loads there, so their latency overlaps the Philox / gather / pow work.
template <int CAP, class Preload>
__device__ __forceinline__ void row_draws(const RowsArgs& a, const DProblem& p, const int b,
                                          const int irow, const bool mine, const int gen,
                                          const bool sbx, const uint32_t* geo, const int* ginfo,
                                          const int* cmap, const double* gin, const Rng& rng,
                                          int& par_v, int& cx0_v, int& cx1_v, int& mut_v,
                                          int& mposv, double& mvalv, const int2 pre_pr,
                                          Preload&& preload) {
  const int V = p.V, Vr = p.Vr;  // stored genes, genes the draws are defined over
  if (mine) {
    const int nm = a.n / 2;
    const int m = irow % nm;
    const int side = irow / nm;
    const int2 pr = pre_pr;  // the row's mating, loaded by the caller ahead of its staging
    par_v = side ? (pr.y | (pr.x << 16)) : (pr.x | (pr.y << 16));
    cx0_v = pack_cx(cx_sub(rng, gen, m, 0, p.n_sub[0], a.cx_prob));
    cx1_v = pack_cx(cx_sub(rng, gen, m, 1, p.n_sub[1], a.cx_prob));
    if (sbx) {  // SBX: the subsets' mating-level draws only (no segment)
      cx0_v &= 1;
      cx1_v &= 1;
    }
  }
  preload();
  static_assert(CAP == 4, "row_draws maps 16 rows x 4 mutations onto the 64 lanes");
  static_assert(VARY_ROWS_MAX <= 16 * VARY_W, "more than 16 rows per wave (vary_rows_per_wg)");
  static_assert(VARY_ROWS_MAX <= (64 / PLAN_MUT) * VARY_W, "plan_draws: 8 rows per wave at most");
  const int lane = threadIdx.x & 63;
  const int kk = lane >> 2, qq = lane & 3;
  // (1) draw qq of row kk: its gap and PM uniform, then the positions (prefix sums of the
  // 1 + gap steps from -1 within the row's four lanes)
  const int irow_k = __shfl(irow, kk);
  const bool live = __shfl(mine ? 1 : 0, kk) != 0 && !sbx;
  const float lq = __log2f(1.0f - 1.0f / (float)Vr);
  int st = 0;
  double uq = 0.0;
  if (live) {
    const u32x4 w = rng.draw((uint32_t)(irow_k * MUT_J + qq), (uint32_t)gen, TAG_MUT_MASK);
    st = 1 + geo_gap(geo, Vr, w.x, lq);
    uq = u53(w.y, w.z);
  }
  {
    const int t1 = __shfl(st, (lane + 63) & 63);
    st += qq >= 1 ? t1 : 0;
    const int t2 = __shfl(st, (lane + 62) & 63);
    st += qq >= 2 ? t2 : 0;
  }
  const int pq = st - 1;                // position of draw qq (increasing in qq)
  const bool hit = live && pq < Vr;     // the hits of a row are its lanes 0 .. count - 1
  int ovf = 0;
  if (qq == CAP - 1 && hit) {           // four mutations: does a fifth fall inside?
    const u32x4 w = rng.draw((uint32_t)(irow_k * MUT_J + CAP), (uint32_t)gen, TAG_MUT_MASK);
    ovf = pq + 1 + geo_gap(geo, Vr, w.x, lq) < Vr ? 1 : 0;
  }
  const unsigned long long hm = __ballot(hit), om = __ballot(ovf != 0);
  // (2) + (3) lane 4 k + q loads row k's crossed parent value and gene bounds at its
  // position and mutates it -- one pow pair deep for the whole wave.  The position is mapped
  // to its stored gene (cmap); a fixed gene of the compact layout (-1) is not stored and its
  // mutation is the identity (integer gene, xl == xu == value): the draw stays, the write
  // goes.
  const double* gl = a.s.gl + (size_t)b * V;
  const double* gu = a.s.gu + (size_t)b * V;
  const int park = __shfl(par_v, kk);
  const int c0k = __shfl(cx0_v, kk), c1k = __shfl(cx1_v, kk);
  const int pc = hit ? pq : 0;
  const int cq = cmap[MV_IDX(pc, Vr, CK_GEN_MUTPOS)];  // unconditional loads
  const int mp = MV_IDX(cq < 0 ? 0 : cq, V, CK_GEN_MUTPOS);
  const int gi = ginfo[mp];
  const int mrow = MV_IDX(swapped_packed(gi, c0k, c1k) ? (park >> 16) : (park & 0xFFFF),
                          a.in_rows, CK_GEN_MUTROW);
  double xv = gin[MV_IDX((size_t)mrow * V + mp, (long long)a.in_rows * V, CK_AT_MUTLOAD)];
  const double lo = gl[MV_IDX(mp, V, CK_AT_BOUNDS)], hi = gu[MV_IDX(mp, V, CK_AT_BOUNDS)];
  if (hit) xv = mutate_gene(xv, lo, hi, (gi & 3) == 0, uq, a.eta);
  mposv = hit ? cq : -1;
  mvalv = xv;
  const int cnt = __popcll((hm >> (4 * (lane & 15))) & 0xFull);  // row lanes k < 16
  mut_v = cnt | ((int)((om >> (4 * (lane & 15) + 3)) & 1ull) << 3);
}

// The draws of a wave's rows from the generation's variation plan (k_genc; engine.h VPlan):
// lane k < nrw holds row k's header (parents, crossover draws, mutation count | overflow
// << 4), lane PLAN_MUT k + q row k's q-th planned mutation (pmw / pmu, loaded at kernel
// start).  Two-point: the lane gathers the crossed parent's value at its stored gene and
// mutates it (mutate_gene, as row_draws) -> mposv / mvalv; the first rows' parent loads go
// out after the gathers, so the pow chains wait for the gathers only.  SBX: the mutations
// apply to the row loop's SBX children, so mposv / mvalv keep the planned word / uniform.
template <int NT, class Preload>
__device__ __forceinline__ void plan_draws(const RowsArgs& a, const DProblem& p, const int b,
                                           const bool mine, const bool sbx, const double* gin,
                                           const int4 hdr, const int pmw, const double pmu,
                                           int& par_v, int& cx0_v, int& cx1_v, int& mut_v,
                                           int& mposv, double& mvalv, Preload&& preload) {
  const int V = p.V;
  if (mine) {
    par_v = hdr.x;
    cx0_v = hdr.y;
    cx1_v = hdr.z;
    mut_v = hdr.w;
  }
  const int lane = threadIdx.x & 63;
  const int kk = lane >> 3, qq = lane & 7;
  const int cnt = __shfl(mut_v, kk) & 15;  // rows past the wave's: mut_v 0
  const bool hit = qq < cnt;
  if (sbx) {
    preload();
    mposv = hit ? pmw : -1;
    mvalv = pmu;
    return;
  }
  const int park = __shfl(par_v, kk);
  const int cq = hit ? MV_IDX(pmw & 0xFFFF, V, CK_GEN_MUTPOS) : 0;
  const int mrow = MV_IDX(hit && ((pmw >> 17) & 1) ? (park >> 16) : (park & 0xFFFF), a.in_rows,
                          CK_GEN_MUTROW);
  const double* gl = a.s.gl + (size_t)b * V;
  const double* gu = a.s.gu + (size_t)b * V;
  double xv = gin[MV_IDX((size_t)mrow * V + cq, (long long)a.in_rows * V, CK_AT_MUTLOAD)];
  const double lo = gl[MV_IDX(cq, V, CK_AT_BOUNDS)], hi = gu[MV_IDX(cq, V, CK_AT_BOUNDS)];
  preload();
  if (hit) xv = mutate_gene(xv, lo, hi, ((pmw >> 16) & 1) != 0, pmu, a.eta);
  mposv = hit ? cq : -1;
  mvalv = xv;
}

// k_gen: variation (mode 1) or gene load (mode 0), the child genes to the pool, the fp32
// ML-scaled mutable row for k_mlp (default_problem.py:119-121) and f2, the encoder-MinMax
// distance (default_problem.py:80-91).
//
// Lane l owns genes l + 64t: coalesced 512-B gene loads/stores, its gene-table words (and,
// REGC, its ML-scaler / encoder coefficients) in registers; the next row's parent genes
// are loaded while the current row is finished.  Two-point crossover draws and the
// mutations are precomputed for all of a wave's rows at once, one row per lane: mutations
// are a geometric-gap process (about two Philox draws per row instead of one word per
// gene), at most MUT_CAP per row cached in registers, the rare rest finished in the row.
// SBX: the SBX crossover option compiled in (a separate instance: its pow()-heavy path
// doubled the two-point kernel's registers, halving its occupancy).
// PLAN (k_genc): mode 1 takes its draws from the variation plan (plan_draws).  EARLY (k_genc's
// two-point slim instance, IDENT): the whole kernel's LDS is staged here (genc_early_lds) and
// phase 1 reads its gene tables from the problem blob.
template <bool IDENT, int NT, bool SBX, bool PLAN = false, bool EARLY = false>
__device__ __forceinline__ int gen_rows(const RowsArgs& a, int gen, int hist_row0, int rows_wg,
                                        unsigned char* smem) {
  static_assert(!EARLY || (IDENT && PLAN && !SBX), "early staging: k_genc two-point only");
  constexpr bool FUSED = EARLY;  // the constraints inside the row loop (genc_fused_lds)
  constexpr bool REGC = GEN_REGC && IDENT && NT <= 8;  // kernels.h gen_regc
  const DProblem& p = a.p;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const RowChunk rc = row_chunk(a.n, rows_wg, wave);
  const int b = MV_IDX(rc.b, a.total / a.n, CK_GEN_STATE), nrw = rc.nrw;
  const int V = p.V, Dm = p.Dm, Dm4 = p.Dm4;
  const bool ev = a.do_eval != 0;
  const VaryOff o = vary_offsets(p);
  const GenLds L = FUSED ? genc_fused_lds(o, p) : gen_lds(o, REGC, IDENT, ev);
  const unsigned char* sblob = a.s.sblob + (size_t)b * o.sb;
  // the rows' matings and destinations first: their round trips (the parents come from the
  // previous k_survive) overlap the LDS staging instead of following it
  const bool mine = lane < nrw;
  const int irow = rc.i0 + wave + VARY_W * lane;
  int2 pre_pr = make_int2(0, 0);
  int4 phdr = make_int4(0, 0, 0, 0);
  int pmw = 0;
  double pmu = 0.0;
  int orow_v = 0;
  if (PLAN && a.mode == 1) {  // lane PLAN_MUT k + q: row k's q-th planned mutation
    const int ir = min(rc.i0 + wave + VARY_W * (lane / PLAN_MUT), a.n - 1);
    const size_t e = ((size_t)b * a.n + ir) * PLAN_MUT + (lane % PLAN_MUT);
    pmw = a.plan_mw[e];
    pmu = a.plan_mu[e];
  }
  if (mine) {
    if (a.mode == 1) {
      if (PLAN) {
        phdr = a.plan_hdr[(size_t)b * a.n + irow];
        const int pa = MV_IDX(phdr.x & 0xFFFF, a.in_rows, CK_GEN_PARENT);
        const int pb = MV_IDX(phdr.x >> 16, a.in_rows, CK_GEN_PARENT);
        phdr.x = pa | (pb << 16);
      } else {
        const int nm = a.n / 2;
        pre_pr = *(const int2*)(a.parents + ((size_t)b * nm + irow % nm) * 2);
        pre_pr.x = MV_IDX(pre_pr.x, a.in_rows, CK_GEN_PARENT);
        pre_pr.y = MV_IDX(pre_pr.y, a.in_rows, CK_GEN_PARENT);
      }
    }
    orow_v = MV_IDX(a.out_map ? a.out_map[(size_t)b * a.n + irow] : irow, a.out_rows, CK_GEN_DST);
  }
  // FUSED: the constraint program's packed lane-op words, straight from the problem blob
  const int n_lane_ops = p.C - p.n_sumdiff;
  const int kops = min(OPS_REG, (n_lane_ops + 63) >> 6);
  unsigned opw[OPS_REG];
  if (FUSED) {
    const unsigned* gw = (const unsigned*)(p.vblob + o.s_opw);
#pragma unroll
    for (int k = 0; k < OPS_REG; ++k) {
      const int c = lane + 64 * k;
      const unsigned w_ = gw[c < n_lane_ops ? c : 0];
      opw[k] = (k < kops && c < n_lane_ops) ? w_ : 0u;
    }
  }
  if (EARLY) {  // phase 2's program + x_init, phase 1's encoder (and scaler) coefficients
    const unsigned ssz = o.s_end - o.s_at;
    glds_copy(smem, p.vblob + o.s_at, ssz, wave, lane);
    glds_copy(smem + ssz, sblob, o.x_end, wave, lane);
    if (ev) {
      glds_copy(smem + L.e_at, sblob + o.e_at, o.sb - o.e_at, wave, lane);
      if (!p.xml_direct) glds_copy(smem + L.c_at, p.vblob + o.c_at, o.c_end - o.c_at, wave, lane);
    }
  } else {
    glds_copy(smem + L.b_at, p.vblob + o.b_at, o.b_end - o.b_at, wave, lane);
    if (ev && !REGC) {
      glds_copy(smem + L.c_at, p.vblob + o.c_at, o.c_end - o.c_at, wave, lane);
      glds_copy(smem + L.e_at, sblob + o.e_at, o.sb - o.e_at, wave, lane);
    }
    if (ev && !IDENT) glds_copy(smem + L.x_at, sblob, o.x_end, wave, lane);
  }
  // per-lane gene-table words and (REGC) coefficients, straight from HBM meanwhile
  int ginf[NT];
  double cS[NT], cM[NT], cE[NT], cN[NT], cX[NT];
  {
    const int* gi = (const int*)(p.vblob + o.ginfo);
    const double* mS = (const double*)(p.vblob + o.mlS);
    const double* mM = (const double*)(p.vblob + o.mlM);
    const double* sE = (const double*)(sblob + o.es);
    const double* sN = (const double*)(sblob + o.em);
    const double* sX = (const double*)(sblob + o.x0);
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      const int g = lane + 64 * t;
      const int w = gi[g < V ? g : V - 1];  // unconditional load (see k_cons load_row)
      ginf[t] = g < V ? w : 0;
      if (REGC) {
        const bool in = ev && g < Dm4;
        cS[t] = in ? mS[g] : 0.0;
        cM[t] = in ? mM[g] : 0.0;
        cE[t] = in ? sE[g] : 0.0;
        cN[t] = in ? sN[g] : 0.0;
        cX[t] = in ? sX[g] : 0.0;
      }
    }
  }
  __builtin_amdgcn_s_waitcnt(0);
  __syncthreads();
  if (MV_CLOCKS && a.gphase && tid == 0) a.gphase[(size_t)blockIdx.x * 8 + 1] = clock64();
  // region B: LDS, or (EARLY) the problem blob itself (only the rare overflow rows read it)
  const unsigned char* rb_ = EARLY ? p.vblob + o.b_at : smem + L.b_at;
  const int* s_ginfo = (const int*)(rb_ + (o.ginfo - o.b_at));
  const uint32_t* s_geo = (const uint32_t*)(rb_ + (o.geo - o.b_at));
  const int* s_mutf = (const int*)(rb_ + (o.mutf - o.b_at));
  const int* s_cmap = (const int*)(rb_ + (o.cmap - o.b_at));
  const int* s_fidx = (const int*)(rb_ + (o.fidx - o.b_at));
  const double* s_mlS = (const double*)(smem + L.c_at + (o.mlS - o.c_at));
  const double* s_mlM = (const double*)(smem + L.c_at + (o.mlM - o.c_at));
  const double* s_es = (const double*)(smem + L.e_at + (o.es - o.e_at));
  const double* s_em = (const double*)(smem + L.e_at + (o.em - o.e_at));
  const double* s_x0 = (const double*)(smem + L.e_at + (o.x0 - o.e_at));
  double* xrow = (double*)(smem + L.rows_at + wave * o.rb);
  // FUSED: the wave's slim row buffer (stored mutable features, SlotRow) and the program's
  // LDS tables (region S at 0, x_init at L.x_at)
  double* frow = (double*)(smem + L.rows_at + wave * o.rbs);
  OpTab ftab;
  ftab.code = nullptr;
  ftab.arg = nullptr;
  ftab.k = nullptr;
  ftab.k1 = (const double*)(smem + (o.s_k - o.s_at));
  ftab.sd = (const int4*)(smem + (o.s_sd - o.s_at));
  ftab.col = (const int*)(smem + (o.s_col - o.s_at));
  ftab.pool = (const int*)(smem + (o.s_pool - o.s_at));
  ftab.C = p.C;
  ftab.n_lane = n_lane_ops;
  ftab.tol = p.tol;
  if (a.hist) {
    ftab.hlo = a.hist + (size_t)b * a.hist_rows * a.hist_w;
    ftab.hhi = ftab.hlo + (size_t)a.hist_rows * a.hist_w;
  }
  const SlotRow fsrow{frow, (const double*)(smem + L.x_at), p.Dm};
  SlimOps fso;
  if (FUSED)
    slim_ops(ftab, opw, kops, p.sd_reg != 0, frow, smem + L.x_at, smem + (o.s_zero - o.s_at),
             p.Dm, lane, fso);
  if (ev && !IDENT) {  // immutable features of this wave's row buffer (written once)
    const double* s_xi = (const double*)(smem + L.x_at);
    for (int f = lane; f < p.D; f += 64) xrow[f] = s_xi[f];
  }

  // this wave's rows: lane k holds row k's packed parents (own | oth << 16), crossover
  // draws, destination and mutations (count | overflow << 3 | (last position + 1) << 4)
  int par_v = 0, cx0_v = 0, cx1_v = 0, mut_v = 0;
  int mposv = -1;        // lane 4 k + q: row k's q-th mutation (stored gene, -1 none / fixed)
  double mvalv = 0.0;    //               and its value
  const double* gin = a.genes_in + (size_t)b * a.in_rows * V;
  const Rng rng(a.seed, state_stream(a.stream_key, a.state_keys, a.key0, b));
  const double* sgl = a.s.gl + (size_t)b * V;  // genetic bounds (SBX rows read all of them)
  const double* sgu = a.s.gu + (size_t)b * V;
  const bool sbx = SBX && a.mode == 1;
  const PoolRsrc pool = pool_rsrc(gin, (size_t)a.in_rows * V);
  unsigned pkey[NT];  // load_parent_row's crossover keys of this lane's genes
#pragma unroll
  for (int t = 0; t < NT; ++t) pkey[t] = parent_key(ginf[t]);
  auto load_row = [&](int k, double* x) {
    k = MV_IDX(k, min(nrw, 64), CK_GEN_LANE);
    load_parent_row<NT>(pool, V, rdl(par_v, k), rdl(cx0_v, k), rdl(cx1_v, k), pkey, lane, x,
                        (long long)a.in_rows * V);
  };
  // Two rows' parent genes in flight ahead of the row being finished: under load an HBM
  // round trip is ~4 us, several rows' worth of work, and one row of prefetch left each row
  // waiting on its loads (r03 phase clocks: ~9.6 k cycles per row).  The first two rows'
  // loads go out before the mutation draws, whose gathers and pow chains then overlap them.
  // k_genc's fused instance keeps one row in flight (its register budget; round 5: 220.6 vs
  // 219.3 M evals/s with two, k_genc 87.3 vs 89.3 us, no spilled registers)
  constexpr bool PF2 = !EARLY;
  double xa[NT], xb[PF2 ? NT : 1];
  auto preload = [&]() {
    if (nrw > 0) load_row(0, xa);
    if constexpr (PF2)
      if (nrw > 1) load_row(1, xb);
  };
  if (a.mode == 1) {
    if constexpr (PLAN)
      plan_draws<NT>(a, p, b, mine, sbx, gin, phdr, pmw, pmu, par_v, cx0_v, cx1_v, mut_v, mposv,
                     mvalv, preload);
    else
      row_draws<MUT_CAP>(a, p, b, irow, mine, gen, sbx, s_geo, s_ginfo, s_cmap, gin, rng, par_v,
                         cx0_v, cx1_v, mut_v, mposv, mvalv, pre_pr, preload);
  } else {
    if (mine) par_v = irow | (irow << 16);
    preload();
  }
  if (MV_CLOCKS && a.gphase && tid == 0) a.gphase[(size_t)blockIdx.x * 8 + 2] = clock64();
  const bool l2 = p.norm == 2;
  // child genes -> pool, fp32 ML row, f2 (row k of this wave, genes already mutated)
  auto finish_row = [&](int k, const double* x) {
    int Vo = V, Dmo = Dm, Dm4o = Dm4;
    asm volatile("" : "+s"(Vo), "+s"(Dmo), "+s"(Dm4o));
    const int i = MV_IDX(rc.i0 + wave + VARY_W * k, a.n, CK_GEN_ROW);
    const int orow = rdl(orow_v, MV_IDX(k, min(nrw, 64), CK_GEN_LANE));
    if (a.genes_out) {
      double* gout = a.genes_out + (size_t)b * a.out_rows * V;
      if constexpr (IDENT) {
        // through a buffer resource over the child's row: the lanes past V fall outside its
        // range and the hardware drops their stores (no per-register exec-mask branches)
        typedef unsigned u32x2 __attribute__((ext_vector_type(2)));
        const __amdgpu_buffer_rsrc_t rr = __builtin_amdgcn_make_buffer_rsrc(
            gout + (size_t)orow * V, (short)0, Vo * 8, 0x00020000);
        if (MV_CHECKS_ON) (void)MV_IDX((long long)orow, (long long)a.out_rows, CK_AT_CHILD);
#pragma unroll
        for (int t = 0; t < NT; ++t) {
          u32x2 w;
          w.x = (unsigned)__double2loint(x[t]);
          w.y = (unsigned)__double2hiint(x[t]);
          __builtin_amdgcn_raw_buffer_store_b64(w, rr, 8u * (unsigned)lane + 512u * t, 0, 0);
        }
      } else {
#pragma unroll
        for (int t = 0; t < NT; ++t)
          if (lane + 64 * t < Vo)
            gout[MV_IDX((size_t)orow * V + lane + 64 * t, (long long)a.out_rows * V, CK_AT_CHILD)] =
                x[t];
      }
    }
    if (!ev) return;
    float* xo = a.xml + ((size_t)b * a.n + i) * Dm4;
    double acc = 0.0;
    if (IDENT && !REGC && p.xml_direct) {  // f2 only, branch-free -- every lane
      // computes its term from in-range LDS reads and the sum takes +0.0 past Dm (acc >= +0,
      // never -0: the bits are those of the guarded sum)
      // (FUSED: unclamped reads at immediate offsets -- past Dm4 an index reads the next
      // array of region E, and past x0 at most 64 NT - Dm4 doubles into the wave row buffers
      // that follow it, inside the allocation; those lanes' terms are never selected.  The
      // other layouts end at region E: their indices are clamped)
      double dv[NT];
#pragma unroll
      for (int t = 0; t < NT; ++t) {
        const int j = lane + 64 * t;
        const int jc = FUSED ? j : (j < Dmo ? j : Dmo - 1);
        dv[t] = (x[t] * s_es[jc] + s_em[jc]) - s_x0[jc];
      }
      if (l2) {  // the norm's branch outside the genes (one uniform branch per row)
#pragma unroll
        for (int t = 0; t < NT; ++t) {
          const double dd = dv[t] * dv[t];
          acc = acc + (lane + 64 * t < Dmo ? dd : 0.0);
        }
      } else {
#pragma unroll
        for (int t = 0; t < NT; ++t) {
          const double m = nanmax_sel(acc, fabs(dv[t]));
          acc = lane + 64 * t < Dmo ? m : acc;
        }
      }
    } else if (IDENT) {  // gene g <-> mutable feature g: no decoding
      const bool wx = !p.xml_direct;  // else k_mlp2 scales the child genes itself
      float* xd = xo;
#pragma unroll
      for (int t = 0; t < NT; ++t) {
        const int j = lane + 64 * t;
        if (j < Dm4o) {
          float v = 0.f;
          if (j < Dmo) {
            const double xf = x[t];
            const double es = REGC ? cE[t] : s_es[j], em = REGC ? cN[t] : s_em[j];
            const double x0 = REGC ? cX[t] : s_x0[j];
            if (wx) {
              const double ms = REGC ? cS[t] : s_mlS[j], mm = REGC ? cM[t] : s_mlM[j];
              v = (float)(xf * ms + mm);
            }
            const double d = (xf * es + em) - x0;
            acc = l2 ? acc + d * d : nanmax(acc, fabs(d));
          }
          if (wx) xd[j] = v;
        }
      }
    } else {  // decode through the row buffer (feature_encoder.py:91-124)
#pragma unroll
      for (int t = 0; t < NT; ++t)
        if (lane + 64 * t < V) scatter_gene(p, xrow, ginf[t], x[t]);
      wave_sync();
      for (int j = lane; j < Dm4; j += 64) {
        float v = 0.f;
        if (j < Dm) {
          const double xf = xrow[s_mutf[j]];
          v = (float)(xf * s_mlS[j] + s_mlM[j]);
          const double d = (xf * s_es[j] + s_em[j]) - s_x0[j];
          acc = l2 ? acc + d * d : nanmax(acc, fabs(d));
        }
        xo[j] = v;
      }
      wave_sync();  // the next row's scatter overwrites xrow
    }
    if constexpr (FUSED) {  // the child into the wave's row buffer for the program below
      // (padded to whole registers, o.rbs: the lanes past V write slots no op reads)
#pragma unroll
      for (int t = 0; t < NT; ++t) frow[lane + 64 * t] = x[t];
    }
    double f3 = 0.0;
    double* hrow = nullptr;
    bool reduced = false;
    if constexpr (FUSED) {  // k_cons's do_row on the registers' child (cons_rows, SLIM)
      wave_sync();
      hrow = a.hist ? a.hist + ((size_t)b * a.hist_rows +
                                MV_IDX(hist_row0 + i, a.hist_rows, CK_CONS_DST)) * a.hist_w
                    : nullptr;
      double* hc = (hrow && a.hist_w > 3) ? hrow + 3 : nullptr;
      double* grow = a.G ? a.G + ((size_t)b * a.n + i) * p.C : nullptr;
      if (fso.sd_reg) {  // f2's sum, the lane ops' f3 part and the sum-diff columns in ONE
                         // butterfly (wave_sum4: each total bit-identical to wave_sum's)
        double a3, sdv[SD_REG], tot[4];
        constraints_slim_parts(ftab, fso, lane, grow, hc, a3, sdv);
        wave_sum4(l2 ? acc : 0.0, a3, sdv[0], sdv[1], lane, tot);
        acc = l2 ? tot[0] : wave_max(acc);
        const double sdt[SD_REG] = {tot[2], tot[3]};
        f3 = constraints_slim_finish(ftab, lane, grow, hc, tot[1], sdt);
        reduced = true;
      } else {
        f3 = constraints_slim(ftab, fso, fsrow, lane, grow, hc);
      }
    }
    if (!reduced) acc = l2 ? wave_sum(acc) : wave_max(acc);
    if (lane == 0) {
      double f2 = l2 ? sqrt(acc) : acc;
      if (p.scale_obj) f2 = f2 * p.f2_scale + 0.0;
      if (a.F) {
        double* Fr = a.F + (size_t)b * a.out_rows * 3;
        Fr[MV_IDX((size_t)orow * 3 + 1, a.out_rows * 3, CK_AT_F2)] = f2;
        if (FUSED) Fr[MV_IDX((size_t)orow * 3 + 2, a.out_rows * 3, CK_AT_F3)] = f3;
      }
      if (a.hist)
        a.hist[(size_t)b * a.hist_rows * a.hist_w +
               MV_IDX((size_t)MV_IDX(hist_row0 + i, a.hist_rows, CK_GEN_ROW) * a.hist_w + 1,
                      (long long)a.hist_rows * a.hist_w, CK_AT_HIST1)] = f2;
      if (FUSED && hrow) *MV_PTR(hrow + 2, ftab.hlo, ftab.hhi, CK_AT_HIST2) = f3;
    }
    if constexpr (FUSED) wave_sync();  // the next row overwrites the row buffer
  };
  // the row's variation (SBX children, mutations) and finish_row, on the registers x
  auto do_row = [&](int k, double (&x)[NT]) __attribute__((always_inline)) {
    if (sbx) {  // SBX children, then every mutation of the row
      const int i = rc.i0 + wave + VARY_W * k;
      const int nm = a.n / 2;
      const int pr = rdl(par_v, k);
      unsigned char* sb = smem + gen_sbx_at(L) + (size_t)wave * gen_sbx_wave_bytes(NT);
      sbx_row<NT>(x, ginf, gin + (size_t)(pr & 0xFFFF) * V, gin + (size_t)(pr >> 16) * V, sgl,
                  sgu, V, s_fidx, i % nm, i / nm, rdl(cx0_v, k) & 1, rdl(cx1_v, k) & 1, rng, gen,
                  a.sbx_eta, lane, (int*)(sb + 64 * NT * 8), (double*)sb);
      const int mv = rdl(mut_v, k);
      if (PLAN && !(mv & 16))
        plan_mutate_row<NT>(x, mv & 15, mposv, mvalv, k, lane, sgl, sgu, V, a.eta);
      else  // every mutation of the row (PLAN: more than PLAN_MUT)
        mutate_row_full<NT>(x, s_geo, s_ginfo, s_cmap, sgl, sgu, p.Vr, i, rng, gen, a.eta, lane);
    } else if (a.mode == 1) {  // apply the row's cached mutations
      if constexpr (PLAN)
        apply_row_mutations<NT, PLAN_MUT>(x, rdl(mut_v, k) & 15, mposv, mvalv, k, lane);
      else
        apply_row_mutations<NT, MUT_CAP>(x, rdl(mut_v, k) & 7, mposv, mvalv, k, lane);
    }
    finish_row(k, x);
  };
  if constexpr (PF2) {
    for (int k = 0; k < nrw; ++k) {  // xa: row k, xb: row k + 1 (in flight), rotated
      double x[NT];
#pragma unroll
      for (int t = 0; t < NT; ++t) {
        x[t] = xa[t];
        xa[t] = xb[t];
      }
      if (k + 2 < nrw) load_row(k + 2, xb);
      do_row(k, x);
    }
  } else {
    // one row in flight, two row buffers taking turns (a rotation through a copy cost ten
    // moves per row: the copy, and the loop-carried copy back).  The next row's loads are
    // unconditional (the last row re-reads row nrw - 1, from L2): loads under a branch made
    // the compiler's counter waits assume they might be missing, so every use of the current
    // row waited for the next row's loads as well.
    double xc[NT];
    for (int k = 0; k < nrw; k += 2) {
      load_row(min(k + 1, nrw - 1), xc);
      do_row(k, xa);
      if (k + 1 >= nrw) break;
      load_row(min(k + 2, nrw - 1), xa);
      do_row(k + 1, xc);
    }
  }
  // Rare: rows with more than MUT_CAP mutations are redone here with every mutation (same
  // lanes, same addresses, so these stores land after the row loop's).
  constexpr int OVF = PLAN ? 16 : 8;  // more mutations than the plan / the register cache
  if (a.mode == 1 && !sbx && __ballot(mut_v & OVF)) {
    const RowsArgs* ap = &a;
    const uint64_t seed2 = *(volatile const uint64_t*)&ap->seed;
    const Rng rng2(seed2, state_stream(a.stream_key, a.state_keys, a.key0, b));
    const double* gl = a.s.gl + (size_t)b * V;
    const double* gu = a.s.gu + (size_t)b * V;
    const int Vr = p.Vr;
    const float lq = __log2f(1.0f - 1.0f / (float)Vr);
    for (int k = 0; k < nrw; ++k) {
      if (!(rdl(mut_v, k) & OVF)) continue;
      const int i = rc.i0 + wave + VARY_W * k;
      double x[NT];
      load_row(k, x);
      int pos = -1;
      for (int j = 0;; ++j) {
        const u32x4 w = rng2.draw((uint32_t)(i * MUT_J + j), (uint32_t)gen, TAG_MUT_MASK);
        pos += 1 + geo_gap(s_geo, Vr, w.x, lq);
        if (pos >= Vr) break;
        const int cp = s_cmap[pos];  // stored gene (-1: fixed, its mutation is the identity)
        if (cp < 0) continue;
        double xv = 0.0;
#pragma unroll
        for (int t = 0; t < NT; ++t)
          if (cp == lane + 64 * t) xv = x[t];
        if ((cp & 63) == lane) {
          xv = mutate_gene(xv, gl[MV_IDX(cp, V, CK_AT_BOUNDS)], gu[MV_IDX(cp, V, CK_AT_BOUNDS)],
                         (s_ginfo[cp] & 3) == 0, u53(w.y, w.z), a.eta);
#pragma unroll
          for (int t = 0; t < NT; ++t)
            if (cp == lane + 64 * t) x[t] = xv;
        }
      }
      finish_row(k, x);
    }
  }
  return orow_v;  // this lane's row destination (k_genc's phase 2 reuses it)
}

template <bool IDENT, int NT, bool SBX>
__global__ __launch_bounds__(VARY_T) void k_gen(int slot, int gen, int hist_row0, int rows_wg) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  gen_rows<IDENT, NT, SBX>(c_rows[slot], gen, hist_row0, rows_wg, smem);
}

// k_cons: the constraint program of each evaluated row (Constraints.evaluate numpy path +
// default_problem.py:93-97,128-129) -> f3 (+ G / history columns).  One workgroup = one
// state x a chunk of its rows, as k_gen; the row's genes (written by k_gen) are scattered
// into the wave's ML row buffer whose immutable features were written once, then each lane
// evaluates its (register-packed) ops.
// SLIM (k_genc, DProblem.slim): region S staged instead of region A, the lane ops' packed
// words loaded straight from the problem blob (see kernels.h).
template <bool FULL, bool IDENT, int NT, bool SLIM = false>
__device__ __forceinline__ void cons_rows(const RowsArgs& a, int hist_row0, int rows_wg,
                                          unsigned char* smem, bool have_dst = false,
                                          int dst_pre = 0) {
  const DProblem& p = a.p;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const RowChunk rc = row_chunk<CONS_W>(a.n, rows_wg, wave);
  const int b = MV_IDX(rc.b, a.total / a.n, CK_GEN_STATE), nrw = rc.nrw;
  const int V = p.V;
  const VaryOff o = vary_offsets(p);
  // row sources: mode 1 reads the children k_gen wrote (destination rows; k_genc passes the
  // destinations its phase 1 already loaded), mode 0 the input
  int src_v = 0, dst_v = 0;
  if (lane < nrw) {
    const int i = rc.i0 + wave + CONS_W * lane;
    dst_v = MV_IDX(have_dst ? dst_pre : (a.out_map ? a.out_map[(size_t)b * a.n + i] : i),
                   a.out_rows, CK_CONS_DST);
    src_v = MV_IDX(a.mode == 1 ? dst_v : i, a.mode == 1 ? a.out_rows : a.in_rows, CK_CONS_DST);
  }
  const double* gsrc = a.mode == 1 ? a.genes_out + (size_t)b * a.out_rows * V
                                   : a.genes_in + (size_t)b * a.in_rows * V;
  // Unconditional (index-clamped) loads: a per-element "if (g < V) load" makes hipcc branch
  // around each load and wait vmcnt(0) per element, serialising the row's round trips.
  auto load_row = [&](int k, double* x) {
    const size_t r0 = (size_t)rdl(src_v, MV_IDX(k, min(nrw, 64), CK_GEN_LANE)) * V;
    const long long lim = (long long)(a.mode == 1 ? a.out_rows : a.in_rows) * V;
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      const int g = lane + 64 * t;
      x[t] = gsrc[MV_IDX(r0 + (g < V ? g : V - 1), lim, CK_AT_SRC2)];
    }
  };
  // two rows in flight (as k_gen); the first two go out before the LDS staging so their
  // round trips overlap it
  double xa[NT], xb[NT];
  if (nrw > 0) load_row(0, xa);
  if (nrw > 1) load_row(1, xb);
  // LDS: [program region (A, or S when SLIM)][X: x_init][one row buffer per wave: the D
  // features, or SLIM the Dm stored mutable features (SlotRow)]
  const unsigned pa = SLIM ? o.s_end - o.s_at : o.a_end;
  const int n_lane = p.C - p.n_sumdiff;
  const int kops = min(OPS_REG, (n_lane + 63) >> 6);
  unsigned opw[OPS_REG];
  if (SLIM) {  // the packed words from HBM / L2, in flight across the staging
    const unsigned* gw = (const unsigned*)(p.vblob + o.s_opw);
#pragma unroll
    for (int k = 0; k < OPS_REG; ++k) {
      const int c = lane + 64 * k;
      const unsigned w = gw[c < n_lane ? c : 0];
      opw[k] = (k < kops && c < n_lane) ? w : 0u;
    }
    glds_copy<CONS_T>(smem, p.vblob + o.s_at, pa, wave, lane);
  } else {
    glds_copy<CONS_T>(smem, p.vblob, pa, wave, lane);
  }
  glds_copy<CONS_T>(smem + pa, a.s.sblob + (size_t)b * o.sb, o.x_end, wave, lane);
  int ginf[NT];
  {
    const int* gi = (const int*)(p.vblob + o.ginfo);
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      const int g = lane + 64 * t;
      const int w = gi[g < V ? g : V - 1];
      ginf[t] = g < V ? w : 0;
    }
  }
  __builtin_amdgcn_s_waitcnt(0);
  __syncthreads();
  if (MV_CLOCKS && a.gphase && tid == 0) a.gphase[(size_t)blockIdx.x * 8 + 4] = clock64();
  double* xrow = (double*)(smem + pa + o.x_end + wave * (SLIM ? o.rbs : o.rb));
  const double* s_xi = (const double*)(smem + pa + o.xi);
  if (!SLIM)
    for (int f = lane; f < p.D; f += 64) xrow[f] = s_xi[f];
  const SlotRow srow{xrow, s_xi, p.Dm};
  SlimOps so;
  OpTab tab;
  if (SLIM) {
    tab.code = nullptr;
    tab.arg = nullptr;
    tab.k = nullptr;
    tab.k1 = (const double*)(smem + (o.s_k - o.s_at));
    tab.sd = (const int4*)(smem + (o.s_sd - o.s_at));
    tab.col = (const int*)(smem + (o.s_col - o.s_at));
    tab.pool = (const int*)(smem + (o.s_pool - o.s_at));
  } else {
    tab.code = (const int*)(smem + o.opc);
    tab.arg = (const int4*)(smem + o.opa);
    tab.k = (const double2*)(smem + o.opk);
    tab.col = (const int*)(smem + o.ocol);
    tab.pool = (const int*)(smem + o.pool);
  }
  tab.C = p.C;
  tab.n_lane = n_lane;
  tab.tol = p.tol;
  if (a.hist) {
    tab.hlo = a.hist + (size_t)b * a.hist_rows * a.hist_w;
    tab.hhi = tab.hlo + (size_t)a.hist_rows * a.hist_w;
  }
  if (SLIM)
    slim_ops(tab, opw, kops, p.sd_reg != 0, xrow, s_xi, smem + (o.s_zero - o.s_at), p.Dm, lane,
             so);
  if (!SLIM) {
#pragma unroll
    for (int k = 0; k < OPS_REG; ++k) {
      const int c = lane + 64 * k;
      opw[k] = (k < kops && c < tab.n_lane) ? pack_op(tab, c) : 0u;
    }
  }
  auto do_row = [&](int k, const double* x) {
    const int i = MV_IDX(rc.i0 + wave + CONS_W * k, a.n, CK_CONS_DST);
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      if (lane + 64 * t < V) {
        if (SLIM)  // IDENT: stored gene c is mutable slot c
          xrow[lane + 64 * t] = x[t];
        else if (IDENT)
          xrow[(ginf[t] >> 17) & 0x7FFF] = x[t];
        else
          scatter_gene(p, xrow, ginf[t], x[t]);
      }
    }
    wave_sync();
    double* grow = a.G ? a.G + ((size_t)b * a.n + i) * p.C : nullptr;
    double* hrow = a.hist ? a.hist + ((size_t)b * a.hist_rows +
                                      MV_IDX(hist_row0 + i, a.hist_rows, CK_CONS_DST)) * a.hist_w
                          : nullptr;
    double* hc = (hrow && a.hist_w > 3) ? hrow + 3 : nullptr;
    double f3;
    if constexpr (SLIM)
      f3 = constraints_slim(tab, so, srow, lane, grow, hc);
    else
      f3 = constraints_regs<FULL>(tab, opw, kops, (const double*)xrow, lane, grow, hc);
    // The row's destination is read from lane k HERE, with every lane active: a readlane
    // of a lane that is inactive at that point returns an undefined value.  (Round 3 read
    // it inside the lane-0 branch below.  Whenever the compiler spilled dst_v, its reload
    // ran under that branch's one-lane EXEC mask, so lane k held a stale register value and
    // f3 was stored at a wild address.  That was the illegal-address fault of the
    // __launch_bounds__(VARY_T, 4) build, caught by the checks build as CK_AT_F3.)
    const int dst = rdl(dst_v, k);
    if (lane == 0) {
      if (a.F)
        a.F[(size_t)b * a.out_rows * 3 + MV_IDX((size_t)dst * 3 + 2, a.out_rows * 3, CK_AT_F3)] =
            f3;
      if (hrow) *MV_PTR(hrow + 2, tab.hlo, tab.hhi, CK_AT_HIST2) = f3;
    }
    wave_sync();  // the next row's scatter overwrites xrow
  };
  for (int k = 0; k < nrw; ++k) {  // xa: row k, xb: row k + 1 (in flight), rotated
    double x[NT];
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      x[t] = xa[t];
      xa[t] = xb[t];
    }
    if (k + 2 < nrw) load_row(k + 2, xb);
    do_row(k, x);
  }
}

template <bool FULL, bool IDENT, int NT>
__global__ __launch_bounds__(CONS_T) void k_cons(int slot, int hist_row0, int rows_wg) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  cons_rows<FULL, IDENT, NT>(c_rows[slot], hist_row0, rows_wg, smem);
}

// k_genc: k_gen and k_cons as two phases of ONE launch over the same row chunks (each wave
// evaluates the constraints of the rows it generated).  Phase 2 reads the children back
// from L2 (written a few microseconds earlier by the same workgroup) instead of HBM, and
// the chain loses a launch boundary; the phases run one after the other, so the kernel
// needs the larger of the two register and LDS footprints, not their sum (the fused row
// loop of round 2, k_rows, kept both phases' registers live: 208 VGPRs).
// k_genc's minimum waves per SIMD for the register allocator: 4 (128 VGPRs; the two-point
// instances up to 8 genes per lane spill a few registers to scratch) for a 4th resident
// workgroup per CU -- with the slim phase-2 LDS (~37 KiB) four fit.  Round 4 A/B on the
// botnet headline: 172.2 vs 161.5 M evals/s (k_genc 119.5 vs 137.6 us, one state group).
// SBX instances: 4 waves up to 5 genes per lane (botnet's compact layout: 140 -> 128
// VGPRs, 6 spilled; SBX option 124.0 -> 133.1 M evals/s, A/B on one box), the allocator's
// choice above that, like the 16-genes-per-lane instances (their register needs would spill
// heavily).  MV_GENC_WAVES / MV_GENC_SBX_WAVES (development builds) override the 4 / 1.
#ifndef MV_GENC_WAVES
#define MV_GENC_WAVES 4
#endif
#ifndef MV_GENC_SBX_WAVES
#define MV_GENC_SBX_WAVES 1
#endif
#define MV_GENC_BOUNDS                                                                  \
  __launch_bounds__(VARY_T, NT > 8 ? 1                                                 \
                                   : (SBX ? (NT <= 5 ? 4 : MV_GENC_SBX_WAVES) : MV_GENC_WAVES))
template <bool IDENT, int NT, bool SBX, bool SLIM>
__global__ MV_GENC_BOUNDS void k_genc(int slot, int gen, int hist_row0, int rows_wg) {
  static_assert(VARY_T == CONS_T, "k_genc runs both phases on the same waves");
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const RowsArgs& a = c_rows[slot];
  if (MV_CLOCKS && a.gphase && threadIdx.x == 0) {
    a.gphase[(size_t)blockIdx.x * 8 + 0] = clock64();
    a.gphase[(size_t)blockIdx.x * 8 + 6] = wall_clock64();
  }
  constexpr bool EARLY = SLIM && !SBX;  // the whole LDS staged at the start (genc_fused_lds)
  const int orow_v = gen_rows<IDENT, NT, SBX, true, EARLY>(a, gen, hist_row0, rows_wg, smem);
  if (MV_CLOCKS && a.gphase && threadIdx.x == 0) a.gphase[(size_t)blockIdx.x * 8 + 3] = clock64();
  // every child store has completed (vmcnt 0) before the barrier, so phase 2's loads of the
  // same rows see them; the phase-1 LDS images are dead and phase 2 stages over them.  Both
  // phases chunk the rows alike (VARY_T == CONS_T), so a lane's destination row is its own.
  if constexpr (!EARLY) {  // EARLY: the constraints ran inside phase 1's row loop
    __builtin_amdgcn_s_waitcnt(0);
    __syncthreads();
    cons_rows<false, IDENT, NT, SLIM>(a, hist_row0, rows_wg, smem, true, orow_v);
  }
  if (MV_CLOCKS && a.gphase && threadIdx.x == 0) {
    a.gphase[(size_t)blockIdx.x * 8 + 5] = clock64();
    a.gphase[(size_t)blockIdx.x * 8 + 7] = wall_clock64();
  }
}

// k_narrow: k_gen + k_cons for narrow rows, one lane per row (narrow.h).
template <int NV, bool FULL>
__global__ __launch_bounds__(NARROW_T) void k_narrow(int slot, int gen, int hist_row0) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  narrow_rows<NV, FULL>(c_rows[slot], gen, hist_row0, smem);
}

// Epilogue of a dense layer: + bias (per state for layer 0) and ReLU into the LDS tile.
template <int MAXCT, int RT>
__device__ __forceinline__ void dense_store(const floatx4 (&acc)[RT][MAXCT], int N,
                                            const float* __restrict__ bias,
                                            const float* __restrict__ bias_state,
                                            const int* row_state, float* __restrict__ out,
                                            int ldo, int wave, int lane) {
  const int nct = N >> 4;
  const int ka = lane >> 4, il = lane & 15;
#pragma unroll
  for (int c = 0; c < MAXCT; ++c) {
    const int ct = wave + c * 4;
    if (ct < nct) {
      const int col = ct * 16 + il;
#pragma unroll
      for (int rt = 0; rt < RT; ++rt) {
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

// ---------------------------------------------------------------------------------------
// Dense layer on MFMA: out[16 RT][N] = relu(in[16 RT][K] . W[K][N] + bias), K % 4 == 0,
// N % 16 == 0 (RT = 2: the 32-row tiles of k_mlp / k_predict; RT = 1: k_predict's 16-row
// tiles for inputs too wide for a 32-row LDS tile).  Software-pipelined: U k-steps of A
// (LDS) and B (global/L2) fragments are loaded before their RT*U MFMAs so the B-load
// latency is paid once per U steps.
template <int MAXCT, int RT = 2>
__device__ __forceinline__ void dense_mfma(const float* __restrict__ in, int ldi, int K,
                           const float* __restrict__ W, int N, const float* __restrict__ bias,
                           const float* __restrict__ bias_state, const int* row_state,
                           float* __restrict__ out, int ldo, int wave, int lane) {
  constexpr int U = MAXCT >= 4 ? 4 : 8;
  const int nct = N >> 4;
  floatx4 acc[RT][MAXCT];
#pragma unroll
  for (int c = 0; c < MAXCT; ++c)
#pragma unroll
    for (int r = 0; r < RT; ++r) acc[r][c] = floatx4{0.f, 0.f, 0.f, 0.f};
  const int ka = lane >> 4;
  const int il = lane & 15;
  const float* inr[RT];
#pragma unroll
  for (int r = 0; r < RT; ++r) inr[r] = in + (il + 16 * r) * ldi + ka;
  const float* wb = W + (size_t)ka * N + il;
  for (int k0 = 0; k0 < K; k0 += 4 * U) {
    float av[RT][U], bf[U][MAXCT];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int kk = k0 + 4 * u;
      const bool ok = kk < K;
#pragma unroll
      for (int r = 0; r < RT; ++r) av[r][u] = ok ? inr[r][kk] : 0.f;
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
#pragma unroll
          for (int r = 0; r < RT; ++r)
            acc[r][c] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[r][u], bf[u][c], acc[r][c], 0, 0, 0);
        }
      }
    }
  }
  dense_store<MAXCT, RT>(acc, N, bias, bias_state, row_state, out, ldo, wave, lane);
}

// dense_mfma in the bf16 perf mode: k-steps of 32 on v_mfma_f32_16x16x32_bf16, B operands
// one dwordx4 per lane and column tile of the packed Wb ([K/32][N][32]), A rows read as 8
// scalars (the tiles' odd row strides are not 16-B aligned) rounded to bf16.  Lane (il, ka)
// holds k = 32 s + 8 ka + j of step s; k past K contributes zeros.
template <int MAXCT, int RT = 2>
__device__ __forceinline__ void dense_mfma_bf(const float* __restrict__ in, int ldi, int K,
                                              const unsigned short* __restrict__ Wb, int N,
                                              const float* __restrict__ bias,
                                              const float* __restrict__ bias_state,
                                              const int* row_state, float* __restrict__ out,
                                              int ldo, int wave, int lane) {
  const int nct = N >> 4;
  floatx4 acc[RT][MAXCT];
#pragma unroll
  for (int c = 0; c < MAXCT; ++c)
#pragma unroll
    for (int r = 0; r < RT; ++r) acc[r][c] = floatx4{0.f, 0.f, 0.f, 0.f};
  const int ka = lane >> 4, il = lane & 15;
  const __bf16* W = (const __bf16*)Wb;
  const int nst = (K + 31) >> 5;
  for (int s = 0; s < nst; ++s) {
    const int k = 32 * s + 8 * ka;
    const bool on = k < K;
    bf16x8 av[RT];
#pragma unroll
    for (int r = 0; r < RT; ++r) {
      const float* ar = in + (il + 16 * r) * ldi + (on ? k : 0);
#pragma unroll
      for (int j = 0; j < 8; ++j) av[r][j] = (__bf16)(on ? ar[j] : 0.f);
    }
    bf16x8 bv[MAXCT];
#pragma unroll
    for (int c = 0; c < MAXCT; ++c) {
      const int ct = wave + c * 4 < nct ? wave + c * 4 : nct - 1;
      bv[c] = *(const bf16x8*)(W + ((size_t)s * N + ct * 16 + il) * 32 + 8 * ka);
    }
#pragma unroll
    for (int c = 0; c < MAXCT; ++c) {
      if (wave + c * 4 < nct) {
#pragma unroll
        for (int r = 0; r < RT; ++r)
          acc[r][c] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av[r], bv[c], acc[r][c], 0, 0, 0);
      }
    }
  }
  dense_store<MAXCT, RT>(acc, N, bias, bias_state, row_state, out, ldo, wave, lane);
}

// Final Dense + softmax for row t (one thread), weights staged in LDS: ws[k*nout + c], wsb[c].
// fp32 logits, Keras's fp32 softmax (rowops.h softmax_e).
__device__ __forceinline__ void last_layer_softmax(const float* in, int ldi, int K, int nout,
                                                   const float* ws, const float* wsb, int t,
                                                   float (&prob)[8]) {
  double z[8];
  double mx = -__builtin_inf();
#pragma unroll
  for (int c = 0; c < 8; ++c) {
    z[c] = 0.0;
    if (c < nout) {
      float s = 0.f;
      for (int k = 0; k < K; ++k) s = fmaf(in[t * ldi + k], ws[k * nout + c], s);
      z[c] = (double)(s + wsb[c]);
      mx = z[c] > mx ? z[c] : mx;
    }
  }
  softmax_all(z, nout, mx, prob);
}

__host__ __device__ inline int max_hidden(const int* dims, int n_layers) {
  int h = 16;
  for (int l = 1; l < n_layers; ++l) h = dims[l] > h ? dims[l] : h;
  return h;
}

// Dense chain over 32-row tiles of the fp32 ML rows -> f1.
template <int MAXCT, bool BF>
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
    if (BF)
      dense_mfma_bf<MAXCT>(in, ldi, K, p.Wb[l], N, p.bias[l], l == 0 ? a.s.bias1 : nullptr,
                           row_state, outb, N + 1, wave, lane);
    else
      dense_mfma<MAXCT>(in, ldi, K, p.W[l], N, p.bias[l], l == 0 ? a.s.bias1 : nullptr,
                        row_state, outb, N + 1, wave, lane);
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

// ---------------------------------------------------------------------------------------
// k_mlp2: the Dense-ReLU chain + final Dense/softmax over 64-row tiles (persistent
// workgroups), for hidden widths that are multiples of 16 and at most 128.
//
// Layer l multiplies the tile's [64][K_l] activations by W_l on v_mfma_f32_16x16x4_f32
// (exact fp32 products).  K is walked in groups of 16: lane (il, ka) of a wave holds
// k = 16 kg + 4 ka + s for the group's four MFMA k-steps s, so its A operands are one
// ds_read_b128 of a row and its B operands one dwordx4 of the packed weights
// Wp_l[kg][n][16].  Wave w owns output column tiles w, w + 4, ... and all four 16-row
// tiles, so each B load feeds four MFMAs.  Layer 0 streams the fp32 ML rows written by
// k_gen through a double-buffered LDS chunk of 64 k (register staged); hidden outputs go to
// an LDS ping-pong; the immutable features' contribution to layer 0 is the per-state bias
// bias1 (k_setup_states).  The last Dense + softmax is a dot product per row on the VALU.
template <int CJ, bool BF, bool DIRECT, bool CO>
#ifndef MV_MLP2_OCC
#define MV_MLP2_OCC 2  // fp32 gene-reading instance: minimum waves per SIMD
#endif
// fp32 instances reading the ML rows (LCLD: k_narrow's xml): two waves per SIMD (222 VGPRs,
// no AGPR spill; round 5: configs[2] 485.6 -> 498.6 M, configs[3] k_mlp2 16.4 -> 9.3 ms per
// generation, 335 -> 363 M; the allocator's choice before was one wave with 48 AGPRs)
#ifndef MV_MLP2_OCC_XML
#define MV_MLP2_OCC_XML 2
#endif
__global__ __launch_bounds__(256, BF ? (CJ == 1 ? 3 : 2) : (DIRECT && CJ == 1 ? MV_MLP2_OCC : MV_MLP2_OCC_XML)) void k_mlp2(int slot, int hist_row0) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const RowsArgs& a = c_rows[slot];
  const DProblem& p = a.p;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int il = lane & 15, ka = lane >> 4;
  const int nl = p.n_layers;
  const int K0 = p.Dm4, N0 = p.dims[1];
  const int K0dm = p.Dm;  // genes per row (= mutable features) on the xml_direct path
  const int hld = mlp2_hmax(p) + 4;
  const int Klast = p.dims[nl - 1], nout = p.dims[nl];
  int* rowst = (int*)smem;
  float* wl = (float*)(smem + 256);
  float* bl = wl + Klast * nout;
  float* A0 = (float*)(smem + mlp2_head(p));
  float* H = A0;  // hidden ping-pong, aliases the layer-0 chunks
  for (int q = tid; q < Klast * nout; q += 256) wl[q] = p.W[nl - 1][q];
  if (tid < nout) bl[tid] = p.bias[nl - 1][tid];
  // the hidden layers' biases in LDS too (their epilogues read one per output element: from
  // global memory each layer's epilogue waited out an L2 round trip)
  float* hbl = bl + nout;
  for (int l = 1, off = 0; l + 1 < nl; off += p.dims[l + 1], ++l)
    for (int q = tid; q < p.dims[l + 1]; q += 256) hbl[off + q] = p.bias[l][q];
  double* sS = (double*)(smem + mlp2_sc_off(p));
  double* sM = sS + K0;
  if (DIRECT)
    for (int q = tid; q < K0; q += 256) {
      sS[q] = p.mlS[q];
      sM[q] = p.mlM[q];
    }
  const int ntiles = (a.total + M2_ROWS - 1) / M2_ROWS;
  const int nkg0 = K0 >> 4;
  const int nch = (nkg0 + 3) >> 2;
  for (int tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
    const int r0 = tile * M2_ROWS;
    // the chunk staging registers are plain locals: captured by a lambda they were
    // address-taken and lived in scratch (64 B per lane per chunk, 41 MiB of WRITE_SIZE per
    // launch in the r01 PMC pass).  xml_direct stages the raw genes (gd) and converts them in
    // M2_CHUNK_STORE, after the current chunk's MFMAs: converting at load time made every
    // chunk wait for its loads before the MFMAs could hide them.
    float4 st0, st1, st2, st3;
    double gd[DIRECT ? 4 : 1][4];
    // xml_direct: the source rows are the tile's child genes (fp64) in the pool, ML-scaled
    // here exactly as k_gen would have, (float)(x * mlS + mlM); row u of this thread:
    // tile row (tid >> 4) + 16 u (CO: (tid >> 5) + 8 u, see the fp32 loop)
    constexpr int NGR = CO ? 8 : 4;
    const double* grow[NGR];
    if (DIRECT) {
#pragma unroll
      for (int u = 0; u < NGR; ++u) {
        const int rr0 = r0 + (CO ? (tid >> 5) + 8 * u : (tid >> 4) + 16 * u);
        const int rr = rr0 < a.total ? rr0 : a.total - 1;
        const int st = rr / a.n, i = rr - st * a.n;
        grow[u] = a.mode == 1
            ? a.genes_out + ((size_t)st * a.out_rows +
                             MV_IDX(a.out_map ? a.out_map[rr] : i, a.out_rows, CK_MLP_ROW)) * K0dm
            : a.genes_in + ((size_t)st * a.in_rows + MV_IDX(i, a.in_rows, CK_MLP_ROW)) * K0dm;
      }
    }
#define M2_CHUNK_LOAD(c)                                                                 \
  {                                                                                      \
    const int cc = (c);                                                                  \
    float4* sts[4] = {&st0, &st1, &st2, &st3};                                           \
    _Pragma("unroll") for (int u = 0; u < 4; ++u) {                                      \
      const int idx = tid + 256 * u;                                                     \
      const int row = idx >> 4, q = idx & 15;                                            \
      const int k = cc * 64 + 4 * q < K0 ? cc * 64 + 4 * q : K0 - 4;                     \
      if (DIRECT) {  /* raw genes; scaled in M2_CHUNK_STORE */                   \
        if (k + 3 < K0dm) {                                                              \
          const double2 g01 = *(const double2*)(grow[u] + k);                           \
          const double2 g23 = *(const double2*)(grow[u] + k + 2);                       \
          gd[u][0] = g01.x;                                                              \
          gd[u][1] = g01.y;                                                              \
          gd[u][2] = g23.x;                                                              \
          gd[u][3] = g23.y;                                                              \
        } else {                                                                         \
          _Pragma("unroll") for (int e = 0; e < 4; ++e) {                                \
            const int kk = k + e;                                                        \
            gd[u][e] = grow[u][kk < K0dm ? kk : K0dm - 1];                               \
          }                                                                              \
        }                                                                                \
      } else {                                                                           \
        const int rr = r0 + row < a.total ? r0 + row : a.total - 1;                      \
        *sts[u] = *(const float4*)(a.xml + (size_t)rr * K0 + k);                         \
      }                                                                                  \
    }                                                                                    \
  }
#define M2_CHUNK_STORE(buf, c)                                                           \
  {                                                                                      \
    const float4 vs[4] = {st0, st1, st2, st3};                                           \
    _Pragma("unroll") for (int u = 0; u < 4; ++u) {                                      \
      const int idx = tid + 256 * u;                                                     \
      const int row = idx >> 4, q = idx & 15;                                            \
      float4 v = vs[u];                                                                  \
      if (DIRECT) {                                                                \
        const int kq = (c) * 64 + 4 * q;                                                 \
        const int k = kq < K0 ? kq : K0 - 4;                                             \
        float v4[4];                                                                     \
        _Pragma("unroll") for (int e = 0; e < 4; ++e) {                                  \
          const int kk = k + e;                                                          \
          v4[e] = kk < K0dm ? (float)(gd[u][e] * sS[kk] + sM[kk]) : 0.f;                 \
        }                                                                                \
        v = make_float4(v4[0], v4[1], v4[2], v4[3]);                                     \
      }                                                                                  \
      *(float4*)(A0 + (buf) * M2_ROWS * M2_ALD + row * M2_ALD + 4 * q) = v;               \
    }                                                                                    \
  }
    const bool ph = MV_CLOCKS && a.mphase && tid == 0 && tile == (int)blockIdx.x;
    long long* phq = a.mphase + (size_t)blockIdx.x * 16;
    if (ph) {
      phq[0] = clock64();
      phq[6] = wall_clock64();
    }
    floatx4 acc[CJ][4];
#pragma unroll
    for (int cj = 0; cj < CJ; ++cj)
#pragma unroll
      for (int rt = 0; rt < 4; ++rt) acc[cj][rt] = floatx4{0.f, 0.f, 0.f, 0.f};
    float b1[CJ][4][4];    // fp32 path: bias1 of the layer-0 outputs this lane writes
    int fin_mc = 0, fin_orow = 0;  // fp32 path, tid < 64: min_class and output row of row tid
    if constexpr (BF) {
      M2_CHUNK_LOAD(0)
      if (ph) phq[1] = clock64();
      __syncthreads();  // the previous tile's readers of rowst / A0 / H are done
      if (tid < M2_ROWS) rowst[tid] = r0 + tid < a.total ? (r0 + tid) / a.n : -1;
      M2_CHUNK_STORE(0, 0)
      __syncthreads();
      if (ph) phq[2] = clock64();
      for (int c = 0; c < nch; ++c) {
        if (c + 1 < nch) M2_CHUNK_LOAD(c + 1)
        const int ng = min(4, nkg0 - 4 * c);
        if (BF)
          mlp2_layer_bf<CJ>(A0 + (c & 1) * M2_ROWS * M2_ALD, M2_ALD, 16 * ng, p.Wb[0], 2 * c, N0,
                            acc, tile_map(N0 >> 4, wave), il, ka);
        else
          mlp2_layer<CJ>(A0 + (c & 1) * M2_ROWS * M2_ALD, M2_ALD,
                         p.Wp[0] + (size_t)4 * c * N0 * 16, ng, N0, acc, tile_map(N0 >> 4, wave),
                         il, ka);
        if (c + 1 < nch) M2_CHUNK_STORE((c + 1) & 1, c + 1)
        __syncthreads();
      }
    } else {
      // fp32 layer 0, software-pipelined with one register set per operand.  Iteration c
      // issues the source rows of chunk c + 1, runs chunk c's MFMAs on W(c) -- loaded at the
      // end of iteration c - 1, so OLDER than those rows, and since vmcnt retires in order
      // the MFMAs' wait leaves the rows in flight (the previous version loaded each k-group's
      // weights after the rows, so its first MFMA waited out the rows' HBM round trip: ~10 k
      // cycles per 2 k-cycle chunk, MV_MLP_PHASES) -- then loads W(c + 1), converts chunk
      // c + 1 into the other LDS buffer (waiting for its rows; only W(c + 1) is younger) and
      // ends on an LDS-only barrier.  Loads use clamped indices, never a condition (a
      // conditional load makes hipcc wait vmcnt(0) where the paths join).
      const TileMap m0 = tile_map(N0 >> 4, wave);
      const int nct0 = N0 >> 4;
      const float* Wp0 = p.Wp[0];
      const int q = tid & 15;  // this thread's 4-k piece of every staged row
      float4 wr[4][CJ];
      double gd[DIRECT ? 4 : 1][4];
      float4 st[DIRECT ? 1 : 4];
      // CO (genes per row even, so rows start 16-B aligned): lane-contiguous staging --
      // thread (row (tid >> 5) + 8 u, piece p = tid & 31) loads the 16 B of genes
      // 2p, 2p + 1 of the chunk, so a wave's load covers two rows' 512 B without gaps
      // (the 4-genes-per-thread mapping touched every 128-B line with four dwordx2 loads)
      const int pc = tid & 31;
      uint4 gv[CO ? 8 : 1];
#define M2F_LOADW(c)                                                                      \
  {                                                                                       \
    _Pragma("unroll") for (int g = 0; g < 4; ++g) {                                       \
      const int kg = 4 * (c) + g < nkg0 ? 4 * (c) + g : nkg0 - 1;                         \
      _Pragma("unroll") for (int cj = 0; cj < CJ; ++cj) {                                 \
        const int ct = m0.cb + 4 * cj < nct0 ? m0.cb + 4 * cj : nct0 - 1;                 \
        wr[g][cj] = *(const float4*)(Wp0 + ((size_t)kg * N0 + ct * 16 + il) * 16 + 4 * ka); \
      }                                                                                   \
    }                                                                                     \
  }
#define M2F_LOADG(c)                                                                      \
  if constexpr (CO) {                                                                     \
    const int cc = (c) < nch ? (c) : nch - 1;                                             \
    const int k = cc * 64 + 2 * pc + 1 < K0dm ? cc * 64 + 2 * pc : K0dm - 2;              \
    _Pragma("unroll") for (int u = 0; u < 8; ++u)                                         \
      gv[CO ? u : 0] = *(const uint4*)(grow[u] + k);                                      \
  } else {                                                                                \
    const int cc = (c) < nch ? (c) : nch - 1;                                             \
    const int k = cc * 64 + 4 * q < K0 ? cc * 64 + 4 * q : K0 - 4;                        \
    _Pragma("unroll") for (int u = 0; u < 4; ++u) {                                       \
      if (DIRECT) {                                                                       \
        _Pragma("unroll") for (int e = 0; e < 4; ++e) {                                   \
          const int kk = k + e < K0dm ? k + e : K0dm - 1;                                 \
          gd[DIRECT ? u : 0][e] = grow[u][kk];                                            \
        }                                                                                 \
      } else {                                                                            \
        const int row = (tid >> 4) + 16 * u;                                              \
        const int rr = r0 + row < a.total ? r0 + row : a.total - 1;                       \
        st[DIRECT ? 0 : u] = *(const float4*)(a.xml + (size_t)rr * K0 + k);              \
      }                                                                                   \
    }                                                                                     \
  }
#define M2F_STORE(c)                                                                      \
  if constexpr (CO) {                                                                     \
    const int k = (c) * 64 + 2 * pc;                                                      \
    float* Ab = A0 + ((c) & 1) * M2_ROWS * M2_ALD;                                        \
    const int k0 = k < K0 ? k : K0 - 1, k1 = k + 1 < K0 ? k + 1 : K0 - 1;                 \
    const double sc0 = sS[k0], sc1 = sS[k1], mn0 = sM[k0], mn1 = sM[k1];                  \
    _Pragma("unroll") for (int u = 0; u < 8; ++u) {                                       \
      const int row = (tid >> 5) + 8 * u;                                                 \
      const uint4 w = gv[CO ? u : 0];                                                     \
      const double d0 = __hiloint2double((int)w.y, (int)w.x);                             \
      const double d1 = __hiloint2double((int)w.w, (int)w.z);                             \
      float2 v;                                                                           \
      v.x = k < K0dm ? (float)(d0 * sc0 + mn0) : 0.f;                                     \
      v.y = k + 1 < K0dm ? (float)(d1 * sc1 + mn1) : 0.f;                                 \
      *(float2*)(Ab + row * M2_ALD + 2 * pc) = v;                                         \
    }                                                                                     \
  } else {                                                                                \
    const int kq = (c) * 64 + 4 * q;                                                      \
    const int k = kq < K0 ? kq : K0 - 4;                                                  \
    float* Ab = A0 + ((c) & 1) * M2_ROWS * M2_ALD;                                        \
    double sc[4], mn[4];                                                                  \
    if (DIRECT) {                                                                         \
      _Pragma("unroll") for (int e = 0; e < 4; ++e) {                                     \
        sc[e] = sS[k + e];                                                                \
        mn[e] = sM[k + e];                                                                \
      }                                                                                   \
    }                                                                                     \
    _Pragma("unroll") for (int u = 0; u < 4; ++u) {                                       \
      const int row = (tid >> 4) + 16 * u;                                                \
      float4 v;                                                                           \
      if (DIRECT) {                                                                       \
        float v4[4];                                                                      \
        _Pragma("unroll") for (int e = 0; e < 4; ++e)                                     \
          v4[e] = k + e < K0dm ? (float)(gd[DIRECT ? u : 0][e] * sc[e] + mn[e]) : 0.f;    \
        v = make_float4(v4[0], v4[1], v4[2], v4[3]);                                      \
      } else {                                                                            \
        v = st[DIRECT ? 0 : u];                                                           \
      }                                                                                   \
      *(float4*)(Ab + row * M2_ALD + 4 * q) = v;                                          \
    }                                                                                     \
  }
#define M2F_MARK(c, k) \
  if (ph && (c) == 2) phq[k] = clock64();
      M2F_LOADG(0)
      M2F_LOADW(0)
      if (ph) phq[1] = clock64();
      // the previous tile's readers of rowst / A0 / H are done (LDS only: no vmcnt(0))
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      if (tid < M2_ROWS) rowst[tid] = r0 + tid < a.total ? (r0 + tid) / a.n : -1;
      M2F_STORE(0)
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      // the layer-0 epilogue's per-state bias (bias1) and the final phase's per-row scalars,
      // loaded now (unconditionally) so that their latency hides under the chunk loop
#pragma unroll
      for (int cj = 0; cj < CJ; ++cj) {
        const int ct = m0.cb + 4 * cj < nct0 ? m0.cb + 4 * cj : nct0 - 1;
#pragma unroll
        for (int rt = 0; rt < 4; ++rt)
#pragma unroll
          for (int jj = 0; jj < 4; ++jj) {
            const int row = (m0.rt0 + (rt < m0.nrt ? rt : 0)) * 16 + ka * 4 + jj;
            const int st0 = rowst[row];
            b1[cj][rt][jj] = a.s.bias1[(size_t)(st0 < 0 ? 0 : st0) * N0 + ct * 16 + il];
          }
      }
      {
        const int rr = r0 + (tid & 63) < a.total ? r0 + (tid & 63) : a.total - 1;
        const int stc = rr / a.n;
        fin_mc = a.s.min_class[stc];
        // out_map may be NULL (mode 0): read a valid dummy instead of branching
        const int* om = a.out_map ? a.out_map : a.s.min_class;
        const int ov = om[a.out_map ? rr : stc];
        fin_orow = MV_IDX(a.out_map ? ov : rr - stc * a.n, a.out_rows, CK_MLP_OUT);
      }
      if (ph) phq[2] = clock64();
      for (int c = 0; c < nch; ++c) {
        M2F_MARK(c, 8)
        M2F_LOADG(c + 1)
        M2F_MARK(c, 9)
        {
          const int ng = min(4, nkg0 - 4 * c);
          const float* Ab = A0 + (c & 1) * M2_ROWS * M2_ALD;
#pragma unroll
          for (int g = 0; g < 4; ++g) {
            if (g < ng) {
              float4 af[4];
#pragma unroll
              for (int rt = 0; rt < 4; ++rt) {
                const int r = m0.rt0 + (rt < m0.nrt ? rt : 0);
                af[rt] = *(const float4*)(Ab + (r * 16 + il) * M2_ALD + g * 16 + 4 * ka);
              }
              mfma_k4<CJ>(af, wr[g], acc, m0.cb, nct0, m0.nrt);
            }
          }
        }
        M2F_MARK(c, 10)
        M2F_LOADW(c + 1)
        if (c + 1 < nch) {
          M2F_STORE(c + 1)
        }
        M2F_MARK(c, 11)
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        M2F_MARK(c, 12)
      }
#undef M2F_LOADW
#undef M2F_LOADG
#undef M2F_STORE
#undef M2F_MARK
      __syncthreads();  // the trailing (clamped, unused) prefetches land before H reuses A0
    }
#undef M2_CHUNK_LOAD
#undef M2_CHUNK_STORE
    if (ph) phq[3] = clock64();
    // hidden layers: layer l writes H[l & 1]
    for (int l = 0, hoff = 0; l + 1 < nl; hoff += l > 0 ? p.dims[l + 1] : 0, ++l) {
      const int N = p.dims[l + 1];
      const TileMap m = tile_map(N >> 4, wave);
      if (l > 0) {
#pragma unroll
        for (int cj = 0; cj < CJ; ++cj)
#pragma unroll
          for (int rt = 0; rt < 4; ++rt) acc[cj][rt] = floatx4{0.f, 0.f, 0.f, 0.f};
        if (BF)
          mlp2_layer_bf<CJ>(H + ((l - 1) & 1) * M2_ROWS * hld, hld, p.dims[l], p.Wb[l], 0, N,
                            acc, m, il, ka);
        else
          mlp2_layer<CJ>(H + ((l - 1) & 1) * M2_ROWS * hld, hld, p.Wp[l], p.dims[l] >> 4, N,
                         acc, m, il, ka);
      }
      float* out = H + (l & 1) * M2_ROWS * hld;
#pragma unroll
      for (int cj = 0; cj < CJ; ++cj) {
        const int ct = m.cb + 4 * cj;
        if (ct < (N >> 4)) {
          const int col = ct * 16 + il;
#pragma unroll
          for (int rt = 0; rt < 4; ++rt) {
            if (rt >= m.nrt) continue;
#pragma unroll
            for (int j = 0; j < 4; ++j) {
              const int row = (m.rt0 + rt) * 16 + ka * 4 + j;
              float bv;
              if (l == 0) {
                if constexpr (BF) {
                  const int s = rowst[row];
                  bv = a.s.bias1[(size_t)(s < 0 ? 0 : s) * N0 + col];
                } else {
                  bv = b1[cj][rt][j];
                }
              } else {
                bv = hbl[hoff + col];
              }
              const float v = acc[cj][rt][j] + bv;
              out[row * hld + col] = v > 0.f ? v : 0.f;
            }
          }
        }
      }
      __syncthreads();
    }
    if (ph) phq[4] = clock64();
    // final Dense + softmax (classifier.py:23-29) -> f1.  Wave w sums the k quarter
    // [w Klast/4, (w+1) Klast/4) of every row (lane = row), wave 0 combines and normalises.
    float* part = mlp2_part_inplace(p) ? H + ((nl - 1) & 1) * M2_ROWS * hld
                                       : A0 + mlp2_region_floats(p);
    {
      const int kq = Klast >> 2;
      const float* ir = H + ((nl - 2) & 1) * M2_ROWS * hld + lane * hld + wave * kq;
      const float* wq = wl + wave * kq * nout;
      float ps[8];
#pragma unroll
      for (int c = 0; c < 8; ++c) ps[c] = 0.f;
      for (int k = 0; k < kq; k += 4) {
        const float4 v = *(const float4*)(ir + k);
#pragma unroll
        for (int c = 0; c < 8; ++c) {
          if (c < nout) {
            ps[c] = fmaf(v.x, wq[k * nout + c], ps[c]);
            ps[c] = fmaf(v.y, wq[(k + 1) * nout + c], ps[c]);
            ps[c] = fmaf(v.z, wq[(k + 2) * nout + c], ps[c]);
            ps[c] = fmaf(v.w, wq[(k + 3) * nout + c], ps[c]);
          }
        }
      }
#pragma unroll
      for (int c = 0; c < 8; ++c)
        if (c < nout) part[(wave * M2_ROWS + lane) * nout + c] = ps[c];
    }
    __syncthreads();
    if (tid < M2_ROWS) {
      const int s = rowst[tid];
      if (s >= 0) {
        double z[8];
        double mx = -__builtin_inf();
#pragma unroll
        for (int c = 0; c < 8; ++c) {
          z[c] = 0.0;
          if (c < nout) {
            const float* q = part + tid * nout + c;
            z[c] = (double)((((q[0] + q[M2_ROWS * nout]) + q[2 * M2_ROWS * nout]) +
                             q[3 * M2_ROWS * nout]) + bl[c]);
            mx = z[c] > mx ? z[c] : mx;
          }
        }
        const double f1 = softmax_pick(z, nout, mx, BF ? a.s.min_class[s] : fin_mc);
        const int i = r0 + tid - s * a.n;
        if (a.F) {
          const int orow = BF ? MV_IDX(a.out_map ? a.out_map[(size_t)s * a.n + i] : i, a.out_rows,
                                       CK_MLP_OUT)
                              : fin_orow;
          a.F[((size_t)MV_IDX(s, a.total / a.n, CK_MLP_OUT) * a.out_rows + orow) * 3] = f1;
        }
        if (a.hist)
          a.hist[((size_t)s * a.hist_rows + MV_IDX(hist_row0 + i, a.hist_rows, CK_MLP_OUT)) *
                 a.hist_w] = f1;
      }
    }
    if (ph) {
      phq[5] = clock64();
      phq[7] = wall_clock64();
    }
  }
}

// ---------------------------------------------------------------------------------------
// k_mlpr: the fp32 classifier of the gene-reading (xml_direct) path for hidden widths up to
// 64 -- the botnet headline's 312-64-64-32-2 chain -- with every wave on its own RW x 16 rows
// and no LDS tile, no barrier in the row loop.  Each Dense layer runs transposed,
// out^T = W^T . in^T, on v_mfma_f32_16x16x4f32: the weights are the A operand (lane (il, ka)
// = output column 16 nb + il, k = 16 kg + 4 ka + s: one dwordx4 of the packed Wp per k-group
// and column block, from L2), the rows the B operand (lane (il, ka) = row il, the same k), so
// column block nb's accumulator holds outputs 16 nb + 4 ka + j of row il -- exactly the next
// layer's B operand for k-group nb: the hidden layers never leave the registers.  Layer 0's B
// operands are the row's genes scaled as k_gen would, (float)(x * mlS + mlM), 32 B per lane
// per k-group from HBM, one k-group ahead in two alternating operand sets.  Every output sums
// the same products in the same k order as k_mlp2 (k-group, then s; the MFMA's k slot is ka
// either way) and the last Dense keeps k_mlp2's four-quarter order, so f1 is bit-identical
// (oracle/device_order.f1_device_order).  Replaces k_mlp2's 64-row tiles, whose layer-0 chunk
// loop waited on its LDS staging (~64 k cycles per tile against ~14 k of MFMA issue).
#ifndef MV_MLPR_OCC
#define MV_MLPR_OCC 3  // waves per SIMD of the 16-row instance (<= 168 registers)
#endif
// LDS: the ML scaler at the mutable features (mlS, mlM), the final Dense layer, the hidden
// layers' packed weights and biases (read per tile: from L2 each hidden layer waited out a
// ~3 k-cycle round trip, MV_MLP_PHASES "hidden" 16.9 k cycles per tile), then per wave its
// tile's bias1 rows (landed by LDS DMA while layer 0 runs) and its last-hidden-layer rows.
struct MlprLds {
  unsigned wl, hw, hb, b1, hs, wst, total;
  int hld;  // fp32 row stride of a wave's last-hidden-layer rows
};
__host__ __device__ inline MlprLds mlpr_lds(const DProblem& p, int rw) {
  const int nl = p.n_layers;
  MlprLds L{};
  L.wl = (unsigned)p.Dm4 * 16;  // mlS, mlM
  L.hld = p.dims[nl - 1] + 4;
  L.hw = L.wl + (((unsigned)(p.dims[nl - 1] * p.dims[nl] + p.dims[nl]) * 4 + 15) & ~15u);
  unsigned w = 0, b = 0;
  for (int l = 1; l + 1 < nl; ++l) {
    w += (unsigned)(p.dims[l] * p.dims[l + 1]);
    b += (unsigned)p.dims[l + 1];
  }
  L.hb = L.hw + w * 4;
  // a wave's bias1 rows are in registers before its last-hidden-layer rows are written: one
  // per-wave region serves both
  L.b1 = L.hb + ((b * 4 + 15) & ~15u);
  L.hs = L.b1;
  L.wst = (unsigned)rw * 4 * 1024;
  const unsigned hsz = (unsigned)(rw * 16 * L.hld) * 4;
  L.wst = L.wst > hsz ? L.wst : hsz;
  L.total = L.b1 + 4u * L.wst;
  return L;
}
// The shapes k_mlpr takes: IDENT gene rows (xml_direct) of an even gene count (16-B aligned
// gene pairs), fp32, every MFMA layer's width a multiple of 16 and at most 64, K0 a multiple
// of 16, at most 8 classes.
__host__ __device__ inline bool mlpr_ok(const DProblem& p) {
  // the fp32 ML-row path (LCLD: k_narrow's xml rows, zero-padded to Dm4) takes the XML
  // instance: the same tiles with the rows' fp32 values as layer 0's operands
  if (p.mlp_bf16 || !p.mlp2 || p.n_layers < 2 || (p.xml_direct && ((p.Dm & 1) || p.Dm < 2)))
    return false;
  for (int l = 0; l + 1 < p.n_layers; ++l)
    if (!p.Wp[l]) return false;
  for (int l = 1; l < p.n_layers; ++l)
    if (p.dims[l] % 16 || p.dims[l] > 64) return false;
  return p.Dm4 % 16 == 0 && p.dims[p.n_layers] <= 8 && mlpr_lds(p, 2).total <= 96 * 1024;
}

template <int RW, int NO, bool XML = false>
__global__ __launch_bounds__(256, RW == 1 ? MV_MLPR_OCC : 2) void k_mlpr(int slot, int hist_row0) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const RowsArgs& a = c_rows[slot];
  const DProblem& p = a.p;
  constexpr int TR = 16 * RW;  // rows per wave tile
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int il = lane & 15, ka = lane >> 4;
  const int nl = p.n_layers;
  const int K0 = p.Dm4, N0 = p.dims[1], Dm = p.Dm;
  const int Klast = p.dims[nl - 1], nout = p.dims[nl];
  const MlprLds L = mlpr_lds(p, RW);
  const int hld = L.hld;
  double* sS = (double*)smem;
  double* sM = sS + K0;
  float* wl = (float*)(smem + L.wl);
  float* bl = wl + Klast * nout;
  float* hs = (float*)(smem + L.hs + wave * L.wst);
  if (!XML)
    for (int q = tid; q < K0; q += 256) {
      sS[q] = p.mlS[q];
      sM[q] = p.mlM[q];
    }
  for (int q = tid; q < Klast * nout; q += 256) wl[q] = p.W[nl - 1][q];
  if (tid < nout) bl[tid] = p.bias[nl - 1][tid];
  float* hw = (float*)(smem + L.hw);
  float* hbs = (float*)(smem + L.hb);
  for (int l = 1, wo = 0, bo = 0; l + 1 < nl; wo += p.dims[l] * p.dims[l + 1], bo += p.dims[l + 1], ++l) {
    for (int q = tid; q < (p.dims[l] * p.dims[l + 1]) >> 2; q += 256)
      *(float4*)(hw + wo + 4 * q) = *(const float4*)(p.Wp[l] + 4 * q);
    for (int q = tid; q < p.dims[l + 1]; q += 256) hbs[bo + q] = p.bias[l][q];
  }
  unsigned char* b1w = smem + L.b1 + wave * L.wst;
  __syncthreads();
  const int ntiles = (a.total + TR - 1) / TR;
  const int nkg0 = K0 >> 4, nb0 = N0 >> 4;
  const float* Wp0 = p.Wp[0];
  for (int tile = blockIdx.x * 4 + wave; tile < ntiles; tile += gridDim.x * 4) {
    const int r0 = tile * TR;
    // development phase clocks (MV_CLOCKS build, MV_MLP_PHASES=1): wave 0's first tile
    const bool ph = MV_CLOCKS && a.mphase && tid == 0 && tile == (int)blockIdx.x * 4;
    long long* phq = a.mphase + (size_t)blockIdx.x * 16;
    if (ph) {
      phq[0] = clock64();
      phq[6] = wall_clock64();
    }
    const double* grow[RW];
    const float* xrw[RW];  // XML: the rows' fp32 ML values (xml [total][K0])
    int rst[RW];
#pragma unroll
    for (int rt = 0; rt < RW; ++rt) {
      const int rr0 = r0 + 16 * rt + il;
      const int rr = rr0 < a.total ? rr0 : a.total - 1;
      const int st = rr / a.n, i = rr - st * a.n;
      rst[rt] = st;
      xrw[rt] = a.xml + (size_t)rr * K0;
      if (!XML) grow[rt] = a.mode == 1
          ? a.genes_out + ((size_t)st * a.out_rows +
                           MV_IDX(a.out_map ? a.out_map[rr] : i, a.out_rows, CK_MLP_ROW)) * Dm
          : a.genes_in + ((size_t)st * a.in_rows + MV_IDX(i, a.in_rows, CK_MLP_ROW)) * Dm;
    }
    // the epilogue's per-state bias1 rows (immutable features folded) by LDS DMA: lane l's
    // 16 B of block (rt, nb) land at b1w + (4 rt + nb) KiB + 16 l; the oldest loads of the
    // tile, so layer 0's waits retire them
#pragma unroll
    for (int rt = 0; rt < RW; ++rt)
#pragma unroll
      for (int nb = 0; nb < 4; ++nb) {
        const int nbc = nb < nb0 ? nb : nb0 - 1;
        __builtin_amdgcn_global_load_lds(a.s.bias1 + (size_t)rst[rt] * N0 + 16 * nbc + 4 * ka,
                                         b1w + (4 * rt + nb) * 1024, 16, 0, 0);
      }
    floatx4 acc[RW][4];
#pragma unroll
    for (int rt = 0; rt < RW; ++rt)
#pragma unroll
      for (int nb = 0; nb < 4; ++nb) acc[rt][nb] = floatx4{0.f, 0.f, 0.f, 0.f};
    // operands: the four column blocks' weights in two alternating sets (L2 hits, one k-group
    // ahead), the RW rows' four genes in a ring of four sets (HBM, three k-groups ahead: with
    // one k-group in flight per wave the launch ran at the latency of a round trip per
    // k-group, ~2.5 us, MV_MLPR A/B v1).  Each step issues the next weights BEFORE its genes:
    // vmcnt retires in order, so waiting for weights issued after the genes of later steps
    // would wait for those genes too.
    float4 wA[4], wB[4];
    double2 g0[RW][2], g1[RW][2], g2[RW][2], g3[RW][2];
    float4 f0[RW], f1[RW], f2[RW], f3[RW];  // XML
#define MR_LOADW(kg, w)                                                                    \
  {                                                                                        \
    const int kgc = (kg) < nkg0 ? (kg) : nkg0 - 1;                                         \
    _Pragma("unroll") for (int nb = 0; nb < 4; ++nb) {                                     \
      const int nbc = nb < nb0 ? nb : nb0 - 1;                                             \
      w[nb] = *(const float4*)(Wp0 + ((size_t)kgc * N0 + nbc * 16 + il) * 16 + 4 * ka);    \
    }                                                                                      \
  }
#define MR_LOADG(kg, g, f)                                                                 \
  {                                                                                        \
    const int kgc = (kg) < nkg0 ? (kg) : nkg0 - 1;                                         \
    const int k = 16 * kgc + 4 * ka;                                                       \
    if constexpr (XML) {                                                                   \
      _Pragma("unroll") for (int rt = 0; rt < RW; ++rt)                                    \
        f[rt] = *(const float4*)(xrw[rt] + k);                                             \
    } else {                                                                               \
      const int k01 = k + 1 < Dm ? k : Dm - 2, k23 = k + 3 < Dm ? k + 2 : Dm - 2;          \
      _Pragma("unroll") for (int rt = 0; rt < RW; ++rt) {                                  \
        g[rt][0] = *(const double2*)(grow[rt] + k01);                                      \
        g[rt][1] = *(const double2*)(grow[rt] + k23);                                      \
      }                                                                                    \
    }                                                                                      \
  }
#define MR_STEP(kg, w, g, f)                                                               \
  {                                                                                        \
    const int kgc = (kg) < nkg0 ? (kg) : nkg0 - 1;                                         \
    const int k = 16 * kgc + 4 * ka;                                                       \
    /* k >= Dm (the zero padding to K0) and the k-groups past nkg0: +0 */                  \
    unsigned msk[4];                                                                       \
    _Pragma("unroll") for (int e = 0; e < 4; ++e)                                          \
      msk[e] = (k + e < Dm && (kg) < nkg0) ? 0xFFFFFFFFu : 0u;                             \
    float xb[RW][4];                                                                       \
    if constexpr (XML) {                                                                   \
      _Pragma("unroll") for (int rt = 0; rt < RW; ++rt)                                    \
        _Pragma("unroll") for (int e = 0; e < 4; ++e)                                      \
          xb[rt][e] = __uint_as_float(__float_as_uint(f4c(f[rt], e)) & msk[e]);            \
    } else {                                                                               \
      const double2 s01 = *(const double2*)(sS + k), s23 = *(const double2*)(sS + k + 2);  \
      const double2 m01 = *(const double2*)(sM + k), m23 = *(const double2*)(sM + k + 2);  \
      const double sc[4] = {s01.x, s01.y, s23.x, s23.y}, mn[4] = {m01.x, m01.y, m23.x, m23.y}; \
      _Pragma("unroll") for (int rt = 0; rt < RW; ++rt) {                                  \
        const double gv[4] = {g[rt][0].x, g[rt][0].y, g[rt][1].x, g[rt][1].y};             \
        _Pragma("unroll") for (int e = 0; e < 4; ++e)                                      \
          xb[rt][e] = __uint_as_float(__float_as_uint((float)(gv[e] * sc[e] + mn[e])) & msk[e]); \
      }                                                                                    \
    }                                                                                      \
    _Pragma("unroll") for (int s = 0; s < 4; ++s)                                          \
      _Pragma("unroll") for (int nb = 0; nb < 4; ++nb)                                     \
        _Pragma("unroll") for (int rt = 0; rt < RW; ++rt)                                  \
          acc[rt][nb] = __builtin_amdgcn_mfma_f32_16x16x4f32(f4c(w[nb], s), xb[rt][s],     \
                                                             acc[rt][nb], 0, 0, 0);        \
  }
    // the empty asm statements with a memory clobber keep each prefetch where it is written:
    // without them instcombine folds phi(load, load) into one load at the loop top and the
    // scheduler sinks every load next to its first use (vmcnt(0) before each MFMA group)
    const int nkg0e = (nkg0 + 3) & ~3;
    MR_LOADW(0, wA)
    MR_LOADG(0, g0, f0)
    MR_LOADG(1, g1, f1)
    MR_LOADG(2, g2, f2)
    if (ph) phq[1] = clock64();
#pragma unroll 1
    for (int kg = 0; kg < nkg0e; kg += 4) {
      MR_LOADW(kg + 1, wB)
      MR_LOADG(kg + 3, g3, f3)
      asm volatile("" ::: "memory");
      MR_STEP(kg, wA, g0, f0)
      MR_LOADW(kg + 2, wA)
      MR_LOADG(kg + 4, g0, f0)
      asm volatile("" ::: "memory");
      MR_STEP(kg + 1, wB, g1, f1)
      MR_LOADW(kg + 3, wB)
      MR_LOADG(kg + 5, g1, f1)
      asm volatile("" ::: "memory");
      MR_STEP(kg + 2, wA, g2, f2)
      MR_LOADW(kg + 4, wA)
      MR_LOADG(kg + 6, g2, f2)
      asm volatile("" ::: "memory");
      MR_STEP(kg + 3, wB, g3, f3)
      if (ph && kg == 0) phq[2] = clock64();
    }
    if (ph) phq[3] = clock64();
    // bias1 landed (its DMA is older than every layer-0 load still in flight)
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    float4 b1v[RW][4];
#pragma unroll
    for (int rt = 0; rt < RW; ++rt)
#pragma unroll
      for (int nb = 0; nb < 4; ++nb)
        b1v[rt][nb] = *(const float4*)(b1w + (4 * rt + nb) * 1024 + 16 * lane);
#undef MR_LOADW
#undef MR_LOADG
#undef MR_STEP
    // layer-0 epilogue: + bias1, ReLU
    floatx4 h[RW][4];
#pragma unroll
    for (int rt = 0; rt < RW; ++rt)
#pragma unroll
      for (int nb = 0; nb < 4; ++nb) {
        const float4 b = b1v[rt][nb];
        const float bv[4] = {b.x, b.y, b.z, b.w};
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const float v = acc[rt][nb][j] + bv[j];
          h[rt][nb][j] = v > 0.f && nb < nb0 ? v : 0.f;  // blocks past N0 feed +0
        }
      }
    // hidden layers: the previous layer's column block kg is this layer's k-group kg
    const float* Wl = hw;
    const float* bh = hbs;
#pragma unroll 1
    for (int l = 1; l + 1 < nl; Wl += p.dims[l] * p.dims[l + 1], bh += p.dims[l + 1], ++l) {
      const int N = p.dims[l + 1], nkg = p.dims[l] >> 4, nbo = N >> 4;
#pragma unroll
      for (int rt = 0; rt < RW; ++rt)
#pragma unroll
        for (int nb = 0; nb < 4; ++nb) acc[rt][nb] = floatx4{0.f, 0.f, 0.f, 0.f};
      // every k-group and column block runs: the previous layer's blocks past its width
      // are +0 (adding +0 products leaves each sum's bits unchanged), and this layer's blocks
      // past N are computed on clamped weights and zeroed below
#pragma unroll
      for (int kg = 0; kg < 4; ++kg) {
        float4 w[4];
        const int kgc = kg < nkg ? kg : nkg - 1;
#pragma unroll
        for (int nb = 0; nb < 4; ++nb) {
          const int nbc = nb < nbo ? nb : nbo - 1;
          w[nb] = *(const float4*)(Wl + ((size_t)kgc * N + nbc * 16 + il) * 16 + 4 * ka);
        }
#pragma unroll
        for (int s = 0; s < 4; ++s)
#pragma unroll
          for (int nb = 0; nb < 4; ++nb)
#pragma unroll
            for (int rt = 0; rt < RW; ++rt)
              acc[rt][nb] = __builtin_amdgcn_mfma_f32_16x16x4f32(f4c(w[nb], s), h[rt][kg][s],
                                                                 acc[rt][nb], 0, 0, 0);
      }
#pragma unroll
      for (int nb = 0; nb < 4; ++nb) {
        const int nbc = nb < nbo ? nb : nbo - 1;
        const float4 b = *(const float4*)(bh + 16 * nbc + 4 * ka);
        const float bv[4] = {b.x, b.y, b.z, b.w};
#pragma unroll
        for (int rt = 0; rt < RW; ++rt)
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const float v = acc[rt][nb][j] + bv[j];
            h[rt][nb][j] = v > 0.f && nb < nbo ? v : 0.f;
          }
      }
    }
    if (ph) phq[4] = clock64();
    // final Dense + softmax (classifier.py:23-29) -> f1, k_mlp2's order: quarter w of the
    // last hidden layer's Klast inputs as one fmaf chain from 0, then ((q0 + q1) + q2) + q3
    // + bias.  The wave's rows go through its LDS rows; lane (row, qh) sums RW quarters.
#pragma unroll
    for (int rt = 0; rt < RW; ++rt)
#pragma unroll
      for (int nb = 0; nb < 4; ++nb)
        if (nb < (Klast >> 4))
          *(float4*)(hs + (16 * rt + il) * hld + 16 * nb + 4 * ka) =
              make_float4(h[rt][nb][0], h[rt][nb][1], h[rt][nb][2], h[rt][nb][3]);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    const int row = lane % TR, qh = lane / TR;
    const int kq = Klast >> 2;
    float ps[RW][NO];
#pragma unroll
    for (int qi = 0; qi < RW; ++qi) {
      const int k0 = (qh * RW + qi) * kq;
      const float* ir = hs + row * hld + k0;
      const float* wq = wl + k0 * nout;
#pragma unroll
      for (int c = 0; c < NO; ++c) ps[qi][c] = 0.f;
#pragma unroll 4
      for (int k = 0; k < kq; ++k) {
        const float v = ir[k];
#pragma unroll
        for (int c = 0; c < NO; ++c)
          if (c < nout) ps[qi][c] = fmaf(v, wq[k * nout + c], ps[qi][c]);
      }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // hs is rewritten by the next tile
    float q[4][NO];
#pragma unroll
    for (int w = 0; w < 4; ++w)
#pragma unroll
      for (int c = 0; c < NO; ++c) q[w][c] = __shfl(ps[w % RW][c], row + TR * (w / RW), 64);
    const int rr0 = r0 + row;
    if (qh == 0 && rr0 < a.total) {
      const int s = rr0 / a.n, i = rr0 - s * a.n;
      double z[8] = {0.0, 0.0, 0.0, 0.0, 0.0, 0.0, 0.0, 0.0};
      double mx = -__builtin_inf();
#pragma unroll
      for (int c = 0; c < NO; ++c) {
        if (c < nout) {
          z[c] = (double)((((q[0][c] + q[1][c]) + q[2][c]) + q[3][c]) + bl[c]);
          mx = z[c] > mx ? z[c] : mx;
        }
      }
      const double f1 = softmax_pick(z, nout, mx, a.s.min_class[s]);
      if (a.F) {
        const int orow = MV_IDX(a.out_map ? a.out_map[rr0] : i, a.out_rows, CK_MLP_OUT);
        a.F[((size_t)MV_IDX(s, a.total / a.n, CK_MLP_OUT) * a.out_rows + orow) * 3] = f1;
      }
      if (a.hist)
        a.hist[((size_t)s * a.hist_rows + MV_IDX(hist_row0 + i, a.hist_rows, CK_MLP_OUT)) *
               a.hist_w] = f1;
    }
    if (ph) {
      phq[5] = clock64();
      phq[7] = wall_clock64();
    }
  }
}

// ---------------------------------------------------------------------------------------
// k_mlpw: the bf16 perf mode for WIDE hidden layers (BASELINE configs[4]: 756-512-512-256-2,
// widths up to 512) -- 64-row persistent tiles, 8 waves.  Activations live in LDS as bf16
// (two [64][hs] ping-pong buffers, 133 KiB at width 512; fp32 tiles of 64 rows would not
// fit, which is why fp32 keeps k_mlp's 32-row tiles), so each weight byte streamed from L2
// serves 64 rows instead of 32.  Per k-step of 32 a wave issues 4 ds_read_b128 (its A
// fragments: lane (il, ka) holds row il, k = 32 s + 8 ka + j), CJ dwordx4 weight loads (the
// next step's prefetched) and 4 CJ v_mfma_f32_16x16x32_bf16.  The last hidden layer's
// outputs stay fp32 in registers and fold straight into the final Dense (partial sums over
// each lane's columns, a 16-lane butterfly, then the 8 waves' parts in order) -> softmax ->
// f1.  Arithmetic = the k_mlp2 bf16 mode's (inputs of every hidden layer rounded to bf16).
constexpr int MW_ROWS = 64;
constexpr int MW_T = 512;
struct MwLds {
  unsigned h0, h1, part, total;
  int hs;  // bf16 row stride of the activation buffers
};
__host__ __device__ inline MwLds mlpw_lds(const DProblem& p) {
  const int nl = p.n_layers;
  int w = (p.Dm4 + 31) & ~31;
  for (int l = 1; l < nl; ++l) w = p.dims[l] > w ? p.dims[l] : w;
  MwLds L{};
  L.hs = w + 8;  // 16-B row padding: consecutive rows start 4 banks apart
  const unsigned head =
      256 + (((unsigned)(p.dims[nl - 1] * p.dims[nl] + p.dims[nl]) * 4 + 15) & ~15u);
  const unsigned hb = (unsigned)MW_ROWS * L.hs * 2;
  L.h0 = head;
  L.h1 = L.h0 + hb;
  L.part = L.h1 + hb;
  L.total = L.part + (unsigned)(MW_T / 64) * MW_ROWS * p.dims[nl] * 4;
  return L;
}

template <int CJ>
__global__ __launch_bounds__(MW_T) void k_mlpw(int slot, int hist_row0) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const RowsArgs& a = c_rows[slot];
  const DProblem& p = a.p;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int il = lane & 15, ka = lane >> 4;
  const int nl = p.n_layers;
  const int K0 = p.Dm4;
  const int Klast = p.dims[nl - 1], nout = p.dims[nl];
  const MwLds L = mlpw_lds(p);
  const int hs = L.hs;
  int* rowst = (int*)smem;
  float* wl = (float*)(smem + 256);
  float* bl = wl + Klast * nout;
  __bf16* H0 = (__bf16*)(smem + L.h0);
  __bf16* H1 = (__bf16*)(smem + L.h1);
  float* part = (float*)(smem + L.part);
  for (int q = tid; q < Klast * nout; q += MW_T) wl[q] = p.W[nl - 1][q];
  if (tid < nout) bl[tid] = p.bias[nl - 1][tid];
  const int ntiles = (a.total + MW_ROWS - 1) / MW_ROWS;
  const int nq = ((K0 + 31) & ~31) >> 3;  // 8-k groups of the layer-0 tile (K zero padded)
  for (int tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
    const int r0 = tile * MW_ROWS;
    __syncthreads();  // the previous tile's readers of rowst / H / part are done
    if (tid < MW_ROWS) rowst[tid] = r0 + tid < a.total ? (r0 + tid) / a.n : -1;
    // layer-0 input: the fp32 ML rows rounded to bf16
    for (int idx = tid; idx < MW_ROWS * nq; idx += MW_T) {
      const int row = idx / nq, q = idx - row * nq;
      const int k = 8 * q;
      const int rr = r0 + row < a.total ? r0 + row : a.total - 1;
      const bool on = k < K0;
      const float* src = a.xml + (size_t)rr * K0 + (on ? k : 0);
      *(bf16x8*)(H0 + row * hs + k) = to_bf16x8(*(const float4*)src, *(const float4*)(src + 4), on);
    }
    __syncthreads();
    for (int l = 0; l + 1 < nl; ++l) {
      const __bf16* in = (l & 1) ? H1 : H0;
      __bf16* out = (l & 1) ? H0 : H1;
      const int K = l == 0 ? K0 : p.dims[l];
      const int N = p.dims[l + 1];
      const int nct = N >> 4;
      const int nst = (K + 31) >> 5;
      const __bf16* W = (const __bf16*)p.Wb[l];
      floatx4 acc[CJ][4];
#pragma unroll
      for (int j = 0; j < CJ; ++j)
#pragma unroll
        for (int rt = 0; rt < 4; ++rt) acc[j][rt] = floatx4{0.f, 0.f, 0.f, 0.f};
      auto load_b = [&](int st, bf16x8 (&bf)[CJ]) {
        const int sc = st < nst ? st : nst - 1;
#pragma unroll
        for (int j = 0; j < CJ; ++j) {
          const int ct = wave + 8 * j < nct ? wave + 8 * j : nct - 1;
          bf[j] = *(const bf16x8*)(W + ((size_t)sc * N + ct * 16 + il) * 32 + 8 * ka);
        }
      };
      auto load_a = [&](int st, bf16x8 (&af)[4]) {
        const int k = 32 * (st < nst ? st : nst - 1) + 8 * ka;
#pragma unroll
        for (int rt = 0; rt < 4; ++rt) {
          af[rt] = *(const bf16x8*)(in + (rt * 16 + il) * hs + (k < K ? k : 0));
          if (k >= K) af[rt] = bf16x8{};
        }
      };
      auto step = [&](const bf16x8 (&bf)[CJ], const bf16x8 (&af)[4]) {
#pragma unroll
        for (int j = 0; j < CJ; ++j) {
          if (wave + 8 * j < nct) {
#pragma unroll
            for (int rt = 0; rt < 4; ++rt)
              acc[j][rt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[rt], bf[j], acc[j][rt], 0, 0, 0);
          }
        }
      };
      // two operand sets used in turn, so each k-step's loads land in the set the step after
      // next consumes: no register rotation (a move of an in-flight load's destination makes
      // the compiler wait vmcnt(0), which is what kept the one-step prefetch from hiding
      // anything)
      bf16x8 bA[CJ], bB[CJ], aA[4], aB[4];
      load_b(0, bA);
      load_a(0, aA);
      int st = 0;
      for (; st + 1 < nst; st += 2) {
        load_b(st + 1, bB);
        load_a(st + 1, aB);
        step(bA, aA);
        load_b(st + 2, bA);  // clamped past the end (an unused load on the last pair)
        load_a(st + 2, aA);
        step(bB, aB);
      }
      if (st < nst) step(bA, aA);
      const bool last = l + 2 == nl;
      // + bias, ReLU in place; hidden outputs to LDS as bf16
#pragma unroll
      for (int j = 0; j < CJ; ++j) {
        const int ct = wave + 8 * j;
        if (ct < nct) {
          const int col = ct * 16 + il;
#pragma unroll
          for (int rt = 0; rt < 4; ++rt) {
#pragma unroll
            for (int jj = 0; jj < 4; ++jj) {
              const int row = rt * 16 + ka * 4 + jj;
              float bv;
              if (l == 0) {
                const int s = rowst[row];
                bv = a.s.bias1[(size_t)(s < 0 ? 0 : s) * N + col];
              } else {
                bv = p.bias[l][col];
              }
              const float v = acc[j][rt][jj] + bv;
              acc[j][rt][jj] = v > 0.f ? v : 0.f;
              if (!last) out[row * hs + col] = (__bf16)acc[j][rt][jj];
            }
          }
        }
      }
      if (last) {
        // the final Dense from the fp32 registers: per class, partial logits over this lane's
        // columns, summed over the 16 lanes sharing the rows, one part per wave
        for (int c = 0; c < nout; ++c) {
          float ps[4][4];
#pragma unroll
          for (int rt = 0; rt < 4; ++rt)
#pragma unroll
            for (int jj = 0; jj < 4; ++jj) ps[rt][jj] = 0.f;
#pragma unroll
          for (int j = 0; j < CJ; ++j) {
            const int ct = wave + 8 * j;
            if (ct < nct) {
              const float wv = wl[(ct * 16 + il) * nout + c];
#pragma unroll
              for (int rt = 0; rt < 4; ++rt)
#pragma unroll
                for (int jj = 0; jj < 4; ++jj) ps[rt][jj] = fmaf(acc[j][rt][jj], wv, ps[rt][jj]);
            }
          }
#pragma unroll
          for (int rt = 0; rt < 4; ++rt)
#pragma unroll
            for (int jj = 0; jj < 4; ++jj) {
              float v = ps[rt][jj];
              v += __shfl_xor(v, 1);
              v += __shfl_xor(v, 2);
              v += __shfl_xor(v, 4);
              v += __shfl_xor(v, 8);
              if (il == 0) part[(wave * MW_ROWS + rt * 16 + ka * 4 + jj) * nout + c] = v;
            }
        }
      }
      __syncthreads();
    }
    if (tid < MW_ROWS) {
      const int s = rowst[tid];
      if (s >= 0) {
        double z[8];
        double mx = -__builtin_inf();
#pragma unroll
        for (int c = 0; c < 8; ++c) {
          z[c] = 0.0;
          if (c < nout) {
            float t = 0.f;
            for (int w = 0; w < MW_T / 64; ++w) t += part[(w * MW_ROWS + tid) * nout + c];
            z[c] = (double)(t + bl[c]);
            mx = z[c] > mx ? z[c] : mx;
          }
        }
        const double f1 = softmax_pick(z, nout, mx, a.s.min_class[s]);
        const int i = r0 + tid - s * a.n;
        if (a.F) {
          const int orow = a.out_map ? a.out_map[(size_t)s * a.n + i] : i;
          a.F[((size_t)s * a.out_rows + orow) * 3] = f1;
        }
        if (a.hist) a.hist[((size_t)s * a.hist_rows + hist_row0 + i) * a.hist_w] = f1;
      }
    }
  }
}

// ---------------------------------------------------------------------------------------
// k_mlpw32: the fp32 (parity-mode) classifier for WIDE hidden layers (BASELINE configs[4]:
// 756-512-512-256-2) -- 64-row persistent tiles, 8 waves, one workgroup per CU.  Exact fp32
// products on v_mfma_f32_16x16x4f32 like k_mlp2; a 64-row fp32 activation tile of width 512
// is 128 KiB, so there is ONE activation buffer: each layer accumulates its outputs in
// registers, a barrier retires every wave's reads of the layer input, then the outputs
// (bias + ReLU) overwrite it.  Per k-group of 16 a lane reads its four rows' A fragments as
// ds_read_b128 (k = 16 kg + 4 ka + s for sub-step s, as k_mlp2's packed Wp) and CJ dwordx4
// of the packed weights, one k-group ahead in two alternating operand sets; 16 CJ MFMAs per
// k-group.  The last
// hidden layer folds into the final Dense from the fp32 registers (as k_mlpw) -> softmax.
// Replaces the 32-row-tile k_mlp for this shape (each weight byte from L2 now serves 64
// rows; the tile's MFMAs per k-group no longer wait out their loads).
struct Mw32Lds {
  unsigned h, part, total;
  int hs;  // fp32 row stride of the activation buffer
};
__host__ __device__ inline Mw32Lds mlpw32_lds(const DProblem& p) {
  const int nl = p.n_layers;
  int w = p.Dm4;
  for (int l = 1; l < nl; ++l) w = p.dims[l] > w ? p.dims[l] : w;
  Mw32Lds L{};
  L.hs = w + 4;  // 16-B row padding: consecutive rows start 4 banks apart
  const unsigned head =
      256 + (((unsigned)(p.dims[nl - 1] * p.dims[nl] + p.dims[nl]) * 4 + 15) & ~15u);
  L.h = head;
  L.part = L.h + (unsigned)MW_ROWS * L.hs * 4;
  L.total = L.part + (unsigned)(MW_T / 64) * MW_ROWS * p.dims[nl] * 4;
  return L;
}
// The shapes k_mlpw32 takes: every MFMA layer's K and N multiples of 16 (Wp packed), at
// most 4 column tiles per wave (N <= 512: the 256-VGPR budget of two waves per SIMD), LDS
// within the CU's 160 KiB.
__host__ __device__ inline bool mlpw32_ok(const DProblem& p) {
  if (p.n_layers < 2 || !p.Wp[0]) return false;
  for (int l = 1; l < p.n_layers; ++l)
    if (p.dims[l] % 16 || p.dims[l] > 512) return false;
  return p.Dm4 % 16 == 0 && p.dims[p.n_layers] <= 8 && mlpw32_lds(p).total <= 160 * 1024;
}

template <int CJ>
__global__ __launch_bounds__(MW_T) void k_mlpw32(int slot, int hist_row0) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const RowsArgs& a = c_rows[slot];
  const DProblem& p = a.p;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int il = lane & 15, ka = lane >> 4;
  const int nl = p.n_layers;
  const int K0 = p.Dm4;
  const int Klast = p.dims[nl - 1], nout = p.dims[nl];
  const Mw32Lds L = mlpw32_lds(p);
  const int hs = L.hs;
  int* rowst = (int*)smem;
  float* wl = (float*)(smem + 256);
  float* bl = wl + Klast * nout;
  float* H = (float*)(smem + L.h);
  float* part = (float*)(smem + L.part);
  for (int q = tid; q < Klast * nout; q += MW_T) wl[q] = p.W[nl - 1][q];
  if (tid < nout) bl[tid] = p.bias[nl - 1][tid];
  const int ntiles = (a.total + MW_ROWS - 1) / MW_ROWS;
  const int nq = K0 >> 2;  // float4 pieces of a layer-0 row
  for (int tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
    const int r0 = tile * MW_ROWS;
    __syncthreads();  // the previous tile's readers of rowst / H / part are done
    if (tid < MW_ROWS) rowst[tid] = r0 + tid < a.total ? (r0 + tid) / a.n : -1;
    // layer-0 input: the fp32 ML rows (k_genc's xml)
    for (int idx = tid; idx < MW_ROWS * nq; idx += MW_T) {
      const int row = idx / nq, q = idx - row * nq;
      const int rr = r0 + row < a.total ? r0 + row : a.total - 1;
      *(float4*)(H + row * hs + 4 * q) = *(const float4*)(a.xml + (size_t)rr * K0 + 4 * q);
    }
    __syncthreads();
    for (int l = 0; l + 1 < nl; ++l) {
      const int K = l == 0 ? K0 : p.dims[l];
      const int N = p.dims[l + 1];
      const int nct = N >> 4;
      const int ng = K >> 4;
      const float* W = p.Wp[l];
      floatx4 acc[CJ][4];
#pragma unroll
      for (int j = 0; j < CJ; ++j)
#pragma unroll
        for (int rt = 0; rt < 4; ++rt) acc[j][rt] = floatx4{0.f, 0.f, 0.f, 0.f};
      auto load_b = [&](int kg, float4 (&b)[CJ]) {
        const int kc = kg < ng ? kg : ng - 1;
#pragma unroll
        for (int j = 0; j < CJ; ++j) {
          const int ct = wave + 8 * j < nct ? wave + 8 * j : nct - 1;
          b[j] = *(const float4*)(W + ((size_t)kc * N + ct * 16 + il) * 16 + 4 * ka);
        }
      };
      auto load_a = [&](int kg, float4 (&af)[4]) {
        const int kc = kg < ng ? kg : ng - 1;
#pragma unroll
        for (int rt = 0; rt < 4; ++rt)
          af[rt] = *(const float4*)(H + (rt * 16 + il) * hs + 16 * kc + 4 * ka);
      };
      auto step = [&](const float4 (&b)[CJ], const float4 (&af)[4]) {
#pragma unroll
        for (int sub = 0; sub < 4; ++sub)
#pragma unroll
          for (int j = 0; j < CJ; ++j) {
            if (wave + 8 * j < nct) {
              const float bv = sub == 0 ? b[j].x : sub == 1 ? b[j].y : sub == 2 ? b[j].z : b[j].w;
#pragma unroll
              for (int rt = 0; rt < 4; ++rt) {
                const float av = sub == 0 ? af[rt].x : sub == 1 ? af[rt].y
                                 : sub == 2 ? af[rt].z : af[rt].w;
                acc[j][rt] = __builtin_amdgcn_mfma_f32_16x16x4f32(av, bv, acc[j][rt], 0, 0, 0);
              }
            }
          }
      };
      // two weight sets used in turn (no register rotation: see k_mlpw); the A fragments are
      // read at each k-group's start (a second set would spill at CJ = 4)
      float4 bA[CJ], bB[CJ], af[4];
      load_b(0, bA);
      int kg = 0;
      for (; kg + 1 < ng; kg += 2) {
        load_b(kg + 1, bB);
        load_a(kg, af);
        step(bA, af);
        load_b(kg + 2, bA);  // clamped past the end (an unused load on the last pair)
        load_a(kg + 1, af);
        step(bB, af);
      }
      if (kg < ng) {
        load_a(kg, af);
        step(bA, af);
      }
      const bool last = l + 2 == nl;
      __syncthreads();  // every wave's reads of this layer's input are done: outputs replace it
      // + bias, ReLU; hidden outputs to LDS (fp32)
#pragma unroll
      for (int j = 0; j < CJ; ++j) {
        const int ct = wave + 8 * j;
        if (ct < nct) {
          const int col = ct * 16 + il;
#pragma unroll
          for (int rt = 0; rt < 4; ++rt) {
#pragma unroll
            for (int jj = 0; jj < 4; ++jj) {
              const int row = rt * 16 + ka * 4 + jj;
              float bv;
              if (l == 0) {
                const int s = rowst[row];
                bv = a.s.bias1[(size_t)(s < 0 ? 0 : s) * N + col];
              } else {
                bv = p.bias[l][col];
              }
              const float v = acc[j][rt][jj] + bv;
              acc[j][rt][jj] = v > 0.f ? v : 0.f;
              if (!last) H[row * hs + col] = acc[j][rt][jj];
            }
          }
        }
      }
      if (last) {
        // the final Dense from the fp32 registers (as k_mlpw)
        for (int c = 0; c < nout; ++c) {
          float ps[4][4];
#pragma unroll
          for (int rt = 0; rt < 4; ++rt)
#pragma unroll
            for (int jj = 0; jj < 4; ++jj) ps[rt][jj] = 0.f;
#pragma unroll
          for (int j = 0; j < CJ; ++j) {
            const int ct = wave + 8 * j;
            if (ct < nct) {
              const float wv = wl[(ct * 16 + il) * nout + c];
#pragma unroll
              for (int rt = 0; rt < 4; ++rt)
#pragma unroll
                for (int jj = 0; jj < 4; ++jj) ps[rt][jj] = fmaf(acc[j][rt][jj], wv, ps[rt][jj]);
            }
          }
#pragma unroll
          for (int rt = 0; rt < 4; ++rt)
#pragma unroll
            for (int jj = 0; jj < 4; ++jj) {
              float v = ps[rt][jj];
              v += __shfl_xor(v, 1);
              v += __shfl_xor(v, 2);
              v += __shfl_xor(v, 4);
              v += __shfl_xor(v, 8);
              if (il == 0) part[(wave * MW_ROWS + rt * 16 + ka * 4 + jj) * nout + c] = v;
            }
        }
      }
      __syncthreads();
    }
    if (tid < MW_ROWS) {
      const int s = rowst[tid];
      if (s >= 0) {
        double z[8];
        double mx = -__builtin_inf();
#pragma unroll
        for (int c = 0; c < 8; ++c) {
          z[c] = 0.0;
          if (c < nout) {
            float t = 0.f;
            for (int w = 0; w < MW_T / 64; ++w) t += part[(w * MW_ROWS + tid) * nout + c];
            z[c] = (double)(t + bl[c]);
            mx = z[c] > mx ? z[c] : mx;
          }
        }
        const double f1 = softmax_pick(z, nout, mx, a.s.min_class[s]);
        const int i = r0 + tid - s * a.n;
        if (a.F) {
          const int orow = a.out_map ? a.out_map[(size_t)s * a.n + i] : i;
          a.F[((size_t)s * a.out_rows + orow) * 3] = f1;
        }
        if (a.hist) a.hist[((size_t)s * a.hist_rows + hist_row0 + i) * a.hist_w] = f1;
      }
    }
  }
}

// Classifier.predict_proba: 16 RT rows per workgroup, full-width first layer.
template <int MAXCT, int RT = 2>
__global__ __launch_bounds__(EVAL_T) void k_predict(MlpArgs a) {
  constexpr int TR = 16 * RT;
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
  float* R2 = (float*)(smem + head + predict_region1_bytes(a.D4, hmax, TR));
  const int D = a.dims[0];
  const int r0 = blockIdx.x * TR;
  for (int q = tid; q < Klast * nout; q += EVAL_T) ws[q] = a.W[nl - 1][q];
  if (tid < nout) wsb[tid] = a.bias[nl - 1][tid];
  for (int idx = tid; idx < TR * a.D4; idx += EVAL_T) {
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
    dense_mfma<MAXCT, RT>(in, ldi, K, a.W[l], N, a.bias[l], nullptr, nullptr, outb, N + 1, wave,
                      lane);
    __syncthreads();
    in = outb;
    ldi = N + 1;
    K = N;
    float* tmp = outb;
    outb = other;
    other = tmp;
  }
  if (tid < TR && r0 + tid < a.n) {
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
  constraints_row<FULL>(global_tab(p), xrow, lane, G + (size_t)r * p.C, nullptr, false);
}

// FeatureEncoder.genetic_to_ml (feature_encoder.py:91-130) for host plugins: genes
// [B][n][V] -> ML rows [B][n][D]; one thread per output feature (immutable features from
// the state's x_init, one-hot features 1.0 where the group's gene equals their category).
__global__ __launch_bounds__(256) void k_decode(const int* __restrict__ fdec,
                                                const double* __restrict__ x_init, int B, int n,
                                                int V, int D, const double* __restrict__ genes,
                                                double* __restrict__ x) {
  const long total = (long)B * n * D;
  for (long t = (long)blockIdx.x * blockDim.x + threadIdx.x; t < total;
       t += (long)gridDim.x * blockDim.x) {
    const long row = t / D;
    const int f = (int)(t - row * D);
    const int b = (int)(row / n);
    const int m = fdec[f];
    double v;
    if (m < 0) {
      v = x_init[(size_t)b * D + f];
    } else {
      const double g = genes[(size_t)row * V + (m & 0xFFFF)];
      const int cat = m >> 16;
      v = cat ? (g == (double)(cat - 1) ? 1.0 : 0.0) : g;
    }
    x[t] = v;
  }
}

hipError_t launch_decode(const DProblem& p, const DStates& s, int B, int n, const double* genes,
                         double* x, hipStream_t stream) {
  const long total = (long)B * n * p.D;
  if (total <= 0) return hipSuccess;
  long blocks = (total + 255) / 256;
  if (blocks > 8192) blocks = 8192;
  MV_LAUNCH(k_decode, dim3((unsigned)blocks), dim3(256), 0, stream, p.fdec, s.x_init, B,
                     n, p.V, p.D, genes, x);
  return hipGetLastError();
}

// Per-state constants: one workgroup per state.
__global__ __launch_bounds__(256) void k_setup_states(int slot,
                                                      const double* x_init, const double* xl,
                                                      const double* xu, const float* W1full,
                                                      const float* b1, double* gl, double* gu,
                                                      unsigned char* sblob, float* bias1,
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
  const VaryOff vo = vary_offsets(p);
  double* s_es = (double*)(sblob + (size_t)b * vo.sb + vo.es);
  double* s_em = (double*)(sblob + (size_t)b * vo.sb + vo.em);
  double* s_x0 = (double*)(sblob + (size_t)b * vo.sb + vo.x0);
  double* s_xi = (double*)(sblob + (size_t)b * vo.sb + vo.xi);
  for (int f = tid; f < p.D; f += blockDim.x) s_xi[f] = xi[f];
  for (int j = p.Dm + tid; j < p.Dm4; j += blockDim.x) {
    s_es[j] = 0.0;
    s_em[j] = 0.0;
    s_x0[j] = 0.0;
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
    s_es[j] = sc;
    s_em[j] = mi;
    s_x0[j] = xi[f] * sc + mi;
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
  const void* fns[] = {(const void*)k_mlp<1, false>, (const void*)k_mlp<2, false>,
                       (const void*)k_mlp<4, false>, (const void*)k_mlp<8, false>,
                       (const void*)k_mlp<1, true>,  (const void*)k_mlp<2, true>,
                       (const void*)k_mlp<4, true>,  (const void*)k_mlp<8, true>,
                       (const void*)k_constraints<false>, (const void*)k_constraints<true>};
  for (const void* f : fns)
    (void)hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, lim);
  (void)hipGetLastError();
  done = true;
}

template <class K>
static void allow_lds(K kern) {
  (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize,
                            160 * 1024);
  (void)hipGetLastError();
}

// Rows per k_gen / k_cons workgroup: chunks of at most VARY_ROWS_MAX rows of one state.
// Among the chunk counts from ceil(n / cap) up, the one whose chunks split evenly over the
// workgroup's waves (least idle wave-row slots) -- O = 100 gives 5 chunks of 20 rows, 5 per
// wave, instead of 4 x 25 (waves of 7 and 6 rows): +1.4 % botnet evals/s, +3.3 % with one
// group.  MV_VARY_ROWS overrides the cap (development sweeps).
static int vary_rows_per_wg(int n) {
  static const char* env = std::getenv("MV_VARY_ROWS");
  static int cap = [] {
    // row_draws maps a wave's rows onto lanes 4 k + q, plan_draws onto PLAN_MUT k + q: at
    // most 64 / PLAN_MUT rows per wave
    constexpr int hi = (64 / PLAN_MUT) * VARY_W < 64 ? (64 / PLAN_MUT) * VARY_W : 64;
    const int v = env ? std::atoi(env) : VARY_ROWS_MAX;
    return v < 4 ? 4 : (v > hi ? hi : v);
  }();
  const int c0 = (n + cap - 1) / cap;
  if (env) return (n + c0 - 1) / c0;
  int best = (n + c0 - 1) / c0, waste = INT32_MAX;
  for (int c = c0; c <= c0 + 3; ++c) {
    const int r = (n + c - 1) / c;
    const int w = c * VARY_W * ((r + VARY_W - 1) / VARY_W) - n;
    if (w < waste) {
      waste = w;
      best = r;
    }
  }
  return best;
}

static int device_cus() {
  int dev = 0, cus = 0;
  if (hipGetDevice(&dev) != hipSuccess ||
      hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
    cus = 256;
  (void)hipGetLastError();
  return cus;
}

// Small attacks (states_all x chunks below four workgroups per CU, k_genc's occupancy): the
// chunks shrink -- down to one row per wave -- until the row launches fill the chip.  Each
// chunk repeats the workgroup prologue, but with few states the CUs would idle instead, and a
// generation's row-kernel latency is one chunk's (e.g. 48 botnet states, 8-GPU strong scaling
// of configs[1]: 240 workgroups of 20 rows -> 1,200 of 4).  Results do not depend on the
// chunking (every draw is keyed by the row inside its state).
static int vary_rows_per_wg(int n, int states_all) {
  int best = vary_rows_per_wg(n);
  static const bool env = std::getenv("MV_VARY_ROWS") != nullptr;
  if (env || states_all <= 0) return best;
  static const int target = 4 * device_cus();
  if ((long long)states_all * ((n + best - 1) / best) >= target) return best;
  const int c = (target + states_all - 1) / states_all;  // chunks per state wanted
  const int r = (n + c - 1) / c;
  return r < VARY_W ? (best < VARY_W ? best : VARY_W) : (r < best ? r : best);
}

static int vary_nt(const DProblem& p) {
  const int m = p.V > p.Dm4 ? p.V : p.Dm4;
  const int nt = (m + 63) / 64;
  return nt <= 1 ? 1 : nt <= 2 ? 2 : nt <= 4 ? 4 : nt <= 8 ? 8 : 16;
}

template <bool IDENT, int NT>
static hipError_t gen_go(dim3 grid, size_t lds, hipStream_t s, int slot, int gen, int h0, int rw,
                         bool sbx) {
  static bool configured = false;
  if (!configured) {
    allow_lds(k_gen<IDENT, NT, false>);
    allow_lds(k_gen<IDENT, NT, true>);
    configured = true;
  }
  if (sbx)
    MV_LAUNCH((k_gen<IDENT, NT, true>), grid, dim3(VARY_T), lds, s, slot, gen, h0, rw);
  else
    MV_LAUNCH((k_gen<IDENT, NT, false>), grid, dim3(VARY_T), lds, s, slot, gen, h0, rw);
  return hipGetLastError();
}

template <bool FULL, bool IDENT, int NT>
static hipError_t cons_go(dim3 grid, size_t lds, hipStream_t s, int slot, int h0, int rw) {
  static bool configured = false;
  if (!configured) {
    allow_lds(k_cons<FULL, IDENT, NT>);
    configured = true;
  }
  MV_LAUNCH((k_cons<FULL, IDENT, NT>), grid, dim3(CONS_T), lds, s, slot, h0, rw);
  return hipGetLastError();
}

// Narrow rows (LCLD-shaped problems): k_narrow does k_gen's and k_cons's work in one launch
// (two-point crossover; the SBX option and variation-only launches keep the wave-per-row
// kernels).  MV_NARROW=0 turns it off (A/B runs).
static bool use_narrow(const RowsArgs& a) {
  const char* s = std::getenv("MV_NARROW");  // read per launch: tests flip it in-process
  return !(s && s[0] == '0') && a.do_eval && narrow_ok(a.p) && !(a.mode == 1 && a.cx_kind == 1) &&
         !a.p.compact;  // the compact layout runs on the wave-per-row kernels only
}

template <int NV, bool FULL>
static hipError_t narrow_go(const RowsArgs& a, int slot, int gen, int hist_row0,
                            hipStream_t stream) {
  static bool configured = false;
  if (!configured) {
    allow_lds(k_narrow<NV, FULL>);
    configured = true;
  }
  const size_t lds = narrow_lds(vary_offsets(a.p), a.p).total;
  const dim3 grid((unsigned)((a.total + NARROW_T - 1) / NARROW_T));
  MV_LAUNCH((k_narrow<NV, FULL>), grid, dim3(NARROW_T), lds, stream, slot, gen,
                     hist_row0);
  return hipGetLastError();
}

static hipError_t launch_narrow(const RowsArgs& a, int slot, int gen, int hist_row0,
                                hipStream_t stream) {
#define NG(NV) \
  return a.p.full_ops ? narrow_go<NV, true>(a, slot, gen, hist_row0, stream) \
                      : narrow_go<NV, false>(a, slot, gen, hist_row0, stream)
  if (a.p.V <= 8) NG(8);
  if (a.p.V <= 16) NG(16);
  NG(32);
#undef NG
}

// k_genc (k_gen + k_cons in one launch) for the wave-per-row evaluation of IDENT problems
// without the LCLD financial ops (the botnet shape).  MV_GENC=0 keeps the two launches.
// k_genc's genes per lane: the exact ceil(max(V, Dm4) / 64) from 4 to 8 (every unused
// register slot costs a masked instruction per row in every phase), else 16.
static int genc_nt(const DProblem& p) {
  const int m = p.V > p.Dm4 ? p.V : p.Dm4;
  const int nt = (m + 63) / 64;
  return nt <= 4 ? 4 : nt <= 8 ? nt : 16;
}

static bool use_genc(const RowsArgs& a) {
  const char* s = std::getenv("MV_GENC");  // read per launch: tests flip it in-process
  return !(s && s[0] == '0') && a.do_eval && a.p.ident && !a.p.full_ops && !use_narrow(a) &&
         (a.p.V > a.p.Dm4 ? a.p.V : a.p.Dm4) > 128;
}

template <int NT>
static hipError_t genc_go(dim3 grid, size_t lds, hipStream_t s, int slot, int gen, int h0, int rw,
                          bool sbx, bool slim) {
  static bool configured = false;
  if (!configured) {
    allow_lds(k_genc<true, NT, false, false>);
    allow_lds(k_genc<true, NT, true, false>);
    allow_lds(k_genc<true, NT, false, true>);
    allow_lds(k_genc<true, NT, true, true>);
    configured = true;
  }
#define GENC(X, Y) \
  MV_LAUNCH((k_genc<true, NT, X, Y>), grid, dim3(VARY_T), lds, s, slot, gen, h0, rw)
  if (sbx) {
    if (slim)
      GENC(true, true);
    else
      GENC(true, false);
  } else {
    if (slim)
      GENC(false, true);
    else
      GENC(false, false);
  }
#undef GENC
  return hipGetLastError();
}

int row_kernel_kind(const RowsArgs& a) {
  if (use_narrow(a)) return 1;
  if (use_genc(a)) return 2;
  return 0;
}

hipError_t launch_gen(const RowsArgs& a, int slot, int gen, int hist_row0, hipStream_t stream) {
  if (a.total <= 0) return hipSuccess;
  if (use_narrow(a)) return launch_narrow(a, slot, gen, hist_row0, stream);
  if (use_genc(a)) {
    const int B = a.total / a.n;
    const int rw = vary_rows_per_wg(a.n, a.states_all);
    const dim3 grid(B * ((a.n + rw - 1) / rw));
    const int nt = genc_nt(a.p);
    const VaryOff o = vary_offsets(a.p);
    const bool sbx = a.mode == 1 && a.cx_kind == 1;
    const GenLds gl = gen_lds(o, gen_regc(a.p, nt), true, true);
    const size_t lg = sbx ? gen_lds_sbx(gl, nt) : gl.total;
    const bool slim = a.p.slim != 0;
    const size_t lc = slim ? cons_lds_slim(o) : cons_lds_total(o);
    static const size_t pad = lds_pad("MV_LDS_PAD_GENC");
    const size_t lds = (slim && !sbx ? genc_fused_lds(o, a.p).total : (lg > lc ? lg : lc)) + pad;
    // k_genc takes mode 1's draws from the variation plan (mv_attack_run's k_survive)
    if (a.mode == 1 && !(a.plan_hdr && a.plan_mw && a.plan_mu)) return hipErrorInvalidValue;
    if (nt == 4) return genc_go<4>(grid, lds, stream, slot, gen, hist_row0, rw, sbx, slim);
    if (nt == 5) return genc_go<5>(grid, lds, stream, slot, gen, hist_row0, rw, sbx, slim);
    if (nt == 6) return genc_go<6>(grid, lds, stream, slot, gen, hist_row0, rw, sbx, slim);
    if (nt == 7) return genc_go<7>(grid, lds, stream, slot, gen, hist_row0, rw, sbx, slim);
    if (nt == 8) return genc_go<8>(grid, lds, stream, slot, gen, hist_row0, rw, sbx, slim);
    return genc_go<16>(grid, lds, stream, slot, gen, hist_row0, rw, sbx, slim);
  }
  const int B = a.total / a.n;
  const int rw = vary_rows_per_wg(a.n, a.states_all);
  const dim3 grid(B * ((a.n + rw - 1) / rw));
  const int nt = vary_nt(a.p);
  const bool ident = a.p.ident != 0;
  const bool sbx = a.mode == 1 && a.cx_kind == 1;
  const GenLds gl = gen_lds(vary_offsets(a.p), gen_regc(a.p, nt), ident, a.do_eval != 0);
  const size_t lds = sbx ? gen_lds_sbx(gl, nt) : gl.total;
#define GEN(I, N) return gen_go<I, N>(grid, lds, stream, slot, gen, hist_row0, rw, sbx)
  if (ident) {
    if (nt == 1) GEN(true, 1);
    if (nt == 2) GEN(true, 2);
    if (nt == 4) GEN(true, 4);
    if (nt == 8) GEN(true, 8);
    GEN(true, 16);
  }
  if (nt == 1) GEN(false, 1);
  if (nt == 2) GEN(false, 2);
  if (nt == 4) GEN(false, 4);
  if (nt == 8) GEN(false, 8);
  GEN(false, 16);
#undef GEN
}

hipError_t launch_cons(const RowsArgs& a, int slot, int hist_row0, hipStream_t stream) {
  if (a.total <= 0 || !a.do_eval) return hipSuccess;
  if (use_narrow(a)) return hipSuccess;  // done by k_narrow in launch_gen
  if (use_genc(a)) return hipSuccess;    // done by k_genc in launch_gen
  const int B = a.total / a.n;
  const int rw = vary_rows_per_wg(a.n, a.states_all);
  const dim3 grid(B * ((a.n + rw - 1) / rw));
  const int nt = vary_nt(a.p);
  const size_t lds = cons_lds_total(vary_offsets(a.p));
#define CONS(F, I, N) return cons_go<F, I, N>(grid, lds, stream, slot, hist_row0, rw)
  if (a.p.full_ops) {  // LCLD programs: one-hot genes, few genes
    if (nt == 1) CONS(true, false, 1);
    if (nt == 2) CONS(true, false, 2);
    if (nt == 4) CONS(true, false, 4);
    if (nt == 8) CONS(true, false, 8);
    CONS(true, false, 16);
  }
  if (a.p.ident) {
    if (nt == 1) CONS(false, true, 1);
    if (nt == 2) CONS(false, true, 2);
    if (nt == 4) CONS(false, true, 4);
    if (nt == 8) CONS(false, true, 8);
    CONS(false, true, 16);
  }
  if (nt == 1) CONS(false, false, 1);
  if (nt == 2) CONS(false, false, 2);
  if (nt == 4) CONS(false, false, 4);
  if (nt == 8) CONS(false, false, 8);
  CONS(false, false, 16);
#undef CONS
}

// Variation + evaluation of the rows in the per-phase chain: k_gen then k_cons.
hipError_t launch_vary(const RowsArgs& a, int slot, int gen, int hist_row0,
                       hipStream_t stream) {
  hipError_t e = launch_gen(a, slot, gen, hist_row0, stream);
  if (e != hipSuccess) return e;
  return launch_cons(a, slot, hist_row0, stream);
}

static int cu_count() {
  static int n = 0;
  if (!n) {
    int dev = 0;
    hipDeviceProp_t prop;
    if (hipGetDevice(&dev) == hipSuccess && hipGetDeviceProperties(&prop, dev) == hipSuccess)
      n = prop.multiProcessorCount;
    if (n <= 0) n = 256;
  }
  return n;
}

template <int CJ, bool BF, bool DIRECT, bool CO>
static hipError_t mlp2_go3(const RowsArgs& a, int slot, int hist_row0, hipStream_t stream) {
  static bool configured = false;
  static size_t occ_lds = 0;
  static int occ = 2;
  if (!configured) {
    allow_lds(k_mlp2<CJ, BF, DIRECT, CO>);
    configured = true;
  }
  static const size_t pad = lds_pad("MV_LDS_PAD_MLP");
  const size_t lds = mlp2_lds(a.p) + pad;
  if (lds != occ_lds) {  // resident workgroups per CU at this LDS size
    int n = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, k_mlp2<CJ, BF, DIRECT, CO>, 256, lds) != hipSuccess ||
        n < 1)
      n = 1;
    (void)hipGetLastError();
    occ = n;
    occ_lds = lds;
  }
  const int ntiles = (a.total + M2_ROWS - 1) / M2_ROWS;
  const int grid = ntiles < occ * cu_count() ? ntiles : occ * cu_count();
  MV_LAUNCH((k_mlp2<CJ, BF, DIRECT, CO>), dim3(grid), dim3(256), lds, stream, slot,
                     hist_row0);
  return hipGetLastError();
}

template <int CJ, bool BF>
static hipError_t mlp2_go(const RowsArgs& a, int slot, int hist_row0, hipStream_t stream) {
  // CO: the fp32 path's lane-contiguous gene staging (rows of an even gene count start
  // 16-B aligned in the pool); MV_MLP_CO=0 turns it off (A/B)
  static const bool co_env = !(std::getenv("MV_MLP_CO") && std::getenv("MV_MLP_CO")[0] == '0');
  if (a.p.xml_direct && !BF && co_env && (a.p.Dm & 1) == 0)
    return mlp2_go3<CJ, BF, true, true>(a, slot, hist_row0, stream);
  return a.p.xml_direct ? mlp2_go3<CJ, BF, true, false>(a, slot, hist_row0, stream)
                        : mlp2_go3<CJ, BF, false, false>(a, slot, hist_row0, stream);
}

template <int RW, int NO, bool XML = false>
static hipError_t mlpr_go(const RowsArgs& a, int slot, int hist_row0, hipStream_t stream) {
  static size_t occ_lds = 0;
  static int occ = 1;
  const size_t lds = mlpr_lds(a.p, RW).total;
  if (lds != occ_lds) {  // resident workgroups per CU at this LDS size
    int n = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, k_mlpr<RW, NO, XML>, 256, lds) != hipSuccess ||
        n < 1)
      n = 1;
    (void)hipGetLastError();
    occ = n;
    occ_lds = lds;
  }
  const int ntiles = (a.total + 16 * RW - 1) / (16 * RW);
  const int need = (ntiles + 3) / 4;
  const int grid = need < occ * cu_count() ? need : occ * cu_count();
  MV_LAUNCH((k_mlpr<RW, NO, XML>), dim3(grid), dim3(256), lds, stream, slot, hist_row0);
  return hipGetLastError();
}

// k_mlpr's rows per wave tile: MV_MLPR_RW=1 (16) or 2 (32, default)
static bool use_mlpr(const DProblem& p) {
  static const bool off = std::getenv("MV_MLPR") && std::getenv("MV_MLPR")[0] == '0';
  return !off && mlpr_ok(p);
}
static int mlpr_rw() {
  static const int rw = std::getenv("MV_MLPR_RW") ? std::atoi(std::getenv("MV_MLPR_RW")) : 1;
  return rw == 1 ? 1 : 2;
}

template <int CJ>
static hipError_t mlpw_go(const RowsArgs& a, int slot, int hist_row0, hipStream_t stream) {
  static bool configured = false;
  if (!configured) {
    allow_lds(k_mlpw<CJ>);
    configured = true;
  }
  const size_t lds = mlpw_lds(a.p).total;
  const int ntiles = (a.total + MW_ROWS - 1) / MW_ROWS;
  const int grid = ntiles < cu_count() ? ntiles : cu_count();  // one 133-KiB workgroup per CU
  MV_LAUNCH((k_mlpw<CJ>), dim3(grid), dim3(MW_T), lds, stream, slot, hist_row0);
  return hipGetLastError();
}

template <int CJ>
static hipError_t mlpw32_go(const RowsArgs& a, int slot, int hist_row0, hipStream_t stream) {
  static bool configured = false;
  if (!configured) {
    allow_lds(k_mlpw32<CJ>);
    configured = true;
  }
  const size_t lds = mlpw32_lds(a.p).total;
  const int ntiles = (a.total + MW_ROWS - 1) / MW_ROWS;
  const int grid = ntiles < cu_count() ? ntiles : cu_count();  // one workgroup per CU
  MV_LAUNCH((k_mlpw32<CJ>), dim3(grid), dim3(MW_T), lds, stream, slot, hist_row0);
  return hipGetLastError();
}

// fp32 wide classifiers (hidden widths above k_mlp2's 128) on k_mlpw32; MV_MLPW32=0 keeps
// the 32-row-tile k_mlp (A/B)
static bool use_mlpw32(const DProblem& p) {
  static const bool off = std::getenv("MV_MLPW32") && std::getenv("MV_MLPW32")[0] == '0';
  return !off && !p.mlp_bf16 && mlpw32_ok(p);
}

// launch_mlp's choice for a problem: 0 k_mlp, 1 k_mlp2 reading the genes (xml_direct),
// 2 k_mlp2 reading the fp32 ML rows, 4 k_mlpw (bf16), 5 k_mlpw32 (fp32 wide), -1 no model
// (3, k_mlp2x, was retired), 6 k_mlpr (gene-reading, hidden widths <= 64)
int mlp_kernel_kind(const DProblem& p) {
  if (p.n_layers == 0) return -1;
  if (use_mlpr(p)) return p.xml_direct ? 6 : 7;
  if (p.mlp2 && !std::getenv("MV_MLP_V1") && !(p.mlp_bf16 && std::getenv("MV_MLPW")))
    return p.xml_direct ? 1 : 2;
  if (p.mlp_bf16 && mlpw_lds(p).total <= 160 * 1024 && !std::getenv("MV_MLPW_OFF")) return 4;
  if (use_mlpw32(p)) return 5;
  return 0;
}

hipError_t launch_mlp(const RowsArgs& a, int slot, int hist_row0, hipStream_t stream) {
  if (a.total <= 0 || a.p.n_layers == 0) return hipSuccess;  // model-less: f1 from the host
  if (use_mlpr(a.p) && !a.p.xml_direct)  // the fp32 ML rows (LCLD)
    return a.p.dims[a.p.n_layers] <= 2 ? mlpr_go<1, 2, true>(a, slot, hist_row0, stream)
                                       : mlpr_go<1, 8, true>(a, slot, hist_row0, stream);
  if (use_mlpr(a.p)) {
    if (a.p.dims[a.p.n_layers] <= 2)
      return mlpr_rw() == 1 ? mlpr_go<1, 2>(a, slot, hist_row0, stream)
                            : mlpr_go<2, 2>(a, slot, hist_row0, stream);
    return mlpr_rw() == 1 ? mlpr_go<1, 8>(a, slot, hist_row0, stream)
                          : mlpr_go<2, 8>(a, slot, hist_row0, stream);
  }
  // (MV_MLPW=1: the bf16 mode runs k_mlpw for narrow nets too -- development A/B)
  if (a.p.mlp2 && !std::getenv("MV_MLP_V1") && !(a.p.mlp_bf16 && std::getenv("MV_MLPW"))) {
    if (a.p.mlp_bf16)
      return mlp2_hmax(a.p) <= 64 ? mlp2_go<1, true>(a, slot, hist_row0, stream)
                                  : mlp2_go<2, true>(a, slot, hist_row0, stream);
    return mlp2_hmax(a.p) <= 64 ? mlp2_go<1, false>(a, slot, hist_row0, stream)
                                : mlp2_go<2, false>(a, slot, hist_row0, stream);
  }
  if (a.p.mlp_bf16 && mlpw_lds(a.p).total <= 160 * 1024 && !std::getenv("MV_MLPW_OFF")) {
    const int hm = max_hidden(a.p.dims, a.p.n_layers);
    return hm <= 128 ? mlpw_go<1>(a, slot, hist_row0, stream)
                     : hm <= 256 ? mlpw_go<2>(a, slot, hist_row0, stream)
                                 : mlpw_go<4>(a, slot, hist_row0, stream);
  }
  if (use_mlpw32(a.p)) {
    const int hm = max_hidden(a.p.dims, a.p.n_layers);
    return hm <= 128 ? mlpw32_go<1>(a, slot, hist_row0, stream)
                     : hm <= 256 ? mlpw32_go<2>(a, slot, hist_row0, stream)
                                 : mlpw32_go<4>(a, slot, hist_row0, stream);
  }
  configure_lds_once();
  const int nl = a.p.n_layers;
  const int hmax = max_hidden(a.p.dims, nl);
  const size_t lds = mlp_lds_bytes(a.p.Dm4, hmax, a.p.dims[nl - 1], a.p.dims[nl]);
  const dim3 grid((a.total + EVAL_TR - 1) / EVAL_TR);
  const int nct = hmax / 16;
#define MLP(M)                                                                           \
  {                                                                                      \
    if (a.p.mlp_bf16)                                                                    \
      MV_LAUNCH((k_mlp<M, true>), grid, dim3(EVAL_T), lds, stream, slot, hist_row0); \
    else                                                                                 \
      MV_LAUNCH((k_mlp<M, false>), grid, dim3(EVAL_T), lds, stream, slot, hist_row0); \
  }
  if (nct <= 4)
    MLP(1)
  else if (nct <= 8)
    MLP(2)
  else if (nct <= 16)
    MLP(4)
  else
    MLP(8)
#undef MLP
  return hipGetLastError();
}

hipError_t launch_rows(const RowsArgs& a, int slot, int gen, int hist_row0,
                       hipStream_t stream) {
  hipError_t e = launch_vary(a, slot, gen, hist_row0, stream);
  if (e != hipSuccess || !a.do_eval) return e;
  return launch_mlp(a, slot, hist_row0, stream);
}

template <int RT>
static hipError_t predict_go(const MlpArgs& a, int nct, size_t lds, hipStream_t stream) {
  static bool configured = false;
  if (!configured) {
    allow_lds(k_predict<1, RT>);
    allow_lds(k_predict<2, RT>);
    allow_lds(k_predict<4, RT>);
    allow_lds(k_predict<8, RT>);
    configured = true;
  }
  const dim3 grid((a.n + 16 * RT - 1) / (16 * RT));
  if (nct <= 4)
    MV_LAUNCH((k_predict<1, RT>), grid, dim3(EVAL_T), lds, stream, a);
  else if (nct <= 8)
    MV_LAUNCH((k_predict<2, RT>), grid, dim3(EVAL_T), lds, stream, a);
  else if (nct <= 16)
    MV_LAUNCH((k_predict<4, RT>), grid, dim3(EVAL_T), lds, stream, a);
  else
    MV_LAUNCH((k_predict<8, RT>), grid, dim3(EVAL_T), lds, stream, a);
  return hipGetLastError();
}

hipError_t launch_predict(const MlpArgs& a, hipStream_t stream) {
  if (a.n <= 0) return hipSuccess;
  const int nl = a.n_layers;
  const int hmax = max_hidden(a.dims, nl);
  const int nct = hmax / 16;
  // 32-row tiles when they fit the LDS, else 16-row tiles (e.g. 756-512-... models)
  const size_t lds32 = predict_lds_bytes(a.D4, hmax, a.dims[nl - 1], a.dims[nl], 32);
  if (lds32 <= 160 * 1024) return predict_go<2>(a, nct, lds32, stream);
  const size_t lds16 = predict_lds_bytes(a.D4, hmax, a.dims[nl - 1], a.dims[nl], 16);
  if (lds16 > 160 * 1024) return hipErrorInvalidValue;
  return predict_go<1>(a, nct, lds16, stream);
}

hipError_t launch_constraints(const DProblem& hp, int slot, int n, const double* x,
                              double* G, hipStream_t stream) {
  if (n <= 0) return hipSuccess;
  configure_lds_once();
  const size_t lds = (size_t)4 * hp.D * sizeof(double);
  const dim3 grid((n + 3) / 4);
  if (hp.full_ops)
    MV_LAUNCH(k_constraints<true>, grid, dim3(256), lds, stream, slot, n, x, G);
  else
    MV_LAUNCH(k_constraints<false>, grid, dim3(256), lds, stream, slot, n, x, G);
  return hipGetLastError();
}

MV_DEFINE_TAKE_CHECKS(take_checks_eval)

hipError_t launch_setup_states(int slot, int B, const double* x_init, const double* xl,
                               const double* xu, const float* W1full, const float* b1, double* gl,
                               double* gu, unsigned char* sblob, float* bias1, double* genes0,
                               hipStream_t stream) {
  if (B <= 0) return hipSuccess;
  MV_LAUNCH(k_setup_states, dim3(B), dim3(256), 0, stream, slot, x_init, xl, xu, W1full,
                     b1, gl, gu, sblob, bias1, genes0);
  return hipGetLastError();
}

}  // namespace mv
