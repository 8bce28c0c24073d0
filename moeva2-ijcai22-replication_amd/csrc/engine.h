// Internal device-side layouts of the MoEvA2 engine (not part of the C ABI).
//
// HBM layout (all per-state arrays are state-major so a state's rows are contiguous):
//   problem constants  : gene tables, feature maps, ML scaler, constraint program, MLP weights
//   per-state constants: x_init[B][D], genetic bounds gl/gu[B][V], encoder MinMax over the
//                        mutable features enc_scale/enc_min/x0_mm[B][Dm], folded layer-1
//                        bias bias1[B][H1] (b1 + W1[immutable rows] . x_ml[immutable])
//   population pool    : genes[B][S][V] fp64, F[B][S][3] fp64, S = P + O slots per state;
//                        pop_slot[B][P] (population order -> slot), free_slot[B][O];
//                        survival selects P of the P+O merged rows and the O losers'
//                        slots receive the next offspring, so genes never move.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

// MV_CLOCKS (development builds: `make variant NAME=clk DEFS=-DMV_CLOCKS=1`): the k_genc /
// k_mlp2 / k_survive phase clocks behind MV_GEN_PHASES / MV_MLP_PHASES / MV_SURV_PHASES.
// Compiled out of the product build, so its kernels carry no clock branches.
#ifndef MV_CLOCKS
#define MV_CLOCKS 0
#endif

namespace mv {

constexpr int MAX_LAYERS = 6;
constexpr int EVAL_TR = 32;      // rows per evaluation tile (two 16-row MFMA tiles)
constexpr int EVAL_T = 256;      // threads per evaluation workgroup (4 waves)
#ifndef MV_VARY_T
#define MV_VARY_T 256
#endif
constexpr int VARY_T = MV_VARY_T; // threads per k_gen / k_cons workgroup
constexpr int VARY_W = VARY_T / 64;  // its waves: wave w takes rows w, w + VARY_W, ...
#ifndef MV_CONS_T
#define MV_CONS_T 256
#endif
// k_cons workgroup threads.  512 makes the kernel alone faster (66 -> 58 us) but the
// four-group attack slower (152.3 -> 149.9 M evals/s, A/B on one box): the concurrent
// schedule is bound by the chip's aggregate issue/latency capacity, not one kernel's.
constexpr int CONS_T = MV_CONS_T;
constexpr int CONS_W = CONS_T / 64;
constexpr int VARY_ROWS_MAX = 32; // rows of one state per k_gen / k_cons workgroup (swept: 16/32/64)
constexpr int VARY_MAX_V = 1024;    // genes per row (16 per lane)
#ifndef MV_SURV_T
#define MV_SURV_T 512
#endif
constexpr int SURV_T = MV_SURV_T;  // threads per survival workgroup (8 waves)
// threads of the N > SURV_NLDS survival instance (configs[3], N = 963): 16 waves, so its
// issue-bound dominance and association passes interleave four waves per SIMD (round 5:
// k_survive 86.8 -> 70.2 ms per launch at configs[3]; 1024 threads at N = 303 measured
// 110 vs 75 us, so the LDS-resident instance keeps SURV_T)
#ifndef MV_SURV_T_BIG
#define MV_SURV_T_BIG 1024
#endif
constexpr int SURV_T_BIG = MV_SURV_T_BIG;
// threads of the N <= SURV_NLDS instance when the attack's states all fit two workgroups per
// CU (SurvArgs.wide): 9 waves (round 5, headline: 640 threads 225.4 vs 220.2 M evals/s with
// 512; 576 / 704 against 640: 227.1 / 225.3 vs 226.3 M; 768: 224.8 M; 896: 200.6 M; with
// 4,000 states (configs[2]) 768 threads lose occupancy: 461.5 vs 481.4 M, so many states
// keep SURV_T)
#ifndef MV_SURV_T_MID
#define MV_SURV_T_MID 576
#endif
constexpr int SURV_T_MID = MV_SURV_T_MID;
constexpr int SURV_NMAX = 1024;  // merged individuals per state (n_pop 640: P + O = 963)
constexpr int SURV_NLDS = 512;   // up to this N the dominance bitsets live in LDS, else in HBM
constexpr int SURV_RMAX = 640;   // reference points
constexpr int ARG_SLOTS = 32;    // constant-memory launch-argument slots per device
constexpr int MAX_GROUPS = 16;   // state groups (streams) of one attack (default 4: api.cpp)
constexpr double INT_WIDEN = 0.5 - 1e-16;  // pymoo apply_float_operation bound widening

struct DProblem {
  int D, V, Dm, Dm4, C, n_ohe;  // Dm4: mutable features padded to a multiple of 16
  // Vr: the genetic length the variation draws are defined over (mutation positions, SBX
  // draw indices, the geometric gap table).  V = Vr except in the attack's compact layout
  // (mv_set_states): there the genes that can never change -- integer genes whose bounds are
  // equal and whose initial value is that bound in every state -- are not stored; V counts
  // the free genes, and region B's cmap / fidx map between the two numberings
  int Vr;
  int n_ohe_feat;         // features of all one-hot groups (ohe_feat length)
  int n_sub[2];           // crossover subsets: 0 real, 1 int (OHE genes are int), over Vr
  const int* gene_kind;   // [V]
  const int* gene_feat;   // [V]
  const int* gene_sub;    // [V] index within its subset (of the full Vr genes)
  const int* gene_info;   // [V4] kind | sub << 2 | feat << 17 (zero padded to a multiple of 4)
  int compact;            // V < Vr: the compact layout (cmap / fidx are not identities)
  const int* ohe_off;     // [n_ohe+1]
  const int* ohe_feat;
  const int* mut_feat;    // [Dm]
  const int* fdec;        // [D] decoder: -1 immutable, else gene | (one-hot category + 1) << 16
  const double* ml_scale; // [D]
  const double* ml_min;   // [D]
  const double* mlS;      // [Dm4] ml_scale gathered at the mutable features
  const double* mlM;      // [Dm4] ml_min   gathered at the mutable features
  // constraint program, ops sorted by code (lane-uniform branches), ABS_SUMDIFF ops last
  const int* op_code;     // [C]
  const int* op_arg;      // [C*4]
  const double* op_k;     // [C*2]
  const int* op_col;      // [C] original constraint column of each sorted op
  const int* idx_pool;
  int n_pool;
  int n_sumdiff;          // ABS_SUMDIFF ops (positions C - n_sumdiff .. C-1), wave-parallel
  // k_vary LDS images (kernels.h vary_offsets): problem blob [vb] and per-state blobs [sb]
  const unsigned char* vblob;
  int full_ops;           // program uses the LCLD financial ops (codes 4..8)
  int ident;              // V == Dm, no one-hot genes, gene g <-> mutable feature g
  double tol;
  int norm;               // 2 or 0 (inf)
  int scale_obj;
  double f2_scale;        // 1/sqrt(D) for L2, 1 for Linf
  // classifier
  int n_layers;
  int dims[MAX_LAYERS + 1];
  const float* W[MAX_LAYERS];     // W[0]: mutable rows only, [Dm4][dims[1]] zero-padded
  const float* bias[MAX_LAYERS];  // bias[0] unused at run time (folded per state)
  // k_mlp2 weights: per hidden layer l, [K_l/16][N_l][16] (16 consecutive k of one output
  // column contiguous; K_0 = Dm4, K_l = dims[l]), so one dwordx4 load is a lane's B operand
  // for four 16x16x4 MFMA k-steps
  const float* Wp[MAX_LAYERS];  // also k_mlpw32's (fp32 wide nets); NULL unless packed
  int mlp2;               // hidden widths fit k_mlp2 (multiples of 16, <= 128)
  // bf16 perf mode (mv_set_mlp_precision, opt-in; fp32 is the parity default): the hidden
  // layers' weights as bf16 bits packed [K/32][N][32] (K zero padded to a multiple of 32:
  // 32 consecutive k of one output column contiguous, so one dwordx4 is a lane's B operand of
  // v_mfma_f32_16x16x32_bf16); activations are rounded to bf16 as they are read, fp32
  // accumulation, final Dense + softmax unchanged
  const unsigned short* Wb[MAX_LAYERS];
  int mlp_bf16;
  // k_mlp2 builds its layer-0 tiles straight from the child genes (IDENT problems: gene g
  // is mutable feature g), so k_gen writes no fp32 ML row: the xml hand-off (Dm4 * 4 B
  // written + read back per row) is gone
  int xml_direct;
  // every lane op of the constraint program is DIFF or RATIO_SAFE, at most OPS_REG per lane
  // (rowops.h), plus ABS_SUMDIFF ops: k_genc's phase 2 stages the slim region S of the
  // problem blob instead of region A (7-10 KiB less LDS per workgroup); tol >= 0
  int slim;
  // slim, with at most SD_REG ABS_SUMDIFF ops of at most 64 pool entries per side: each
  // lane's operands of those ops are LDS addresses held in registers (rowops.h
  // constraints_slim)
  int sd_reg;
};

struct DStates {
  int B;
  const double* x_init;     // [B][D]
  const double* gl;         // [B][V]
  const double* gu;         // [B][V]
  const unsigned char* sblob;  // [B][sb]: encoder scale/min and scaled origin at the
                               // mutable features [Dm4] each, then x_init [D] (kernels.h)
  const float* bias1;       // [B][H1]
  const int* min_class;     // [B]
};

// Row-tile evaluation (optionally preceded by variation) -----------------------------
struct RowsArgs {
  DProblem p;
  DStates s;
  int n;                    // rows per state
  int total;                // B * n
  int states_all;           // the attack's states over all its state groups (row chunking)
  int mode;                 // 0: genes given; 1: crossover + mutation from parents
  const double* genes_in;   // mode 0: [B][in_rows][V]; mode 1: parent pool [B][in_rows][V]
  int in_rows;              // rows per state in genes_in
  const int* parents;       // mode 1: [B][n/2][2] row indices into genes_in
  double* genes_out;        // [B][out_rows][V] or NULL
  int out_rows;
  const int* out_map;       // [B][n] destination row per evaluated row (NULL: identity)
  double* F;                // [B][out_rows][3] (rows follow out_map) or NULL
  double* G;                // [B][n][C] or NULL
  double* hist;             // [B][hist_rows][hist_w] or NULL
  int hist_rows, hist_w;
  uint64_t seed;
  uint32_t stream_key;
  int state_keys;           // 1: state b draws from stream stream_key + key0 + b (per-state
  uint32_t key0;            //    streams, mv_set_state_streams); 0: every state shares stream_key
  double eta;               // 20
  double cx_prob;           // 0.9
  int cx_kind;              // 0: two-point (the reference), 1: SBX (north_star option)
  double sbx_eta;           // SBX distribution index (30)
  int do_eval;              // 0: variation only
  float* xml;               // scratch [total][Dm4]: fp32 ML rows between k_vary and k_mlp
  long long* gphase;        // development (MV_GEN_PHASES): k_genc clocks [grid][8], or NULL
  long long* mphase;        // development (MV_MLP_PHASES): k_mlp2 clocks [grid][8]
  // mode 1 under k_genc: the generation's variation plan, written by the previous k_survive
  // (VPlan below); NULL: the row kernels draw the crossover / mutations themselves
  const int4* plan_hdr;     // [B][n]
  const int* plan_mw;       // [B][n][PLAN_MUT]
  const double* plan_mu;    // [B][n][PLAN_MUT]
};

// Variation plan of one generation (k_survive's tail -> k_genc): every draw of the row
// kernels' variation that does not depend on gene values, per offspring row i of a state
// (mating m = i % (n / 2), side = i / (n / 2)):
//   hdr  int4: x = parents packed (own | other << 16, pool slots), y / z = the real / int
//        subsets' crossover draws (pack_cx: on | lo << 1 | hi << 16; SBX: on only),
//        w = stored mutations count (<= PLAN_MUT) | overflow << 4 (the row has more: the row
//        kernel redoes it with every mutation)
//   mw   [PLAN_MUT] int: stored gene (bits 0-15) | real << 16 | from the other parent << 17
//        (two-point: the gene lies in its subset's crossover segment)
//   mu   [PLAN_MUT] double: the mutation's PM uniform
// The draws are the ones the row kernels used to make (the same Philox indices and tags), so
// the populations are bit-identical; only the gene value a mutation applies to, and its
// det_pow, stay in the row kernel.
constexpr int PLAN_MUT = 8;
// k_survive stages the plan's tables in LDS: geo [Vr + 1], cmap [Vr], ginfo [V] words
__host__ __device__ inline int plan_tab_words(int Vr, int V) { return 2 * Vr + 1 + V; }

// Survival ------------------------------------------------------------------------------
struct SurvArgs {
  int N;                    // merged individuals
  int n_survive;
  int P;                    // population part of the merge (slot mode)
  int O;                    // offspring part (slot mode)
  const double* F;          // dense: [B][N][3]; slot mode: pool F [B][S][3]
  int S;                    // slots per state (slot mode)
  const int* pop_slot;      // slot mode: [B][P]   (NULL -> dense mode)
  int* free_slot;           // slot mode: [B][O]   (read, then rewritten)
  int* pop_slot_out;        // slot mode: [B][n_survive]
  const double* ref;        // [R][3]
  int R;
  double mu;
  uint64_t seed;
  int gen;
  uint32_t stream_key;
  int state_keys;           // as RowsArgs
  uint32_t key0;
  double* ideal;            // [B][3]
  double* worst;            // [B][3]
  double* extreme;          // [B][9]
  int* has_extreme;         // [B]
  int* survivors;           // dense: [B][n_survive] merged indices
  int* rank;                // [B][N]
  int* order;               // [B][N]
  int* n_ranked;            // [B]
  int* niche;               // [B][N]
  double* dist;             // [B][N]
  double* nadir;            // [B][3]
  int* parents_out;         // [B][n_m][2] (slots in slot mode, positions otherwise) or NULL
  int O_next;               // offspring of the next generation (selection)
  int sel_gen;
  long long* phase;         // [B][16] clock64() at phase boundaries (development), or NULL
  unsigned long long* dom_g;  // N > SURV_NLDS: dominance bitsets [B][dom_stride] in HBM
  size_t dom_stride;
  // next generation's variation plan (RowsArgs VPlan), written after the tournament when
  // plan_hdr != NULL: rows per state O_next, the attack layout's tables and crossover options
  int4* plan_hdr;
  int* plan_mw;
  double* plan_mu;
  const uint32_t* geo;      // [Vr + 1] geometric gap table (problem blob region B)
  const int* cmap;          // [Vr] gene -> stored gene (-1 fixed)
  const int* ginfo;         // [V] stored gene info (kind | subset index << 2 | ...)
  int Vr, V, n_sub0, n_sub1;
  double cx_prob;
  int cx_sbx;               // SBX: the subsets' mating-level draws only
  int wide;                 // N <= SURV_NLDS: SURV_T_MID threads per state instead of SURV_T
};

// Stand-alone classifier forward (Classifier.predict_proba) -------------------------------
struct MlpArgs {
  int n_layers;
  int dims[MAX_LAYERS + 1];
  const float* W[MAX_LAYERS];     // W[0] zero-padded to D4 rows
  const float* bias[MAX_LAYERS];
  int D4;
  int n;
  const double* x;                // [n][D] ML-scaled rows
  double* proba;                  // [n][n_out]
};

// ObjectiveCalculator._calculate_objective (objectives.hip) -------------------------------
struct ObjArgs {
  long total;                     // B * n rows
  int n;                          // rows per state
  int D, C, n_ohe, n_out, cls, norm;
  const double* x;                // [B][n][D] ML-space candidates
  const double* x_init;           // [B][D]
  const double* mm_scale;         // [D] min_max_scaler (distance)
  const double* mm_min;           // [D]
  const int* ohe_off;             // [n_ohe+1] full-type-mask one-hot groups
  const int* ohe_feat;
  const double* G;                // [B*n][C] constraints (tol-clamped)
  const double* proba;            // [B*n][n_out]
  double* obj;                    // [B][n][3]: CV, f1, f2
  int* range_bad;                 // [B][n]: scaled row or origin outside [-1e-4, 1+1e-4]
};

}  // namespace mv
