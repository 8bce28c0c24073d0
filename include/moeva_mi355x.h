/*
 * moeva_mi355x.h -- C ABI of the MI355X-native MoEvA2 engine (libmoeva_mi355x.so).
 *
 * The reference is pure Python: its hot path is reached through
 *   Moeva2.generate(x, minimize_class)             src/attacks/moeva2/moeva2.py:174-207
 *   DefaultProblem._evaluate(x, out)               src/attacks/moeva2/default_problem.py:99-140
 * and, inside pymoo 0.4.2.2 (not vendored), R-NSGA-III survival + mating.  Each entry
 * point below replaces one of those surfaces; the Python host package
 * (moeva2_amd.attacks.moeva2.*) binds them with ctypes exactly as a maintainer would add
 * to the reference.
 *
 * Conventions
 *  - status codes (MV_OK == 0); mv_last_error() returns a thread-local message;
 *  - no exceptions cross the ABI; no torch types; plain pointers and sizes;
 *  - pointers documented "dev" are device (HBM) pointers owned by the caller
 *    (e.g. torch tensors' data_ptr()); "host" pointers are read synchronously;
 *  - every launch is ordered on the caller's hipStream_t (passed as void*; NULL = default
 *    stream) and is asynchronous unless stated;
 *  - one mv_engine per (device, problem); an engine is thread-compatible, not thread-safe.
 */
#ifndef MOEVA_MI355X_H
#define MOEVA_MI355X_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

enum {
  MV_OK = 0,
  MV_ERR_ARG = 1,   /* invalid argument / shape */
  MV_ERR_HIP = 2,   /* HIP runtime error */
  MV_ERR_STATE = 3, /* call out of order (e.g. no states bound) */
};

/* gene kinds (feature_encoder.py:169-181 get_type_mask_genetic) */
enum { MV_GENE_REAL = 0, MV_GENE_INT = 1, MV_GENE_OHE = 2 };

/* constraint op codes: one op == one constraint column, evaluated on the ML-space row
 * x_f (default_problem.py:93-97 then constraints.evaluate numpy path). */
enum {
  MV_OP_DIFF = 1,          /* x[a0] - x[a1]                        botnet_constraints.py:283-285 */
  MV_OP_RATIO_SAFE = 2,    /* (x[a1]!=0 ? x[a0]/x[a1] : 0) - k0     botnet_constraints.py:304-306 */
  MV_OP_ABS_SUMDIFF = 3,   /* |sum(pool[a0:a1]) - sum(pool[a1:a2])| botnet_constraints.py:127-148 */
  MV_OP_LCLD_INSTALL = 4,  /* |x3 - x0 r (1+r)^x1/((1+r)^x1-1)| - k0, r=x2/1200  lcld:174-177 */
  MV_OP_LCLD_TERM = 5,     /* |(36-x[a0])(60-x[a0])|               lcld_constraints.py:186 */
  MV_OP_ABS_RATIO = 6,     /* |x[a0] - x[a1]/x[a2]|                lcld_constraints.py:189-207 */
  MV_OP_MONTHDIFF = 7,     /* |x[a0] - (month(x[a1]) - month(x[a2]))| lcld_constraints.py:195-201 */
  MV_OP_RATIO_MASKED = 8,  /* |x[a0] - (x[a2]==0|inf|nan ? -1 : x[a1]/x[a2])| lcld:210-216 */
  MV_OP_XOR_AUG = 9,       /* |x[a0] - xor(x[a1]>=k0, x[a2]>=k1)|  examples/utils.py:7-29 */
};

typedef struct mv_problem_desc {
  int32_t D;                  /* ML feature count */
  int32_t V;                  /* genetic length (n_var) */
  int32_t Dm;                 /* mutable feature count (mutable_mask.sum()) */
  int32_t C;                  /* constraint count */
  int32_t n_ohe;              /* mutable one-hot groups */
  const int32_t* gene_kind;   /* host [V] MV_GENE_* */
  const int32_t* gene_feat;   /* host [V] feature (REAL/INT) or group index (OHE) */
  const int32_t* ohe_offsets; /* host [n_ohe+1] CSR offsets into ohe_feats */
  const int32_t* ohe_feats;   /* host [..] features of each group, category order */
  const int32_t* mut_feats;   /* host [Dm] mutable features, ascending */
  const double* ml_scale;     /* host [D] ML MinMaxScaler scale_ (NULL: identity) */
  const double* ml_min;       /* host [D] ML MinMaxScaler min_   (NULL: identity) */
  const int32_t* op_code;     /* host [C] MV_OP_* */
  const int32_t* op_arg;      /* host [C*4] integer operands */
  const double* op_karg;      /* host [C*2] real operands */
  int32_t n_pool;             /* index pool size for MV_OP_ABS_SUMDIFF */
  const int32_t* idx_pool;    /* host [n_pool] */
  double tol;                 /* constraints <= tol -> 0  (1e-3 in every reference class) */
  int32_t norm;               /* 2 = L2, 0 = Linf  (default_problem.py:80-91) */
  int32_t scale_objectives;   /* f2 MinMax scaling (utils.py:11-22) */
} mv_problem_desc;

typedef struct mv_model_desc {
  int32_t n_layers;           /* Dense layers; hidden relu, last softmax */
  const int32_t* dims;        /* host [n_layers+1], dims[0] == D */
  const float* const* W;      /* host per layer [dims[l] x dims[l+1]] row-major (Keras kernel) */
  const float* const* b;      /* host per layer [dims[l+1]] */
} mv_model_desc;

typedef struct mv_engine mv_engine;

const char* mv_last_error(void);
int mv_device_count(int32_t* n);

/* Upload problem constants + classifier weights to `device`.  model may be NULL: a
 * constraints-only engine, or the engine behind a host classifier plugin (mv_evaluate then
 * leaves f1 to the caller; mv_attack_run needs a model). */
int mv_engine_create(int32_t device, const mv_problem_desc* problem, const mv_model_desc* model,
                     mv_engine** out);
void mv_engine_destroy(mv_engine* e);

/* Bind B initial states (host arrays, copied).  xl/xu are the per-state feature bounds
 * Constraints.get_feature_min_max(dynamic_input=x) (moeva2.py:141-142).  Derives on device:
 * encoder MinMax (feature_encoder.py:39-40), genetic bounds (:145-163), the initial
 * genetic vector (sampling.py:64-78) and the immutable-feature fold of the first layer. */
int mv_set_states(mv_engine* e, int32_t B, const double* x_init, const double* xl,
                  const double* xu, const int32_t* minimize_class, void* stream);

/* DefaultProblem._evaluate for n rows per bound state.
 * genes dev [B][n][V] -> F dev [B][n][3] (f1 misclassification, f2 distance, f3 constraint sum);
 * G dev [B][n][C] (constraint values after the tol clamp and G*(G>0)) or NULL. */
int mv_evaluate(mv_engine* e, int32_t n, const double* genes, double* F, double* G, void* stream);

/* FeatureEncoder.genetic_to_ml (feature_encoder.py:129-130) on device, for host-evaluated
 * plugins (a Constraints subclass without a device program, a non-Dense classifier):
 * genes dev [B][n][V] -> x dev [B][n][D] with the bound states' x_init. */
int mv_decode(mv_engine* e, int32_t n, const double* genes, double* x, void* stream);

/* Every entry point taking device buffers fails with MV_ERR_ARG when a buffer is device
 * memory of another GPU than the engine's (mlp's, objcalc's; for mv_survive and
 * mv_select_parents, which take no engine: the current device's). */
/* Constraints.evaluate (numpy path: values <= tol set to 0) on ML-space rows:
 * x dev [n][D] -> G dev [n][C].  Works on an engine created without a model. */
int mv_constraints(mv_engine* e, int32_t n, const double* x, double* G, void* stream);

/* R-NSGA-III AspirationPointSurvival._do + NonDominatedSorting + niching, batched over B
 * independent populations of N merged individuals (pymoo 0.4.2.2 rnsga3.py/nsga3.py).
 * F dev [B][N][3]; ref_points dev [R][3]; state in/out dev: ideal [B][3], worst [B][3],
 * extreme [B][3][3], has_extreme [B] (0 before the first call).
 * Outputs dev: survivors [B][n_survive] (merged indices, new population order),
 * rank [B][N] (front index, -1 = unranked) and, for the fronts-ordered individuals
 * (order [B][N], count n_ranked [B]): niche [B][N], dist [B][N].  Any output may be NULL
 * except survivors.  Requires N <= 1024 (above 512 the dominance bitsets live in an HBM
 * scratch), R <= 640. */
int mv_survive(int32_t B, int32_t N, int32_t n_survive, const double* F, int32_t R,
               const double* ref_points, double mu, uint64_t seed, int32_t gen,
               double* ideal, double* worst, double* extreme, int32_t* has_extreme,
               int32_t* survivors, int32_t* rank, int32_t* order, int32_t* n_ranked,
               int32_t* niche, double* dist, double* nadir, void* stream);

/* TournamentSelection(comp_by_cv_then_random) for B populations of P: parents dev
 * [B][ceil(O/2)][2] (population positions). */
int mv_select_parents(int32_t B, int32_t P, int32_t O, uint64_t seed, int32_t gen,
                      int32_t* parents, void* stream);

/* MixedVariableCrossover(two-point) + MixedVariableMutation(PM, eta 20), no evaluation:
 * pop dev [B][P][V], parents dev [B][O/2][2] -> off dev [B][O][V]. */
/* Crossover of mv_variation / mv_attack_run: kind 0 = two-point (moeva2.py:90-101, the
 * reference's operator; default), 1 = SBX (SimulatedBinaryCrossover, pymoo 0.4.2.2
 * real_sbx / int_sbx semantics with distribution index eta, prob_per_variable 0.5; the
 * stale comment at moeva2.py:87 names prob 0.9, eta 30).  prob: mating-level probability. */
int mv_set_crossover(mv_engine* e, int32_t kind, double eta, double prob);
int mv_variation(mv_engine* e, int32_t P, int32_t O, uint64_t seed, int32_t gen,
                 const double* pop, const int32_t* parents, double* off, void* stream);

/* Classifier.predict_proba (classifier.py:23-29) for a Dense(relu)...Dense(softmax)
 * model: x dev [n][dims[0]] (ML-scaled, fp64, cast to fp32 like Keras) -> proba dev
 * [n][n_out] fp64. */
typedef struct mv_mlp mv_mlp;
int mv_mlp_create(int32_t device, const mv_model_desc* model, mv_mlp** out);
void mv_mlp_destroy(mv_mlp* m);
int mv_mlp_predict(mv_mlp* m, int32_t n, const double* x, double* proba, void* stream);

/* ObjectiveCalculator._calculate_objective (objective_calculator.py:44-84) batched over B
 * initial states x n candidates (ML space), the scoring behind success_rate_3d (:106-119)
 * and get_successful_attacks (:152-223).  Per row: CV = calc_constraint_violation of
 * [constraints.evaluate(x) | get_one_hot_encoding_constraints(type_mask, x)] (utils.py:43-54),
 * f1 = predict_proba(ml_scaler(x))[:, minimize_class], f2 = ||mm(x_init) - mm(x)||_{2|inf}
 * on the min_max_scaler.  The constraint program is taken from a (model-less) engine, the
 * classifier from an mv_mlp. */
typedef struct mv_objcalc_desc {
  int32_t D;                  /* ML feature count */
  int32_t n_ohe;              /* one-hot groups of the FULL type mask, get_ohe_masks order */
  const int32_t* ohe_offsets; /* host [n_ohe+1] CSR offsets */
  const int32_t* ohe_feats;   /* host [..] features of each group */
  const double* mm_scale;     /* host [D] min_max_scaler scale_ (distance) */
  const double* mm_min;       /* host [D] min_max_scaler min_ */
  const double* ml_scale;     /* host [D] ml_scaler scale_, or NULL (ml_scaler None) */
  const double* ml_min;       /* host [D] or NULL */
  int32_t norm;               /* 2 = L2, 0 = Linf */
} mv_objcalc_desc;
typedef struct mv_objcalc mv_objcalc;
int mv_objcalc_create(int32_t device, const mv_objcalc_desc* desc, mv_objcalc** out);
void mv_objcalc_destroy(mv_objcalc* o);
/* x_init dev [B][D], x dev [B][n][D] -> obj dev [B][n][3] (CV, f1, f2) and range_bad dev
 * [B][n] (1 where the scaled row or origin leaves [-1e-4, 1+1e-4]: the reference asserts,
 * objective_calculator.py:72-76). */
int mv_objcalc_run(mv_objcalc* o, mv_engine* constraints, mv_mlp* classifier, int32_t B,
                   int32_t n, const double* x_init, const double* x, int32_t minimize_class,
                   double* obj, int32_t* range_bad, void* stream);
/* The same scoring with the constraint matrix and / or the class probabilities supplied by
 * the caller (device buffers): G dev [B*n][C] (Constraints.evaluate(x_f), C >= 0) and proba
 * dev [B*n][n_out].  This is the plugin path of ObjectiveCalculator._calculate_objective
 * (objective_calculator.py:44-84) for a Constraints subclass without a device program or a
 * predict_proba model that is not a Dense MLP: the host evaluates the plugin, the device
 * does the one-hot term, the CV sum, the ML/min-max scaling checks and the distance. */
int mv_objcalc_score(mv_objcalc* o, int32_t B, int32_t n, const double* x_init, const double* x,
                     const double* G, int32_t C, const double* proba, int32_t n_out,
                     int32_t minimize_class, double* obj, int32_t* range_bad, void* stream);
typedef struct mv_attack_params {
  int32_t n_gen;          /* Moeva2 n_gen (termination "n_gen") */
  int32_t pop_size;       /* P = n_ref_points + n_obj (203 for n_pop 200) */
  int32_t n_offsprings;   /* O (even) */
  uint64_t seed;          /* Moeva2 seed */
  int32_t n_ref;          /* R reference points */
  const double* ref_points; /* host [R][3] */
  double mu;              /* RNSGA3 mu (0.05) */
  int32_t history;        /* 0 none, 1 "reduced" (F), 2 "full" (F|G) */
} mv_attack_params;

/* Whole attack on device: init population + evaluate + (n_gen-1) x {select, vary+evaluate,
 * survive}, no host round trip.  Asynchronous on `stream`.  Replaces Moeva2.generate's
 * per-state pymoo.minimize calls (moeva2.py:128-171, 194-205) for ALL bound states.
 * Schedule: per generation the row kernel (k_genc for wide IDENT rows such as botnet,
 * k_narrow for LCLD-shaped rows, else k_gen + k_cons), the classifier (k_mlp2 / k_mlpw /
 * k_mlp) and k_survive (survival + the next tournament), the states split into up to 4
 * groups, each chain on its own stream. */
int mv_attack_run(mv_engine* e, const mv_attack_params* params, void* stream);
/* 0: auto (default), 1: per-phase kernel chain -- the same schedule.  2 (the retired
 * whole-attack kernel, measured slower than the chain) is rejected with MV_ERR_ARG. */
int mv_set_attack_mode(mv_engine* e, int32_t mode);
/* Random streams of the bound states (no reference counterpart; an engine option).
 * enabled = 0 (default, the reference's behaviour): every state draws from the same Philox
 * stream, as Moeva2 re-seeds each state's pymoo.minimize with the same seed
 * (moeva2.py:158-165).  enabled = 1: state b draws from its own stream, keyed by its GLOBAL
 * index first_state + b (pass the shard's offset under sharding, so results do not depend on
 * the GPU count).  Each state's attack is statistically the same either way; across states
 * the outcomes become independent, which is what the end-to-end parity test needs to resolve
 * 1 pp (tests/test_gpu_e2e.py).  Applies to mv_attack_run and mv_variation. */
int mv_set_state_streams(mv_engine* e, int32_t enabled, int64_t first_state);
/* Classifier precision of the engine's fitness path (mv_evaluate, mv_attack_run): 0 = fp32
 * (default; the parity mode: exact fp32 products on v_mfma_f32_16x16x4f32, as Keras computes
 * classifier.py:23-29), 1 = bf16 perf mode (hidden-layer weights and activations rounded to
 * bf16, fp32 accumulation on v_mfma_f32_16x16x32_bf16; f1 is no longer Keras's value, so
 * results are not parity results).  No reference counterpart: an engine option. */
int mv_set_mlp_precision(mv_engine* e, int32_t bf16);
/* Kept for ABI stability: the whole-attack kernel was retired, so *ms = 0 and *whole = 0. */
int mv_get_attack_time(mv_engine* e, double* ms, int32_t* whole);
/* Final population: genes dev [B][P][V], F dev [B][P][3] (either may be NULL). */
int mv_attack_population(mv_engine* e, double* genes, double* F, void* stream);
/* The final population's non-dominated members: the per-state result's X / F (moeva2.py:
 * 167-171 returns pymoo's Result, whose X / F are the last population's first front).  The
 * relation is pareto_operation.py:35-51's: i dominates j when F_i < F_j in some objective and
 * F_i > F_j in none; a member is in the front when no member of its state's final population
 * dominates it (the comparisons of a numpy any(<) / any(>) broadcast, so the mask is
 * bit-identical to one computed on the host from mv_attack_population's F).  Outputs dev:
 * front [B][P] uint8 (1 = member), offsets [B+1] int32 (state b's members are rows
 * offsets[b] .. offsets[b+1]-1, population order), X [B*P][V] / Fx [B*P][3] (worst-case size;
 * the first offsets[B] rows are written).  Any output may be NULL. */
int mv_attack_front(mv_engine* e, uint8_t* front, int32_t* offsets, double* X, double* Fx,
                    void* stream);
/* History rows per state = P + (n_gen-1)*O, width 3 (reduced) or 3+C (full): hist [B][rows][w]
 * a device buffer or page-locked host memory (hipHostMalloc / registered: one DMA). */
int mv_attack_history(mv_engine* e, double* hist, void* stream);
/* The attack's gene layout for the bound states (engine extension; no reference
 * counterpart).  mv_set_states finds the genes no attack on those states can change --
 * integer genes whose bounds are equal and whose initial value is that bound in every state
 * (crossover swaps equal values, mutation clamps back to the bound; botnet: 120 of 432) --
 * and the attack neither stores, moves nor sums them: their features are evaluated as
 * immutable features (decoded from x_init, folded into the layer-1 bias, absent from f2's
 * sum).  Every draw stays defined over all V genes, so the populations are those of the
 * full layout; f1 / f2 follow the engine's summation order over the stored genes
 * (oracle/device_order.py, `fixed`).  mv_evaluate / mv_decode / mv_variation always use
 * every gene.  stored (may be NULL) [V] receives 1 for a stored gene, 0 for a fixed one;
 * *n_stored the stored count (= V when nothing is fixed, or MV_COMPACT=0). */
int mv_get_stored_genes(mv_engine* e, int32_t* stored, int32_t* n_stored);
/* The layout mv_set_states would derive for B states (host arrays as mv_set_states; host
 * computation only, no device work): stored [V] 1 / 0 and *n_stored, as mv_get_stored_genes
 * reports after binding them. */
int mv_gene_layout(mv_engine* e, int32_t B, const double* x_init, const double* xl,
                   const double* xu, int32_t* stored, int32_t* n_stored);
/* Fix the layout of the NEXT mv_set_states call (one call only; the request is consumed by
 * it, refused or not, so a later binding on a shared engine derives its own): stored [V]
 * (1 = stored) as
 * mv_gene_layout returned it for the WHOLE job, so a job split into batches or shards
 * (Moeva2.generate_sharded) runs every state in the same layout -- a state's f1 / f2
 * summation order, hence its trajectory, then does not depend on which states share its
 * batch.  mv_set_states fails with MV_ERR_ARG when an unstored gene is not fixed in a bound
 * state.  stored = NULL returns to deriving the layout from each bound batch (default). */
int mv_set_gene_layout(mv_engine* e, const int32_t* stored, int32_t V);
/* Per-kernel timing of the last mv_attack_run when enabled (one state group then): each
 * profiled launch -- the row kernel(s), the classifier and k_survive of every generation --
 * is made with hipExtLaunchKernelGGL and a start / stop HIP event pair, which stamp the
 * kernel's own execution (no dispatch gap); summed ms.  A step that launches no kernel
 * (k_cons under k_genc / k_narrow) reads 0. */
int mv_set_profiling(mv_engine* e, int32_t enabled);
int mv_get_kernel_times(mv_engine* e, double* vary_ms, double* mlp_ms, double* survive_ms,
                        int32_t* n_generations);
/* Same events, split by kernel: ms[0] the row kernel's variation part (k_gen; k_genc or
 * k_narrow: the whole row kernel), ms[1] k_cons (constraints + f3; 0 when k_genc or k_narrow
 * ran), ms[2] the classifier (f1), ms[3] k_survive (survival + next tournament), summed over
 * the profiled generations. */
int mv_get_phase_times(mv_engine* e, double* ms, int32_t* n_generations);
/* The kernels an attack generation runs for its offspring rows under the engine's current
 * options: 0 = k_gen then k_cons, 1 = k_narrow (one lane per row, both in one launch; the
 * k_cons events then bracket nothing), 2 = k_genc (k_gen and k_cons as two phases of one
 * launch; likewise).  Lets a profiler attribute ms[0] + ms[1] of mv_get_phase_times. */
int mv_get_row_kernel(mv_engine* e, int32_t* kind);
/* The classifier kernel an attack generation runs: 0 = k_mlp (one tile of rows per
 * workgroup, any widths), 1 = k_mlp2 reading the child genes (no fp32 ML row is written),
 * 2 = k_mlp2 reading the fp32 ML rows, 4 = k_mlpw (bf16 weights), 5 = k_mlpw32 (fp32 wide
 * nets: 64-row tiles, one activation buffer), -1 = no device classifier
 * (3, the retired k_mlp2x, is no longer returned).
 * Lets a profiler price the ML-row bytes of the row kernel and the classifier. */
int mv_get_mlp_kernel(mv_engine* e, int32_t* kind);

/* Device index checks (debug builds compiled with -DMV_CHECKS, `make checks`): synchronises
 * the device, then returns and clears the first failed check of the row, classifier and
 * survival kernels since the last call -- record[0] check code (csrc/check.h; 0 = none),
 * [1] workgroup, [2] thread, [3] value, [4] bound, [5] number of failures -- and *compiled = 1
 * in a checks build (0 otherwise: record is all zero).  A checks build also fails
 * mv_attack_population with MV_ERR_STATE when a check failed.  No reference counterpart. */
int mv_debug_checks(int32_t* record, int32_t* compiled);
/* Checks builds: the inputs of the first survival whose survivors were not distinct (check
 * 26) -- out[3096] doubles: [0] 1 if valid, [1] generation, [2] state in its group, [3] N,
 * [4..6] carried ideal, [7..9] worst, [10..18] extremes, [19] has_extreme, [20] n_survive,
 * [21] seed (uint64 bits), [24..24+3N) merged F.  Cleared by the call; zeros otherwise. */
int mv_debug_survival_dump(double* out);

/* The engine's pow for the variation operators (host build of csrc/detmath.h det_pow, the
 * same IEEE operation sequence as the device code): out[i] = det_pow(x[i], y[i]) for host
 * arrays.  Replaces np.power in softmax_mutation.py:77-103 (polynomial mutation) and the
 * SBX option's calc_betaq; oracle/device_order.py:det_pow restates it. */
int mv_det_pow(int64_t n, const double* x, const double* y, double* out);

#ifdef __cplusplus
}
#endif
#endif /* MOEVA_MI355X_H */
