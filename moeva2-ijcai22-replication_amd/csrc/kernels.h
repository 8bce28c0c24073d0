// Launch wrappers shared by the C-ABI layer (api.cpp) and the kernel files.
#pragma once
#include <hip/hip_runtime.h>

#include "engine.h"

namespace mv {

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

hipError_t launch_predict(const MlpArgs& a, hipStream_t stream);

// Launch-argument ring (constant memory, per device): stage a copy on `stream`, launch with
// the returned slot, then release it on the same stream after the slot's last launch.
hipError_t stage_rows(const RowsArgs& a, hipStream_t stream, int* slot);
hipError_t release_rows(int slot, hipStream_t stream);
size_t surv_lds_bytes(int N, int R, int P);

hipError_t launch_vary(const RowsArgs& a, int slot, int gen, int hist_row0,
                       hipStream_t stream);
hipError_t launch_mlp(const RowsArgs& a, int slot, int hist_row0, hipStream_t stream);
hipError_t launch_rows(const RowsArgs& a, int slot, int gen, int hist_row0,
                       hipStream_t stream);
hipError_t launch_constraints(const DProblem& hp, int slot, int n, const double* x,
                              double* G, hipStream_t stream);
hipError_t launch_setup_states(int slot, int B, const double* x_init, const double* xl,
                               const double* xu, const float* W1full, const float* b1, double* gl,
                               double* gu, double* enc_scale, double* enc_min, double* x0_mm,
                               float* bias1, double* genes0, hipStream_t stream);
hipError_t launch_survive(const SurvArgs& a, int B, hipStream_t stream);
hipError_t launch_select(int B, int P, int O, uint64_t seed, uint32_t stream_key, int gen,
                         const int* pop_slot, int* parents, hipStream_t stream);
hipError_t launch_init_pool(int B, int P, int O, int V, int S, const double* genes0,
                            double* pool, int* pop_slot, int* free_slot, hipStream_t stream);
hipError_t launch_gather_pop(int B, int P, int V, int S, const int* pop_slot, const double* pool,
                             const double* poolF, double* genes, double* F, hipStream_t stream);

}  // namespace mv
