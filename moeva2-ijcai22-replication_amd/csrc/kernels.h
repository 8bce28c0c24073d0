// Launch wrappers shared by the C-ABI layer (api.cpp) and the kernel files.
#pragma once
#include <hip/hip_runtime.h>

#include "engine.h"

namespace mv {

// LDS of k_rows: row bookkeeping + R1 (A tile / ping) + R2 (4 ML rows / pong).
__host__ __device__ inline size_t eval_region1_bytes(int Dm4, int hmax) {
  const size_t a = (size_t)EVAL_TR * (Dm4 + 1) * sizeof(float);
  const size_t h = (size_t)EVAL_TR * (hmax + 1) * sizeof(float);
  const size_t r = a > h ? a : h;
  return (r + 15) & ~(size_t)15;
}
__host__ __device__ inline size_t eval_lds_bytes(int D, int Dm4, int hmax) {
  const size_t head = (size_t)EVAL_TR * (2 * sizeof(int) + 2 * sizeof(double));
  const size_t rows = (size_t)4 * D * sizeof(double);
  const size_t h = (size_t)EVAL_TR * (hmax + 1) * sizeof(float);
  const size_t r2 = rows > h ? rows : h;
  return head + eval_region1_bytes(Dm4, hmax) + r2;
}

hipError_t launch_predict(const MlpArgs& a, hipStream_t stream);
__host__ __device__ inline size_t mlp_lds_bytes(int Dm4, int hmax) {
  return 256 + eval_region1_bytes(Dm4, hmax) + (size_t)EVAL_TR * (hmax + 1) * sizeof(float);
}

size_t surv_lds_bytes(int N, int R, int P);

hipError_t launch_rows(const RowsArgs& a, hipStream_t stream);
hipError_t launch_vary(const RowsArgs& a, hipStream_t stream);
hipError_t launch_mlp(const RowsArgs& a, hipStream_t stream);
hipError_t launch_constraints(const DProblem& p, int n, const double* x, double* G,
                              hipStream_t stream);
hipError_t launch_variation(const RowsArgs& a, hipStream_t stream);
hipError_t launch_setup_states(const DProblem& p, int B, const double* x_init, const double* xl,
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
