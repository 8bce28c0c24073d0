// Whole-attack kernel (gfx950), shared body of attack_ident.hip / attack_ohe.hip: one workgroup per initial state runs the entire MoEvA2 GA
// loop of Moeva2._one_generate + pymoo.minimize (src/attacks/moeva2/moeva2.py:128-171) --
// evaluate the initial population, then (n_gen - 1) x {crossover + mutation + evaluation
// of the offspring, R-NSGA-III survival + the next tournament} -- in ONE launch.
//
// Initial states are independent (moeva2.py:194-205), so a state needs no other
// workgroup's data: its generation chain is a sequence of workgroup phases separated by
// barriers instead of four kernel launches per generation.  Two workgroups share a CU
// (LDS <= 80 KiB, <= 128 VGPRs), so one state's latency-bound survival overlaps the other
// state's HBM / MFMA-bound evaluation on the same CU.
//
// Phases (per state, per generation):
//   rows_state  variation (mode 1) or gene load (mode 0) of the generation's rows, one row per
//               wave at a time: child genes -> pool, f2 (encoder MinMax distance), the fp32
//               ML-scaled row -> xml, the ML-space row -> the wave's LDS row buffer ->
//               constraint program -> f3 (default_problem.py:99-140 minus the classifier).
//               The child genes are read once (parents) and written once.
//   mlp_state   the Dense-ReLU chain on v_mfma_f32_16x16x4_f32 over 64-row tiles of the
//               state's xml rows, final Dense + softmax -> f1 (classifier.py:23-29).
//   survive_state (survival.h) survival + tournament, state carried in HBM slots.
// Every phase reuses the per-phase kernels' arithmetic unchanged (rowops.h, survival.h), so
// the attack is bit-identical to the k_gen/k_cons/k_mlp2/k_survive chain (tested).
#pragma once
#include <mutex>

#include "engine.h"
#include "kernels.h"
#include "philox.h"
#include "rowops.h"
#include "rows_fused.h"
#include "survival.h"
#include "wave.h"

namespace mv {

// per translation unit: the constant-memory argument ring of this TU's kernels
static __constant__ AttackArgs c_att[ATT_SLOTS];

namespace {
struct AttRing {
  bool ready = false;
  AttackArgs* host = nullptr;  // pinned [ATT_SLOTS]
  hipEvent_t ev[ATT_SLOTS] = {};
  int next = 0;
};
constexpr int ATT_MAX_DEV = 64;
AttRing g_att[ATT_MAX_DEV];
std::mutex g_att_mu;
}  // namespace

// ---------------------------------------------------------------------------------------
// Classifier phase: k_mlp2's Dense chain over the n xml rows of one state (64-row tiles),
// with T threads.  Same k order, same final-layer split into four k quarters, so f1 is
// bit-identical to k_mlp2's.
__device__ __forceinline__ TileMap tile_map_w(int nct, int wave, int W) {
  const int cw = nct >= 3 ? 4 : nct;
  const int groups = W / cw;
  int nrt = 4 / groups;
  if (nrt < 1) nrt = 1;
  const int g = wave / cw;
  const int rt0 = g * nrt;
  return TileMap{wave % cw, rt0, rt0 < 4 ? nrt : 0};
}

template <int CJ, int T>
__device__ __forceinline__ void mlp_state(const RowsArgs& a, const int b, const int hist_row0,
                                          unsigned char* smem) {
  constexpr int W = T / 64;
  const DProblem& p = a.p;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int il = lane & 15, ka = lane >> 4;
  const int nl = p.n_layers;
  const int K0 = p.Dm4, N0 = p.dims[1];
  const int hld = mlp2_hmax(p) + 4;
  const int Klast = p.dims[nl - 1], nout = p.dims[nl];
  int* rowst = (int*)smem;
  float* wl = (float*)(smem + 256);
  float* bl = wl + Klast * nout;
  float* A0 = (float*)(smem + mlp2_head(p));
  float* H = A0;
  for (int q = tid; q < Klast * nout; q += T) wl[q] = p.W[nl - 1][q];
  if (tid < nout) bl[tid] = p.bias[nl - 1][tid];
  const int n = a.n;
  const size_t rbase = (size_t)b * (a.xml_rows ? a.xml_rows : n);  // the state's first xml row
  const int ntiles = (n + M2_ROWS - 1) / M2_ROWS;
  const int nkg0 = K0 >> 4;
  const int nch = (nkg0 + 3) >> 2;
  constexpr int U = 1024 / T;  // float4 per thread per 64 x 64 chunk
  for (int tile = 0; tile < ntiles; ++tile) {
    const int r0 = tile * M2_ROWS;
    // staging registers as plain locals (a lambda-captured array is address-taken -> scratch)
    float4 st0, st1, st2, st3;
    static_assert(U <= 4, "chunk staging holds at most 4 float4 per thread");
#define MS_CHUNK_LOAD(c)                                                                 \
  {                                                                                      \
    const int cc = (c);                                                                  \
    float4* sts[4] = {&st0, &st1, &st2, &st3};                                           \
    _Pragma("unroll") for (int u = 0; u < U; ++u) {                                      \
      const int idx = tid + T * u;                                                       \
      const int row = idx >> 4, q = idx & 15;                                            \
      const int k = cc * 64 + 4 * q < K0 ? cc * 64 + 4 * q : K0 - 4;                     \
      const int rr = r0 + row < n ? r0 + row : n - 1;                                    \
      *sts[u] = *(const float4*)(a.xml + (rbase + rr) * K0 + k);                         \
    }                                                                                    \
  }
#define MS_CHUNK_STORE(buf)                                                              \
  {                                                                                      \
    const float4 vs[4] = {st0, st1, st2, st3};                                           \
    _Pragma("unroll") for (int u = 0; u < U; ++u) {                                      \
      const int idx = tid + T * u;                                                       \
      const int row = idx >> 4, q = idx & 15;                                            \
      *(float4*)(A0 + (buf) * M2_ROWS * M2_ALD + row * M2_ALD + 4 * q) = vs[u];           \
    }                                                                                    \
  }
    MS_CHUNK_LOAD(0)
    __syncthreads();  // the previous tile's (or phase's) readers of the LDS are done
    if (tid < M2_ROWS) rowst[tid] = r0 + tid < n ? b : -1;
    MS_CHUNK_STORE(0)
    __syncthreads();
    floatx4 acc[CJ][4];
#pragma unroll
    for (int cj = 0; cj < CJ; ++cj)
#pragma unroll
      for (int rt = 0; rt < 4; ++rt) acc[cj][rt] = floatx4{0.f, 0.f, 0.f, 0.f};
    const TileMap m0 = tile_map_w(N0 >> 4, wave, W);
    for (int c = 0; c < nch; ++c) {
      if (c + 1 < nch) MS_CHUNK_LOAD(c + 1)
      const int ng = min(4, nkg0 - 4 * c);
      if (m0.nrt > 0)
        mlp2_layer<CJ>(A0 + (c & 1) * M2_ROWS * M2_ALD, M2_ALD,
                       p.Wp[0] + (size_t)4 * c * N0 * 16, ng, N0, acc, m0, il, ka);
      if (c + 1 < nch) MS_CHUNK_STORE((c + 1) & 1)
      __syncthreads();
    }
#undef MS_CHUNK_LOAD
#undef MS_CHUNK_STORE
    for (int l = 0; l + 1 < nl; ++l) {
      const int N = p.dims[l + 1];
      const TileMap m = tile_map_w(N >> 4, wave, W);
      if (l > 0) {
#pragma unroll
        for (int cj = 0; cj < CJ; ++cj)
#pragma unroll
          for (int rt = 0; rt < 4; ++rt) acc[cj][rt] = floatx4{0.f, 0.f, 0.f, 0.f};
        if (m.nrt > 0)
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
              const float bv = l == 0 ? a.s.bias1[(size_t)b * N0 + col] : p.bias[l][col];
              const float v = acc[cj][rt][j] + bv;
              out[row * hld + col] = v > 0.f ? v : 0.f;
            }
          }
        }
      }
      __syncthreads();
    }
    float* part = mlp2_part_inplace(p) ? H + ((nl - 1) & 1) * M2_ROWS * hld
                                       : A0 + mlp2_region_floats(p);
    if (wave < 4) {
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
    if (tid < M2_ROWS && r0 + tid < n) {
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
      const double f1 = softmax_pick(z, nout, mx, a.s.min_class[b]);
      const int i = r0 + tid;
      if (a.F) {
        const int orow = a.out_map ? a.out_map[(size_t)b * n + i] : i;
        a.F[((size_t)b * a.out_rows + orow) * 3] = f1;
      }
      if (a.hist) a.hist[((size_t)b * a.hist_rows + hist_row0 + i) * a.hist_w] = f1;
    }
  }
}

// ---------------------------------------------------------------------------------------
// The phases are separate (non-inlined) functions: inlined into one body, the register
// allocator kept hundreds of argument scalars live across the generation loop and spilled
// them (SGPRs into VGPRs, VGPRs into scratch), even with the argument pointer laundered per
// generation (opaque() below).
// The argument block is addressed through the TU's __constant__ array inside each phase,
// so its fields are scalar loads (through a generic pointer they became flat loads, each a
// VMEM round trip on every use).  b / gen / slot are wave-uniform: readfirstlane says so.
template <bool IDENT, int NT, bool FULL, int T>
__device__ __noinline__ void rows_phase(int slot, int va, int b, int gen, int h0) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  slot = __builtin_amdgcn_readfirstlane(slot);
  const AttackArgs& A = c_att[slot];
  const RowsArgs& a = __builtin_amdgcn_readfirstlane(va) ? A.va : A.ev;
  rows_state<IDENT, NT, FULL, T>(a, __builtin_amdgcn_readfirstlane(b),
                                 __builtin_amdgcn_readfirstlane(gen),
                                 __builtin_amdgcn_readfirstlane(h0), 0, a.n, smem);
}
template <int CJ, int T>
__device__ __noinline__ void mlp_phase(int slot, int va, int b, int h0) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  slot = __builtin_amdgcn_readfirstlane(slot);
  const AttackArgs& A = c_att[slot];
  mlp_state<CJ, T>(__builtin_amdgcn_readfirstlane(va) ? A.va : A.ev,
                   __builtin_amdgcn_readfirstlane(b), __builtin_amdgcn_readfirstlane(h0), smem);
}
template <int NWMAX, int T>
__device__ __noinline__ void survive_phase(int slot, int b, int N, int gen, int next) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  slot = __builtin_amdgcn_readfirstlane(slot);
  const AttackArgs& A = c_att[slot];
  survive_state<NWMAX, T>(A.sa, __builtin_amdgcn_readfirstlane(b),
                          __builtin_amdgcn_readfirstlane(N), __builtin_amdgcn_readfirstlane(gen),
                          __builtin_amdgcn_readfirstlane(gen) + 1,
                          __builtin_amdgcn_readfirstlane(next) ? A.parents : nullptr, smem);
}

// T threads per workgroup; two workgroups per CU (min 2 T / 256 waves per SIMD).
#ifndef MV_SKIP_ROWS
#define MV_SKIP_ROWS 0
#endif
#ifndef MV_SKIP_MLP
#define MV_SKIP_MLP 0
#endif
#ifndef MV_SKIP_SURV
#define MV_SKIP_SURV 0
#endif
typedef const AttackArgs __attribute__((address_space(4)))* CAtt;

// Phase boundary: the phases hand data to each other through global memory (xml rows -> the
// classifier, F -> survival, tournament parents / slots -> the next variation), written by
// some waves and read by others.  A workgroup barrier alone does not wait for a wave's
// outstanding stores, so every wave drains its memory counters first.
__device__ __forceinline__ void phase_barrier() {
  __builtin_amdgcn_s_waitcnt(0);
  __syncthreads();
}
__device__ __forceinline__ CAtt opaque(CAtt p) {
  uint64_t v = (uint64_t)p;
  asm volatile("" : "+s"(v));
  return (CAtt)v;
}

template <bool IDENT, int NT, bool FULL, int CJ, int NWMAX, int T>
__global__ __launch_bounds__(T, 2 * T / 256) void k_attack(int slot) {
  const CAtt A0 = (CAtt)&c_att[slot];
  const int B = A0->B, P = A0->P, O = A0->O, G = A0->G;
  long long* const prof = A0->prof;
  long long t_rows = 0, t_mlp = 0, t_surv = 0, t0 = 0, t1 = 0;
#define MV_STAMP(acc)                    \
  if (prof) {                            \
    t1 = clock64();                      \
    acc += t1 - t0;                      \
    t0 = t1;                             \
  }
  for (int b = blockIdx.x; b < B; b += gridDim.x) {
    if (prof) t0 = clock64();
    const long long tb = t0;
    // generation 0: pymoo _initialize -- evaluate the initial population, survival with
    // n_survive == len(pop) (sets ideal/worst/extremes), first tournament
    if (!MV_SKIP_ROWS) rows_phase<IDENT, NT, FULL, T>(slot, 0, b, 0, 0);
    phase_barrier();
    MV_STAMP(t_rows)
    if (!MV_SKIP_MLP) mlp_phase<CJ, T>(slot, 0, b, 0);
    phase_barrier();
    MV_STAMP(t_mlp)
    if (!MV_SKIP_SURV) survive_phase<NWMAX, T>(slot, b, P, 0, G > 1);
    phase_barrier();
    MV_STAMP(t_surv)
    for (int g = 1; g < G; ++g) {
      const int h0 = P + (g - 1) * O;
      if (!MV_SKIP_ROWS) rows_phase<IDENT, NT, FULL, T>(slot, 1, b, g, h0);
      phase_barrier();
      MV_STAMP(t_rows)
      if (!MV_SKIP_MLP) mlp_phase<CJ, T>(slot, 1, b, h0);
      phase_barrier();
      MV_STAMP(t_mlp)
      if (!MV_SKIP_SURV) survive_phase<NWMAX, T>(slot, b, P + O, g, g + 1 < G);
      phase_barrier();
      MV_STAMP(t_surv)
    }
    if (prof && threadIdx.x == 0) {
      prof[(size_t)b * 4 + 0] = t_rows;
      prof[(size_t)b * 4 + 1] = t_mlp;
      prof[(size_t)b * 4 + 2] = t_surv;
      prof[(size_t)b * 4 + 3] = t0 - tb;
    }
    t_rows = t_mlp = t_surv = 0;
  }
#undef MV_STAMP
}

// Stage `args` in this TU's constant ring (stream-ordered) and launch k_attack<...>: every
// state resident when it fits (two workgroups per CU), else workgroups loop over states.
template <bool I, int N, bool F, int C, int NW>
static hipError_t att_launch(const AttackArgs& args, size_t lds, int grid, hipStream_t stream) {
  int dev = 0;
  hipError_t e = hipGetDevice(&dev);
  if (e != hipSuccess) return e;
  if (dev < 0 || dev >= ATT_MAX_DEV) return hipErrorInvalidDevice;
  std::lock_guard<std::mutex> lock(g_att_mu);
  static bool configured = false;
  if (!configured) {
    (void)hipFuncSetAttribute((const void*)k_attack<I, N, F, C, NW, ATT_T>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    (void)hipGetLastError();
    configured = true;
  }
  AttRing& r = g_att[dev];
  if (!r.ready) {
    e = hipHostMalloc((void**)&r.host, ATT_SLOTS * sizeof(AttackArgs));
    for (int i = 0; i < ATT_SLOTS && e == hipSuccess; ++i)
      e = hipEventCreateWithFlags(&r.ev[i], hipEventDisableTiming);
    if (e != hipSuccess) return e;
    r.ready = true;
  }
  const int slot = r.next;
  r.next = (r.next + 1) % ATT_SLOTS;
  e = hipEventSynchronize(r.ev[slot]);  // the slot's previous launch has finished
  if (e != hipSuccess) return e;
  r.host[slot] = args;
  e = hipMemcpyToSymbolAsync(HIP_SYMBOL(c_att), r.host + slot, sizeof(AttackArgs),
                             (size_t)slot * sizeof(AttackArgs), hipMemcpyHostToDevice, stream);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL((k_attack<I, N, F, C, NW, ATT_T>), dim3(grid), dim3(ATT_T), lds, stream,
                     slot);
  e = hipGetLastError();
  if (e != hipSuccess) return e;
  return hipEventRecord(r.ev[slot], stream);
}

}  // namespace mv
