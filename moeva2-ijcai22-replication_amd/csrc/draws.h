// Variation draws shared by the row kernels (rowops.h) and k_survive's variation plan
// (survival.h): crossover segments, the geometric-gap mutation process.
#pragma once
#include <stdint.h>

#include "philox.h"

namespace mv {

constexpr int MUT_J = 1024;    // Philox indices per row of the mutation stream (V <= 1024)

// Crossover draws of one mating for one variable-type subset (oracle crossover_draws):
// on = u53 < prob; genes of the subset with index in [lo, hi) are swapped.
struct CxSub {
  int on, lo, hi;
};

__device__ __forceinline__ CxSub cx_sub(const Rng& rng, int gen, int m, int s, int n,
                                        double prob) {
  CxSub c{0, 0, 0};
  if (n <= 0) return c;
  const u32x4 w = rng.draw((uint32_t)(m * 2 + s), (uint32_t)gen, TAG_CX);
  c.on = u53(w.x, w.y) < prob;
  if (n - 1 <= 0) return c;
  const int a = 1 + (int)(((uint64_t)w.z * (uint64_t)(n - 1)) >> 32);
  if (n - 1 == 1) {
    c.lo = a;
    c.hi = n;
  } else {
    int b = 1 + (int)(((uint64_t)w.w * (uint64_t)(n - 2)) >> 32);
    if (b >= a) ++b;
    c.lo = a < b ? a : b;
    c.hi = a < b ? b : a;
  }
  return c;
}

// Geometric gap of the mutation process (oracle mutation_draws): the number of
// non-mutated genes before the next mutated one is the largest k in [0, V] with
// w < T[k], T[k] = floor((1 - 1/V)^k * 2^32) (T[0] unused), found by binary search.
__device__ __forceinline__ int geo_gap(const uint32_t* T, int V, uint32_t w, float lq) {
  // estimate from log2(w / 2^32) / log2(1 - 1/V), then step to the exact table answer
  int k = (int)(__log2f(((float)w + 0.5f) * 2.3283064365386963e-10f) / lq);
  k = k < 0 ? 0 : (k > V ? V : k);
  while (k < V && w < T[k + 1]) ++k;
  while (k > 0 && !(w < T[k])) --k;
  return k;
}

// Crossover draws of one subset packed into one word: on | lo << 1 | hi << 16.
__device__ __forceinline__ int pack_cx(const CxSub& c) { return c.on | (c.lo << 1) | (c.hi << 16); }
__device__ __forceinline__ bool swapped_packed(int info, int cx0, int cx1) {
  const int sub = (info >> 2) & 0x7FFF;
  const int c = (info & 3) == 0 ? cx0 : cx1;
  return (c & 1) && sub >= ((c >> 1) & 0x7FFF) && sub < (c >> 16);
}

}  // namespace mv
