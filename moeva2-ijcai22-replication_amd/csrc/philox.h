// Philox4x32-10 counter-based RNG for the MoEvA2 engine (gfx950).
//
// The reference draws from numpy's MT19937 inside pymoo, re-seeded with the same seed
// for every initial state (src/attacks/moeva2/moeva2.py:158-165).  The engine replaces
// that stream with Philox so every draw is a pure function of
//     key     = (seed lo32, seed hi32)
//     counter = (index, stream_key, generation, tag)
// which makes results independent of the state's position, the shard and the launch
// geometry.  oracle/philox.py states the same layout on the CPU.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace mv {

enum : uint32_t {
  TAG_SEL_PERM = 1,
  TAG_SEL_CHOICE = 2,
  TAG_CX = 3,
  TAG_MUT_MASK = 4,
  TAG_MUT_U = 5,
  TAG_NICHE_PERM = 6,
  TAG_NICHE_MEMBER = 7,
  TAG_SBX = 8,
};

struct u32x4 {
  uint32_t x, y, z, w;
};

__device__ __forceinline__ u32x4 philox(uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3,
                                        uint32_t k0, uint32_t k1) {
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    if (r) {
      k0 += 0x9E3779B9u;
      k1 += 0xBB67AE85u;
    }
    // one v_mad_u64_u32 per 32x32->64 product (hi and lo together)
    const uint64_t p0 = (uint64_t)0xD2511F53u * c0;
    const uint64_t p1 = (uint64_t)0xCD9E8D57u * c2;
    const uint32_t n0 = (uint32_t)(p1 >> 32) ^ c1 ^ k0;
    const uint32_t n2 = (uint32_t)(p0 >> 32) ^ c3 ^ k1;
    c0 = n0;
    c1 = (uint32_t)p1;
    c2 = n2;
    c3 = (uint32_t)p0;
  }
  return {c0, c1, c2, c3};
}

struct Rng {
  uint32_t k0, k1, sk;
  __device__ __forceinline__ Rng(uint64_t seed, uint32_t stream_key)
      : k0((uint32_t)seed), k1((uint32_t)(seed >> 32)), sk(stream_key) {}
  __device__ __forceinline__ u32x4 draw(uint32_t index, uint32_t gen, uint32_t tag) const {
    return philox(index, sk, gen, tag, k0, k1);
  }
};

// The Philox stream of state b: shared by every state (the reference re-seeds each state's
// pymoo.minimize with the same seed, moeva2.py:158-165) or, with per-state streams
// (mv_set_state_streams), one stream per global state id key0 + b.
__device__ __forceinline__ uint32_t state_stream(uint32_t sk, int state_keys, uint32_t key0,
                                                 int b) {
  return state_keys ? sk + key0 + (uint32_t)b : sk;
}

// 53-bit uniform in [0,1): MT19937 genrand_res53 form on two Philox words.
__device__ __forceinline__ double u53(uint32_t a, uint32_t b) {
  return ((double)(a >> 5) * 67108864.0 + (double)(b >> 6)) * (1.0 / 9007199254740992.0);
}

}  // namespace mv
