"""Philox4x32-10 counter-based RNG (numpy) -- TEST INFRASTRUCTURE ONLY.

This is the CPU statement of the draw layout that the HIP kernels in
``moeva2-ijcai22-replication_amd/csrc/philox.h`` use.  Only ``tests/``,
``__graft_entry__.smoke()`` and ``bench.py``'s cpu_baseline leg may import it.

The reference draws from numpy's global MT19937 (``np.random.*`` inside pymoo,
re-seeded with the same seed for every initial state by ``pymoo.optimize.minimize``
called at ``src/attacks/moeva2/moeva2.py:158-165``).  ``north_star`` replaces
that stream with Philox so that GPU draws are reproducible; it does not
reproduce the MT sequence.

Counter layout (shared with the kernels):
    key     = (seed & 0xffffffff, seed >> 32)
    counter = (index, stream_key, generation, tag)
``stream_key`` is 0 for every state by default, mirroring the reference's
"same seed for every initial state" behaviour (moeva2.py:163).
"""
import numpy as np

M0 = np.uint64(0xD2511F53)
M1 = np.uint64(0xCD9E8D57)
W0 = 0x9E3779B9
W1 = 0xBB67AE85
MASK32 = np.uint64(0xFFFFFFFF)

# stream tags (must match csrc/philox.h)
TAG_SEL_PERM = 1
TAG_SEL_CHOICE = 2
TAG_CX = 3
TAG_MUT_MASK = 4
TAG_MUT_U = 5
TAG_NICHE_PERM = 6
TAG_NICHE_MEMBER = 7
TAG_SBX = 8


def philox4x32_10(c0, c1, c2, c3, k0, k1):
    """Vectorised Philox4x32-10. Counters are broadcastable uint32-valued arrays."""
    c0 = np.asarray(c0, dtype=np.uint64) & MASK32
    c1 = np.asarray(c1, dtype=np.uint64) & MASK32
    c2 = np.asarray(c2, dtype=np.uint64) & MASK32
    c3 = np.asarray(c3, dtype=np.uint64) & MASK32
    c0, c1, c2, c3 = np.broadcast_arrays(c0, c1, c2, c3)
    c0, c1, c2, c3 = c0.copy(), c1.copy(), c2.copy(), c3.copy()
    k0 = int(k0) & 0xFFFFFFFF
    k1 = int(k1) & 0xFFFFFFFF
    for r in range(10):
        if r:
            k0 = (k0 + W0) & 0xFFFFFFFF
            k1 = (k1 + W1) & 0xFFFFFFFF
        p0 = M0 * c0
        p1 = M1 * c2
        hi0, lo0 = p0 >> np.uint64(32), p0 & MASK32
        hi1, lo1 = p1 >> np.uint64(32), p1 & MASK32
        c0, c1, c2, c3 = (hi1 ^ c1 ^ np.uint64(k0)), lo1, (hi0 ^ c3 ^ np.uint64(k1)), lo0
    return (c0.astype(np.uint32), c1.astype(np.uint32), c2.astype(np.uint32),
            c3.astype(np.uint32))


def u53(a, b):
    """53-bit uniform double in [0, 1) from two uint32 words (MT19937 genrand_res53 form)."""
    a = np.asarray(a, dtype=np.uint64) >> np.uint64(5)
    b = np.asarray(b, dtype=np.uint64) >> np.uint64(6)
    return (a.astype(np.float64) * 67108864.0 + b.astype(np.float64)) / 9007199254740992.0


class Stream:
    """Draws for one (seed, stream_key, generation, tag)."""

    def __init__(self, seed, generation, tag, stream_key=0):
        self.k0 = seed & 0xFFFFFFFF
        self.k1 = (seed >> 32) & 0xFFFFFFFF
        self.g = generation
        self.tag = tag
        self.sk = stream_key

    def words(self, index):
        return philox4x32_10(index, self.sk, self.g, self.tag, self.k0, self.k1)
