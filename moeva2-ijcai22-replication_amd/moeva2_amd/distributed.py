"""Multi-GPU sharding of an attack over initial states.

Initial states are independent (src/attacks/moeva2/moeva2.py:194-205 runs one pymoo
minimize per state), and every Philox draw is keyed by the row inside its state, so a
state's result does not depend on which GPU runs it.  Rank r of a world of size G takes
the contiguous slice [r*ceil(B/G), (r+1)*ceil(B/G)); no collective runs inside the
generation loop; one all_gather (RCCL over xGMI on MI355X, gloo in the CPU tests) returns
the per-state results to every rank.
"""
from __future__ import annotations

import math
from typing import Callable, Optional, Sequence, Tuple

import numpy as np


def shard_bounds(n_states: int, world: int, rank: int) -> Tuple[int, int]:
    """[lo, hi) of the states rank `rank` owns."""
    if world < 1 or not 0 <= rank < world:
        raise ValueError(f"bad rank {rank} of world {world}")
    per = math.ceil(n_states / world) if n_states else 0
    lo = min(rank * per, n_states)
    return lo, min(lo + per, n_states)


def all_gather_states(local, n_states: int, group=None):
    """Concatenate every rank's per-state tensor (leading dim = its shard) in rank order.

    Shards are padded to ceil(B/G) rows so one fixed-size all_gather suffices."""
    import torch
    import torch.distributed as dist

    world = dist.get_world_size(group)
    per = math.ceil(n_states / world) if n_states else 0
    pad = torch.zeros((per,) + tuple(local.shape[1:]), dtype=local.dtype, device=local.device)
    pad[: local.shape[0]] = local
    out = [torch.empty_like(pad) for _ in range(world)]
    dist.all_gather(out, pad, group=group)
    parts = []
    for r in range(world):
        lo, hi = shard_bounds(n_states, world, r)
        parts.append(out[r][: hi - lo])
    return torch.cat(parts, dim=0)


def generate_sharded(attack: Callable, x: np.ndarray, minimize_class, group=None,
                     empty: Optional[Callable] = None) -> Sequence:
    """Run `attack(x_shard, minimize_class_shard) -> tuple of per-state tensors` on this
    rank's slice of the initial states and all-gather every returned tensor.

    A rank whose slice is empty (B < world, or the last ranks when ceil(B/world) leaves a
    remainder) does not call `attack`: it contributes `empty()` -- zero-row tensors of the
    shapes `attack` returns -- so every rank still enters the same all_gather."""
    import torch.distributed as dist

    B = x.shape[0]
    mc = np.broadcast_to(np.asarray(minimize_class), (B,))
    if not (dist.is_available() and dist.is_initialized()):  # one process: no collective
        return tuple(attack(x, mc))
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    lo, hi = shard_bounds(B, world, rank)
    if hi > lo or empty is None:
        outs = attack(x[lo:hi], mc[lo:hi])
    else:
        outs = empty()
    return tuple(all_gather_states(t, B, group) for t in outs)
