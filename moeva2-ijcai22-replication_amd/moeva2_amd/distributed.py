"""Multi-GPU sharding of an attack over initial states.

Initial states are independent (src/attacks/moeva2/moeva2.py:194-205 runs one pymoo
minimize per state), and every Philox draw is keyed by the row inside its state, so a
state's result does not depend on which GPU runs it.  Rank r of a world of size G takes
the contiguous slice [r*ceil(B/G), (r+1)*ceil(B/G)); no collective runs inside the
generation loop; one all_gather (RCCL over xGMI on MI355X, gloo in the CPU tests) returns
the per-state results to every rank.

Two gathers are offered: ``generate_sharded`` returns the final populations of every state
(genes + F: 271 MB per copy for the 387 botnet states), ``generate_scored_sharded`` scores
each rank's own populations with the ObjectiveCalculator on its GPU first
(``success_flags``) and gathers only what 04_moeva.py:112-131 keeps of them -- the per-state
o1..o7 flags (uint8) and one successful candidate per state (D fp64) -- 2.3 MB for botnet.
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


def success_flags(obj, x_f, thresholds):
    """The ObjectiveCalculator verdict on one rank's final populations, computed where the
    tensors live (the GPU in the product path).

    obj (b, n, 3): per candidate [constraint violation, f1, f2] (objective_calculator.py:44-84);
    x_f (b, n, D): the candidates in ML space.  Returns
      flags (b, 7) uint8: o1..o7 of _objective_respected (:86-101) reached by at least one
        candidate of the state (success_rate_3d's per-state "> 0", :121-128);
      best (b, D) float64: the candidate _get_one_successful(preferred_metrics=
        "misclassification", max_inputs=1) returns (:153-182) -- NaN where the state has no
        o7-successful candidate.  The reference indexes the f1 argsort with the o7 mask in
        ORIGINAL row order (``sorted_index[objective_respected[:, -1]][:1]``), i.e. it keeps
        sorted_index[k0] for the first o7-successful row k0: the candidate with the
        (k0+1)-th smallest f1, which need not be successful itself.  That is reproduced
        here, with a stable f1 sort (numpy's default argsort orders equal f1 in an
        implementation-defined way).
    NaN objectives compare false, as in numpy."""
    import torch

    cv, f1, f2 = obj[..., 0], obj[..., 1], obj[..., 2]
    c = cv <= 0
    m = f1 < float(thresholds["f1"])
    l = f2 <= float(thresholds["f2"])
    resp = torch.stack([c, m, l, c & m, c & l, m & l, c & m & l], dim=-1)
    b, n = obj.shape[0], obj.shape[1]
    flags = resp.any(dim=1).to(torch.uint8) if n else torch.zeros((b, 7), dtype=torch.uint8,
                                                                  device=obj.device)
    D = x_f.shape[-1]
    best = torch.full((b, D), float("nan"), dtype=torch.float64, device=x_f.device)
    if b and n:
        order = torch.sort(f1, dim=1, stable=True).indices  # np.argsort(f1) (NaN last)
        k0 = torch.argmax(resp[..., 6].to(torch.uint8), dim=1)  # first o7-successful row
        idx = order[torch.arange(b, device=obj.device), k0]
        ok = flags[:, 6] != 0
        rows = x_f[torch.arange(b, device=x_f.device), idx]
        best[ok] = rows[ok].to(torch.float64)
    return flags, best


def generate_scored_sharded(attack_scored: Callable, x: np.ndarray, minimize_class, D: int,
                            group=None, device=None):
    """``generate_sharded`` for ``attack_scored(x_shard, mc_shard) -> (flags, best)`` (see
    success_flags): only the per-state flags and successful candidates cross the links.
    Returns (flags (B, 7) uint8, best (B, D) float64) on every rank, in state order."""
    import torch

    def empty():
        return (torch.zeros((0, 7), dtype=torch.uint8, device=device),
                torch.zeros((0, D), dtype=torch.float64, device=device))

    return generate_sharded(attack_scored, x, minimize_class, group, empty=empty)
