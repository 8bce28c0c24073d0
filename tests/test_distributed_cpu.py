"""The N>1 path on CPU: world_size-2 gloo process group, sharding of the initial states and
the final all_gather (moeva2_amd.distributed), against the unsharded computation."""
import os
import socket

import numpy as np
import pytest

torch = pytest.importorskip("torch")

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def fake_attack(x, mc):
    """A deterministic per-state stand-in for Moeva2.generate(return_device=True); like the
    engine (mv_set_states rejects B = 0) it refuses an empty slice."""
    if len(x) == 0:
        raise ValueError("bad mv_set_states arguments")
    xs = torch.as_tensor(np.asarray(x, np.float64))
    genes = xs[:, None, :].repeat(1, 3, 1) * torch.arange(1, 4, dtype=torch.float64)[None, :, None]
    F = torch.stack([xs.sum(1), xs.max(1).values, torch.as_tensor(mc, dtype=torch.float64)], 1)
    return genes, F[:, None, :]


def fake_empty():
    return (torch.empty((0, 3, 5), dtype=torch.float64),
            torch.empty((0, 1, 3), dtype=torch.float64))


def _worker(rank, world, port, B, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch.distributed as dist

    from moeva2_amd.distributed import generate_sharded

    dist.init_process_group("gloo", rank=rank, world_size=world)
    x = np.arange(B * 5, dtype=np.float64).reshape(B, 5)
    genes, F = generate_sharded(fake_attack, x, np.arange(B) % 2, empty=fake_empty)
    q.put((rank, genes.numpy(), F.numpy()))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("B,world", [(7, 2), (8, 2), (1, 2), (5, 4), (2, 3)])
def test_sharded_attack_gathers_every_state(B, world):
    """Every rank ends with every state in state order, including ranks whose slice is
    empty (B < world, or ceil(B/world) leaving the last ranks nothing)."""
    import torch.multiprocessing as mp

    from moeva2_amd.distributed import shard_bounds

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, B, q)) for r in range(world)]
    for pr in procs:
        pr.start()
    res = [q.get(timeout=120) for _ in procs]
    for pr in procs:
        pr.join(timeout=120)
        assert pr.exitcode == 0
    x = np.arange(B * 5, dtype=np.float64).reshape(B, 5)
    ref_g, ref_F = fake_attack(x, np.arange(B) % 2)
    for _, genes, F in res:  # every rank holds every state, in state order
        np.testing.assert_array_equal(genes, ref_g.numpy())
        np.testing.assert_array_equal(F, ref_F.numpy())
    per = -(-B // world)
    assert [shard_bounds(B, world, r) for r in range(world)] == \
        [(min(r * per, B), min(r * per + per, B)) for r in range(world)]


def _bench_worker(rank, world, port, B_all, shard, q):
    """bench.py's step on a gloo group: the rank's shard of global_states is bound once
    (the engine rejects B = 0: mv_set_states), the attack must be called with exactly that
    shard, and generate_sharded gathers every state's result on every rank."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import sys

    import torch.distributed as dist

    sys.path.insert(0, ROOT)
    from bench import global_states
    from moeva2_amd.distributed import generate_sharded, shard_bounds

    dist.init_process_group("gloo", rank=rank, world_size=world)
    X_all = np.arange(B_all * 5, dtype=np.float64).reshape(B_all, 5)
    X_glob = global_states(X_all, world, shard)
    lo, hi = shard_bounds(X_glob.shape[0], world, rank)
    bound = X_glob[lo:hi]
    calls = []

    def attack(xs, mc):
        assert len(bound) > 0 and np.array_equal(xs, bound)  # the engine's input contract
        calls.append(len(xs))
        return fake_attack(xs, mc)

    outs = [generate_sharded(attack, X_glob, 1, empty=fake_empty) for _ in range(2)]
    q.put((rank, calls, [o[0].numpy() for o in outs], X_glob))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("B_all,world,shard", [(5, 2, False), (5, 2, True), (1, 2, True),
                                               (3, 3, False)])
def test_bench_step_is_generate_sharded(B_all, world, shard):
    """bench.py --gpus N times generate_sharded: weak scaling tiles the states x N (one copy
    per rank), strong scaling (--shard) splits them, an empty rank joins the all_gather."""
    import torch.multiprocessing as mp

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_bench_worker, args=(r, world, port, B_all, shard, q))
             for r in range(world)]
    for pr in procs:
        pr.start()
    res = [q.get(timeout=120) for _ in procs]
    for pr in procs:
        pr.join(timeout=120)
        assert pr.exitcode == 0
    n_glob = B_all if shard else B_all * world
    for rank, calls, outs, X_glob in res:
        assert X_glob.shape[0] == n_glob
        ref_g, _ = fake_attack(X_glob, np.ones(n_glob))
        for g in outs:
            np.testing.assert_array_equal(g, ref_g.numpy())
        per = -(-n_glob // world)
        mine = max(0, min(n_glob, (rank + 1) * per) - rank * per)
        assert calls == ([mine] * 2 if mine else [])


THR = {"f1": 0.5, "f2": 0.3}


def fake_scored_objectives(x):
    """Deterministic per-state final-population objectives (b, n=6, 3) and ML candidates
    (b, 6, 5) with ties in f1, NaNs and states without an o7 success."""
    xs = torch.as_tensor(np.asarray(x, np.float64))
    b = xs.shape[0]
    k = torch.arange(6, dtype=torch.float64)
    s = xs.sum(1)[:, None]
    cv = torch.remainder(s + k, 3.0) - 1.0          # <= 0 for two of three candidates
    f1 = torch.remainder(0.37 * s + 0.11 * k, 1.0)
    f1[:, 4] = f1[:, 1]                              # an f1 tie
    f2 = torch.remainder(0.23 * s + 0.07 * k, 0.6)
    f2[torch.arange(b) % 3 == 2, 5] = float("nan")   # NaN compares false
    obj = torch.stack([cv, f1, f2], dim=-1)
    xf = xs[:, None, :] + k[None, :, None]
    return obj, xf


def ref_success(obj, xf):
    """numpy restatement of objective_calculator.py:86-101 (_objective_respected), :121-128
    (any over the population) and :153-182 (_get_one_successful, misclassification asc,
    max_inputs=1), literally: the f1 argsort indexed by the o7 mask in original row order
    (stable order among equal f1).  Also returns how many states the plain "o7-successful
    row of smallest f1" rule would answer differently."""
    flags, best, differs = [], [], 0
    for o, x in zip(obj, xf):
        c, m, l = o[:, 0] <= 0, o[:, 1] < THR["f1"], o[:, 2] <= THR["f2"]
        r = np.column_stack([c, m, l, c * m, c * l, m * l, c * m * l])
        flags.append(r.any(axis=0))
        sorted_index = np.argsort(o[:, 1], kind="stable")
        sel = sorted_index[r[:, -1]][:1]
        best.append(x[sel[0]] if sel.size else np.full(x.shape[1], np.nan))
        if sel.size:
            naive = int(np.argmin(np.where(r[:, -1], o[:, 1], np.inf)))
            differs += int(not np.array_equal(x[naive], x[sel[0]]))
    return np.array(flags), np.array(best), differs


def _scored_worker(rank, world, port, B, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch.distributed as dist

    from moeva2_amd.distributed import generate_scored_sharded, success_flags

    dist.init_process_group("gloo", rank=rank, world_size=world)
    x = np.arange(B * 5, dtype=np.float64).reshape(B, 5)
    calls = []

    def attack(xs, mc):
        if len(xs) == 0:
            raise ValueError("bad mv_set_states arguments")
        calls.append(len(xs))
        obj, xf = fake_scored_objectives(xs)
        return success_flags(obj, xf, THR)

    flags, best = generate_scored_sharded(attack, x, 1, 5)
    q.put((rank, calls, flags.numpy(), best.numpy()))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("B,world", [(7, 2), (1, 2), (5, 4), (2, 3), (9, 3)])
def test_scored_sharded_gathers_flags(B, world):
    """generate_scored_sharded: every rank scores its own slice and only per-state o1..o7
    flags (uint8) and one successful candidate per state are gathered; every rank ends with
    the unsharded verdict in state order, empty ranks included."""
    import torch.multiprocessing as mp

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_scored_worker, args=(r, world, port, B, q))
             for r in range(world)]
    for pr in procs:
        pr.start()
    res = [q.get(timeout=120) for _ in procs]
    for pr in procs:
        pr.join(timeout=120)
        assert pr.exitcode == 0
    x = np.arange(B * 5, dtype=np.float64).reshape(B, 5)
    obj, xf = fake_scored_objectives(x)
    ref_f, ref_b, differs = ref_success(obj.numpy(), xf.numpy())
    assert ref_f[:, 6].any() and not ref_f[:, 6].all() or B < 3
    assert differs > 0 or B < 5  # the reference's indexing is what is checked
    per = -(-B // world)
    for rank, calls, flags, best in res:
        assert flags.dtype == np.uint8 and flags.shape == (B, 7)
        np.testing.assert_array_equal(flags.astype(bool), ref_f)
        np.testing.assert_array_equal(best, ref_b)
        mine = max(0, min(B, (rank + 1) * per) - rank * per)
        assert calls == ([mine] if mine else [])
