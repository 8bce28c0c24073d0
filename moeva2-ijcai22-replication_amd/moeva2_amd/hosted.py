"""Host fallback for plugins the engine cannot compile.

The reference accepts any ``Constraints`` subclass (src/attacks/moeva2/constraints.py:8-77)
and any classifier with ``predict_proba`` (classifier.py:11-29).  The engine runs the shipped
LCLD / botnet constraint classes as device programs and Dense-MLP classifiers on MFMA; for
anything else the plugin's own method is called on the host, once per generation for all
states at once:

* device: variation, tournament, survival, the encoder and f2 (and whichever of f1 / f3 the
  engine can compute), and the genetic -> ML decode (``mv_decode``);
* host: ``constraints.evaluate(x_f)`` -> f3 = sum(G * (G > 0)) (default_problem.py:93-97,
  128-129) and/or ``classifier.predict_proba(ml_scaler.transform(x_f))[:, c]`` -> f1
  (default_problem.py:119-124).

Cost: one device -> host copy of the decoded ML rows (B x n x D fp64) and one host -> device
copy of the f1 / f3 columns per generation, plus the plugin's own host time; a generation
is then host-bound.  The generation loop issues the same device calls, with
the same Philox draws, as mv_attack_run, so with equal F columns both loops give the same
populations (tests/test_gpu_parity.py::test_hosted_plugins_*).
"""
from __future__ import annotations

from typing import Optional

import numpy as np

from . import _native
from .problem import has_device_classifier, has_device_program, ml_transform


class HostPlugins:
    """Which objective columns come from host plugins, and how to fill them."""

    def __init__(self, constraints, classifier, ml_scaler):
        self.constraints = constraints
        self.classifier = classifier
        self.ml_scaler = ml_scaler
        self.host_constraints = not has_device_program(constraints)
        self.host_classifier = not has_device_classifier(classifier)

    @property
    def any(self) -> bool:
        return self.host_constraints or self.host_classifier

    def fill(self, eng, genes, F, minimize_class, G_out: Optional[list] = None):
        """genes (B, n, V) device -> writes the host columns of F (B, n, 3) in place.
        G_out: if a list, the host constraint matrix (B, n, C) is appended (full history)."""
        import torch

        if not self.any:
            return
        B, n, V = genes.shape
        D = eng.prog.D
        xd = torch.empty((B, n, D), dtype=torch.float64, device=genes.device)
        eng.decode(genes, xd)
        x_f = xd.cpu().numpy().reshape(B * n, D)
        if self.host_constraints:
            g = np.asarray(self.constraints.evaluate(x_f), dtype=np.float64)
            g = g * (g > 0)
            F[:, :, 2] = torch.as_tensor(g.sum(axis=1).reshape(B, n), device=F.device)
            if G_out is not None:
                G_out.append(g.reshape(B, n, -1))
        if self.host_classifier:
            proba = np.asarray(self.classifier.predict_proba(ml_transform(self.ml_scaler, x_f)))
            mc = np.repeat(np.broadcast_to(np.asarray(minimize_class), (B,)), n)
            f1 = proba[np.arange(B * n), mc].astype(np.float64)
            F[:, :, 0] = torch.as_tensor(f1.reshape(B, n), device=F.device)


def hosted_attack(eng, plugins: HostPlugins, genes0, minimize_class, n_gen, P, O, seed, ref,
                  mu, history_mode):
    """The MoEvA2 generation loop driven from the host around device calls (the path of a
    host plugin).  genes0: (B, V) initial genetic vectors (sampling.py:64-78).  Returns
    genes (B, P, V), F (B, P, 3) and the history (B, P + (n_gen-1) O, 3 | 3 + C) or None."""
    import torch

    if getattr(eng, "state_streams", (False, 0))[0]:
        raise ValueError("per-state random streams are a device-loop option (mv_attack_run); "
                         "the host-plugin loop draws every state from the shared stream")
    dev = torch.device("cuda", eng.device)
    B, V = genes0.shape
    g0 = torch.as_tensor(np.ascontiguousarray(genes0, np.float64), device=dev)
    pop = g0[:, None, :].repeat(1, P, 1).contiguous()
    hist, Gh = [], [] if history_mode == 2 else None

    def evaluate(genes):
        n = genes.shape[1]
        F = torch.empty((B, n, 3), dtype=torch.float64, device=dev)
        Gd = None
        if history_mode == 2 and not plugins.host_constraints:
            Gd = torch.empty((B, n, eng.prog.C), dtype=torch.float64, device=dev)
        eng.evaluate(genes, F, Gd)
        plugins.fill(eng, genes, F, minimize_class, Gh)
        if history_mode == 1:
            hist.append(F.clone())
        elif history_mode == 2:
            G = Gd if Gd is not None else torch.as_tensor(Gh.pop(), device=dev)
            hist.append(torch.cat([F, G], dim=2))
        return F

    ideal = torch.full((B, 3), np.inf, dtype=torch.float64, device=dev)
    worst = torch.full((B, 3), -np.inf, dtype=torch.float64, device=dev)
    extreme = torch.zeros((B, 9), dtype=torch.float64, device=dev)
    has = torch.zeros((B,), dtype=torch.int32, device=dev)
    refd = torch.as_tensor(np.ascontiguousarray(ref, np.float64), device=dev)

    def survive(F, gen):
        surv = torch.empty((B, P), dtype=torch.int32, device=dev)
        _native.survive(F.contiguous(), refd, P, mu, seed, gen, ideal, worst, extreme, has, surv)
        return surv.long()

    def take(t, idx):
        return torch.gather(t, 1, idx[:, :, None].expand(-1, -1, t.shape[2])).contiguous()

    F = evaluate(pop)
    s = survive(F, 0)
    pop, F = take(pop, s), take(F, s)
    n_m = (O + 1) // 2
    for g in range(1, n_gen):
        parents = torch.empty((B, n_m, 2), dtype=torch.int32, device=dev)
        _native.select_parents(B, P, O, seed, g, parents)
        off = torch.empty((B, O, V), dtype=torch.float64, device=dev)
        eng.variation(P, O, seed, g, pop, parents, off)
        Fo = evaluate(off)
        mp, mF = torch.cat([pop, off], dim=1), torch.cat([F, Fo], dim=1)
        s = survive(mF, g)
        pop, F = take(mp, s), take(mF, s)
    h = torch.cat(hist, dim=1) if hist else None
    return pop, F, h
