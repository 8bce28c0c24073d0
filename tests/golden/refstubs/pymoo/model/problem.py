import numpy as np
class Problem:
    def __init__(self, n_var=-1, n_obj=1, n_constr=0, xl=None, xu=None, **kwargs):
        self.n_var, self.n_obj, self.n_constr = n_var, n_obj, n_constr
        self.xl = None if xl is None else np.asarray(xl, dtype=float)
        self.xu = None if xu is None else np.asarray(xu, dtype=float)
    @staticmethod
    def calc_constraint_violation(G):
        # pymoo 0.4.2.2 Problem.calc_constraint_violation (recalled): sum of positive parts
        if G is None:
            return None
        if G.shape[1] == 0:
            return np.zeros(G.shape[0])[:, None]
        return np.sum(G * (G > 0), axis=1)[:, None]
