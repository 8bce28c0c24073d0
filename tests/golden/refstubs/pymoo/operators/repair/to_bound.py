import numpy as np
def set_to_bounds_if_outside_by_problem(problem, X):
    # pymoo 0.4.2.2 (recalled, unpinned): clip to problem bounds
    X = np.array(X, dtype=float, copy=True)
    xl = np.repeat(problem.xl[None, :], X.shape[0], axis=0)
    xu = np.repeat(problem.xu[None, :], X.shape[0], axis=0)
    X[X < xl] = xl[X < xl]
    X[X > xu] = xu[X > xu]
    return X
