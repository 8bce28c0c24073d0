import numpy as np
def crossover_mask(X, M):
    # pymoo 0.4.2.2 crossover_mask (recalled, unpinned): swap masked genes between parents
    _X = np.copy(X)
    _X[0][M] = X[1][M]
    _X[1][M] = X[0][M]
    return _X
