from numpy import *  # noqa: F401,F403  (autograd.numpy.column_stack == numpy.column_stack)
