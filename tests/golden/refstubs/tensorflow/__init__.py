# Stub: the numpy path never calls TF; the reference only needs these names at import time.
class Tensor:  # used in type annotations (constraints.py:259)
    pass
int64 = "int64"
float32 = "float32"
def convert_to_tensor(x, dtype=None):
    return x
