"""Device operators.  Every op takes torch tensors; ROCm tensors run the hand-written gfx950 HIP
kernels in ``csrc/kernels`` (no eager fallback), CPU tensors run the fp64/fp32 oracles in
``ops/reference.py`` that the GPU tests compare against."""
from .native import NativeUnavailableError, available  # noqa: F401
from .layout import BIAS_COL, LABEL_COL, NCOLS, NFEAT_MAX  # noqa: F401
