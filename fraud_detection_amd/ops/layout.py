"""Padded row layout shared by every kernel (csrc/kernels/common.h).

A device row is 32 columns: ``[0, d)`` standardized features (d <= 30), ``30`` = 1.0 (intercept
column; logistic weight ``w[30]`` is the intercept), ``31`` = label (training buffers) or 0.
bf16 rows are 64 B, fp8 (OCP e4m3fn) rows are 32 B.
"""
import torch

NCOLS = 32
BIAS_COL = 30
LABEL_COL = 31
NFEAT_MAX = 30

DTYPE_KIND = {"bf16": 0, "f32": 1, "fp8": 2}
TORCH_STORAGE = {"bf16": torch.bfloat16, "f32": torch.float32, "fp8": torch.uint8}
DEFAULT_FP8_SCALE = 4.0  # features * 4 keeps |x| <= 112 standard deviations inside e4m3 (max 448)


def storage_kind(t: torch.Tensor) -> str:
    if t.dtype == torch.bfloat16:
        return "bf16"
    if t.dtype == torch.float32:
        return "f32"
    if t.dtype == torch.uint8:
        return "fp8"
    raise ValueError(f"unsupported row storage dtype {t.dtype}")


def check_rows(t: torch.Tensor, name: str = "rows") -> None:
    if t.dim() != 2 or t.shape[1] != NCOLS:
        raise ValueError(f"{name}: expected [n, {NCOLS}] padded rows, got {tuple(t.shape)}")
    if not t.is_contiguous():
        raise ValueError(f"{name}: must be contiguous")
    if t.is_cuda and t.data_ptr() % 16 != 0:
        raise ValueError(f"{name}: device rows must be 16-byte aligned")
