"""The in-tree extension imports on a CPU-only host (hipcc cross-compiled for gfx950): catches
undefined symbols / stale objects before a GPU run does."""
import torch  # noqa: F401  (before the extension: shared HIP runtime)


def test_native_extension_imports_and_targets_gfx950():
    import fraud_detection_amd._fdx_native as m

    assert m.ARCH == "gfx950"
    for name in ("kernelshap", "kernelshap_tree", "auc_radix", "predict_h2h", "predict_shap_sync", "smote_generate", "scaler_stats_cast",
                 "host_device_pointer", "predict_shap", "logreg_pass_fp8"):
        assert hasattr(m, name), name


def test_auc_radix_workspace_layout_is_aligned():
    """Host-side check of the radix AUC workspace (csrc/kernels/auc.hip auc_radix_layout): every
    region 256-byte aligned and disjoint for odd and even n -- an odd n once shifted the u64
    counters off alignment (GPU fault, round 3)."""
    import fraud_detection_amd._fdx_native as m

    for n in (0, 1, 3, 255, 256, 257, 3_000_001, 20_000_000, (1 << 31) + 7):
        off = m.auc_radix_layout(n)
        sizes = [4 * n, 4 * n, n, n, 256 * 1024 * 4, 24, 256 * 4]
        assert all(o % 256 == 0 for o in off), (n, off)
        for i in range(7):
            assert off[i] + sizes[i] <= off[i + 1], (n, i, off)
        assert m.auc_radix_workspace_bytes(n) == off[7]
