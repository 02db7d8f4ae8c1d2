"""The in-tree extension imports on a CPU-only host (hipcc cross-compiled for gfx950): catches
undefined symbols / stale objects before a GPU run does."""
import torch  # noqa: F401  (before the extension: shared HIP runtime)


def test_native_extension_imports_and_targets_gfx950():
    import fraud_detection_amd._fdx_native as m

    assert m.ARCH == "gfx950"
    for name in ("kernelshap", "kernelshap_tree", "auc_radix", "predict_h2h", "predict_shap_sync", "smote_generate", "scaler_stats_cast",
                 "host_device_pointer", "predict_shap", "logreg_pass_fp8"):
        assert hasattr(m, name), name
