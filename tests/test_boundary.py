"""The drop-in boundary without a GPU: the C-ABI library loads and exports every
entry point include/artsbir.h declares, rejects bad shapes with a status and a
message, and the Python mirror of models.py has the reference's constructor
signatures, parameter names and counts (models.py:191-379 of the reference)."""
import ctypes
import os
import re

import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "artsbir.h")


def _declared():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    src = re.sub(r"//[^\n]*", "", src)
    return sorted(set(re.findall(r"\b(artsbir_[a-z0-9_]+)\s*\(", src)))


def test_library_exports_every_declared_symbol():
    import _hip
    lib = _hip.lib()
    names = _declared()
    assert len(names) >= 40
    missing = [n for n in names if not hasattr(lib, n)]
    assert not missing, missing
    # and the ctypes signature table covers exactly the header
    assert sorted(_hip.SIGNATURES) == names
    assert lib.artsbir_version() >= 1


def test_no_cpu_fallback_when_library_missing(monkeypatch):
    import _hip
    monkeypatch.setattr(_hip, "_lib", None)
    monkeypatch.setattr(_hip, "LIB_PATH", os.path.join(ROOT, "does-not-exist.so"))
    with pytest.raises(RuntimeError, match="no fallback"):
        _hip.lib()


def test_capi_rejects_bad_shapes_without_touching_the_gpu():
    import _hip
    lib = _hip.lib()
    d = _hip.ConvDesc(_hip.DT_BF16, 2, 8, 8, 3, 64, 3, 3, 1, 1)
    rc = lib.artsbir_conv2d_fwd(ctypes.byref(d), None, None, None, 0, 0, 0, None, None, None, 0, None, None)
    assert rc != 0 and b"multiple of 8" in lib.artsbir_last_error()
    rc = lib.artsbir_gemm_nt(_hip.DT_BF16, 16, 16, 12, None, 12, None, None, 16, 0, 0, None, None, None)
    assert rc != 0 and b"K=12" in lib.artsbir_last_error()
    with pytest.raises(_hip.HipError, match="gemm_nt"):
        _hip.call("artsbir_gemm_nt", _hip.DT_BF16, 16, 16, 12, None, 12, None, None, 16, 0, 0, None, None, None)


@pytest.mark.parametrize("output_dim,count", [(1024, 38_316_896), (512, 37_267_808)])
def test_modified_resnet_signature_keys_and_counts(output_dim, count):
    import models
    from oracle import encoder as oenc
    m = models.ModifiedResNet((3, 4, 6, 3), output_dim, heads=32, input_resolution=224, width=64)
    ref = oenc.ModifiedResNet((3, 4, 6, 3), output_dim, heads=32, input_resolution=224, width=64)
    assert sum(p.numel() for p in m.parameters()) == count
    sd, rsd = m.state_dict(), ref.state_dict()
    assert list(sd) == list(rsd)
    for k in sd:
        assert sd[k].shape == rsd[k].shape, k
    # a checkpoint written from the reference layout loads strictly
    m.load_state_dict(rsd, strict=True)


def test_classification_head_keys():
    import models
    m = models.ModifiedResNet_with_classification((3, 4, 6, 3), 1024, heads=32, input_resolution=224, width=64,
                                                  num_classes=125)
    keys = list(m.state_dict())
    assert "classifier.weight" in keys and "classifier.bias" in keys  # models.py:370
    assert m.state_dict()["classifier.weight"].shape == (125, 1024)
    assert "classifier2.weight" not in keys


def test_encoder_refuses_cpu_input():
    import models
    m = models.ModifiedResNet((1, 1, 1, 1), 32, heads=8, input_resolution=64, width=16)
    with pytest.raises(RuntimeError, match="GPU"):
        with torch.no_grad():
            m(torch.zeros(1, 3, 64, 64))


def test_grad_order_covers_every_parameter_once():
    import models
    m = models.ModifiedResNet((2, 1, 1, 1), 64, heads=8, input_resolution=64, width=16)
    order = [id(p) for p in m.grad_order()]
    assert len(order) == len(set(order))
    assert sorted(order) == sorted(id(p) for p in m.parameters())
