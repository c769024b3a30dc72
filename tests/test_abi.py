"""CPU checks of the drop-in boundary: libaos_gpu.so loads here (no GPU) and exports every symbol
declared in include/aos_gpu.h; the product library never links the oracle."""
import ctypes
import os
import subprocess

import aos_gpu


def test_library_exports_every_header_symbol():
    if not os.path.exists(aos_gpu.LIB_PATH):
        aos_gpu.build()
    lib = ctypes.CDLL(aos_gpu.LIB_PATH)
    names = aos_gpu.header_functions()
    assert len(names) >= 11
    missing = [n for n in names if not hasattr(lib, n)]
    assert not missing, missing


def test_product_does_not_reference_the_oracle():
    if not os.path.exists(aos_gpu.LIB_PATH):
        aos_gpu.build()
    syms = subprocess.run(["nm", "-D", aos_gpu.LIB_PATH], capture_output=True, text=True).stdout
    assert "orc_" not in syms
    deps = subprocess.run(["ldd", aos_gpu.LIB_PATH], capture_output=True, text=True).stdout
    assert "oracle" not in deps


def test_create_fails_loudly_without_gpu():
    import torch
    if torch.cuda.is_available():
        return
    try:
        aos_gpu.Ctx()
    except RuntimeError as e:
        assert "libaos_gpu error" in str(e)
    else:
        raise AssertionError("aos_create must fail without a gfx950 device (no CPU fallback)")
