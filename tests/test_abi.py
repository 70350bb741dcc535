"""The C-ABI library loads on a CPU host and exports exactly what include/fmdiff.h declares.

No compute call is made (there is no GPU here); the GPU tests call through these entry points."""
import ctypes
import os
import re

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(REPO, "include", "fmdiff.h")


def _declared():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    src = re.sub(r"//[^\n]*", "", src)
    return sorted(set(re.findall(r"\b(fmd_[a-z0-9_]+)\s*\(", src)))


def test_header_declares_entry_points():
    names = _declared()
    assert len(names) >= 25
    for must in ("fmd_conv", "fmd_wgrad", "fmd_gn_prep", "fmd_attn_mfma_fwd", "fmd_flow_euler", "fmd_adamw_sched"):
        assert must in names


def test_library_exports_every_declared_symbol():
    from fmdiff import _lib
    if not os.path.exists(_lib.LIB_PATH):
        pytest.skip("libfmdiff_hip.so not built (run __graft_entry__.build())")
    try:
        L = ctypes.CDLL(_lib.LIB_PATH)
    except OSError as e:  # HIP runtime absent on this host
        pytest.skip(f"HIP runtime not loadable here: {e}")
    missing = [n for n in _declared() if not hasattr(L, n)]
    assert not missing, missing
    # the ctypes table covers every declared function with a signature
    assert sorted(_lib.SIGNATURES) == _declared()
    lib = _lib.lib()
    for n in _declared():
        assert getattr(lib, n).argtypes is not None


def test_struct_mirrors_match_header_field_order():
    from fmdiff import _lib
    src = open(HEADER).read()
    for cname, py in (("fmd_conv_desc", _lib.ConvDesc), ("fmd_wgrad_desc", _lib.WgradDesc),
                      ("fmd_gn_apply_desc", _lib.GnApplyDesc), ("fmd_gb_job", _lib.GbJob),
                      ("fmd_conv_small_desc", _lib.ConvSmallDesc),
                      ("fmd_lincomb_desc", _lib.LincombDesc)):
        m = re.search(r"typedef\s+struct\s*(?:\w+\s*)?\{([^{}]*)\}\s*" + cname + r"\s*;", src, flags=re.S)
        assert m, cname
        body = re.sub(r"/\*.*?\*/", "", m.group(1), flags=re.S)
        body = re.sub(r"//[^\n]*", "", body)
        fields = []
        for decl in body.split(";"):
            parts = [p for p in decl.strip().split(",") if p.strip()]
            fields += [re.findall(r"[A-Za-z_]\w*", re.sub(r"\[[^\]]*\]", "", p))[-1] for p in parts]
        assert fields == [f.rstrip("_") for f, _ in py._fields_], cname


def test_product_path_has_no_cpu_fallback():
    import torch
    from fmdiff.runtime import ops
    x = torch.zeros(1, 8, 8, 16, dtype=torch.bfloat16)
    with pytest.raises(RuntimeError):
        ops.conv(x, 16, torch.zeros(16, 9, 16, dtype=torch.bfloat16))


def test_every_host_module_imports():
    """Import every host-side module of the package (no GPU needed): catches syntax/import errors in
    code paths only the GPU tests exercise."""
    import importlib
    import pkgutil

    import fmdiff
    names = [m.name for m in pkgutil.walk_packages(fmdiff.__path__, "fmdiff.")]
    assert "fmdiff.runtime.engine" in names
    for n in names:
        importlib.import_module(n)
