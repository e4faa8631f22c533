"""CPU: the C-ABI library loads, exports every symbol include/shadow_routing.h declares, and
refuses to run without a GPU (no CPU fallback)."""
import ctypes
import os
import re

import pytest

from shadow_amd import _native as N

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def header_functions():
    txt = open(os.path.join(ROOT, "include", "shadow_routing.h")).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b(srg_[a-z_0-9]+)\s*\(", txt)))


def test_header_matches_binding_list():
    assert header_functions() == sorted(N.EXPORTS)


def test_library_exports_all_symbols():
    L = N.lib()
    for name in header_functions():
        assert hasattr(L, name), name
    assert b"gfx950" in L.srg_version()


def test_library_is_gfx950_code_object():
    data = open(N.LIB_PATH, "rb").read()
    assert b"gfx950" in data


def test_no_cpu_fallback_without_gpu():
    import torch
    if torch.cuda.is_available():
        pytest.skip("a GPU is present")
    h = ctypes.c_void_p()
    err = ctypes.create_string_buffer(512)
    rc = N.lib().srg_create(ctypes.byref(h), 0, err, len(err))
    assert rc == N.SRG_ERR_HIP
    assert b"no CPU fallback" in err.value
    from shadow_amd import HipError, NetworkGraph
    from helpers import kat_gml
    g = NetworkGraph.parse(kat_gml(True))
    with pytest.raises(HipError):
        g.compute_shortest_paths([0, 1, 2])


def test_struct_layouts():
    assert ctypes.sizeof(N.EdgeList) == 4 + 4 + 8 + 5 * 8
    assert ctypes.sizeof(N.Stats) == 8 * 8 + 4 + 4 + 8 + 8 + 8 + 4 + 4 + 8 + 8 + 8 + 8 + 4 + 4 + 8 + 8 + 8 + 8 + 8 + 4 + 4 + 4 + 4 + 8
