"""The C-ABI library: loads without a GPU, exports every symbol include/flipwalk.h
declares, validates inputs before touching the device, and the product path refuses to
run without a GPU (no CPU fallback)."""
import ctypes
import os
import re

import numpy as np
import pytest

from flipcomplexityempirical_amd import _lib

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def header_functions():
    src = open(os.path.join(ROOT, "include", "flipwalk.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(fw_[a-z_]+)\s*\(", src)))


def test_every_declared_symbol_is_exported_and_bound():
    L = _lib.load()
    declared = header_functions()
    assert len(declared) >= 16
    bound = {name for name, _, _ in _lib.SIGNATURES}
    assert set(declared) == bound
    for name in declared:
        assert hasattr(L, name), name


def test_version_and_device_count_without_gpu():
    L = _lib.load()
    assert L.fw_version() == 0x000700
    assert L.fw_device_count() >= 0


def test_build_info_names_sources_and_flags():
    """fw_build_info: a hash over the kernel / header / ABI sources and the compile flags
    (bench lines and PMC profiles carry it); a rebuilt in-tree library hashes the
    sources as they are now."""
    import hashlib
    info = _lib.build_info()
    m = re.match(r"src=([0-9a-f]{16}) flags=(.*)$", info)
    assert m, info
    assert "--offload-arch=gfx950" in m.group(2)
    csrc = os.path.join(ROOT, "flipcomplexityempirical_amd", "csrc")
    blob = b"".join(open(os.path.join(csrc, f), "rb").read() for f in
                    ("fw_api.hip", "fw_kernels.hip", "fw_grid16.hip", "fw_grid16_lean.hip",
                     "fw_grid16_w2.hip",
                     "fw_internal.h", "fw_device.h", "fw_math.h"))
    blob += open(os.path.join(ROOT, "include", "flipwalk.h"), "rb").read()
    assert m.group(1) == hashlib.sha256(blob).hexdigest()[:16], "library older than its sources"


def _csr(adj):
    rowptr = np.zeros(len(adj) + 1, np.int32)
    rowptr[1:] = np.cumsum([len(a) for a in adj])
    col = np.array([u for a in adj for u in a], np.int32)
    return rowptr, col


@pytest.mark.parametrize("adj,why", [
    ([[1], [0, 2], [0]], "not symmetric"),  # 2 lists 0 but 0 does not list 2
    ([[2, 1], [0], [0]], "ascending"),
    ([[0, 1], [0], []], "self loop"),
])
def test_graph_validation_before_device(adj, why):
    L = _lib.load()
    rowptr, col = _csr(adj)
    h = ctypes.c_void_p()
    rc = L.fw_graph_create(_lib.ptr(rowptr), _lib.ptr(col), None, len(adj), len(col), 0,
                           ctypes.byref(h))
    assert rc == _lib.FW_EINVAL
    assert L.fw_last_error().decode()


def test_null_arguments_rejected():
    L = _lib.load()
    assert L.fw_graph_create(None, None, None, 0, 0, 0, None) == _lib.FW_EINVAL
    assert L.fw_chains_run(None, 10, 10) == _lib.FW_EINVAL
    assert L.fw_chains_read(None, 0, None, 0) == _lib.FW_EINVAL
    assert L.fw_eval_flips(None, None, 2, None, None, 0, 0, 0, None, None, None, None) == \
        _lib.FW_EINVAL


def test_product_path_fails_loudly_without_gpu():
    if _lib.load().fw_device_count() > 0:
        pytest.skip("a GPU is visible")
    from flipcomplexityempirical_amd.chain import DeviceGraph
    from flipcomplexityempirical_amd.graph import grid_graph
    with pytest.raises(_lib.FlipwalkUnavailable):
        DeviceGraph(grid_graph(4, 4))
