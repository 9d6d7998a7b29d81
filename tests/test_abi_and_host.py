"""CPU tests: the C ABI library loads and exports every symbol include/pfsgnn.h
declares (no compute calls -- there is no GPU here), the host-side layout /
batching / parameter logic, and the fail-loudly behaviour without a GPU."""
import os
import re
import subprocess

import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "pfs-neural-net_amd")


def header_functions():
    txt = open(os.path.join(ROOT, "include", "pfsgnn.h")).read()
    return sorted(set(re.findall(r"\b(pfsgnn_\w+)\s*\(", txt)))


@pytest.fixture(scope="module")
def lib():
    so = os.path.join(PKG, "pfsgnn", "libpfsgnn.so")
    if not os.path.exists(so):
        subprocess.run(["make", "-C", PKG, "-j8"], check=True, capture_output=True)
    from pfsgnn import native
    return native.lib()


def test_library_exports_every_header_symbol(lib):
    from pfsgnn import native
    funcs = header_functions()
    assert len(funcs) >= 30
    for f in funcs:
        assert hasattr(lib, f), f"libpfsgnn.so does not export {f}"
        assert f in native._SIGS, f"native.py binds no signature for {f}"
    assert lib.pfsgnn_version().decode().startswith("pfsgnn")


def test_library_is_gfx950_code_object(lib):
    so = os.path.join(PKG, "pfsgnn", "libpfsgnn.so")
    blob = open(so, "rb").read()
    assert b"amdgcn-amd-amdhsa--gfx950" in blob or b"gfx950" in blob


def test_block_tail_struct_layout_matches(lib):
    """native.BlockTail mirrors pfsgnn_block_tail field for field: same size, and
    the last field where C puts it (every pointer is 8-byte aligned)."""
    import ctypes
    from pfsgnn import native
    assert lib.pfsgnn_block_tail_bytes() == ctypes.sizeof(native.BlockTail)
    assert native.BlockTail.Qt.offset == ctypes.sizeof(native.BlockTail) - 8
    assert lib.pfsgnn_class_bwd_bytes() == ctypes.sizeof(native.ClassBwd)
    assert native.ClassBwd.g_hsum.offset == ctypes.sizeof(native.ClassBwd) - 8


def test_workspace_query_is_host_only(lib):
    b = lib.pfsgnn_workspace_bytes(16, 2394, 128, 10)
    assert 1 << 20 < b < 1 << 31


def test_no_gpu_fails_loudly():
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    import pfsgnn
    with pytest.raises(pfsgnn.NativeUnavailable):
        pfsgnn.HipBackend()


def test_batch_collation_follows_inc(monkeypatch):
    import pfsgnn
    from pfsgnn import config
    monkeypatch.setattr(config, "device", torch.device("cpu"))
    gs = []
    for NF, NC in [(3, 2), (3, 2)]:
        e = torch.arange(NF * NC)
        ei = torch.stack([e // NC, e % NC])
        gs.append(pfsgnn.BipartiteData(ei, torch.zeros(NF, 1), torch.zeros(NC, 2), torch.zeros(NF * NC, 4),
                                       torch.zeros(1, 4)))
    b = pfsgnn.Batch.from_data_list(gs)
    assert b.edge_index[:, 6].tolist() == [3, 2]      # shifted by (x_s rows, x_t rows)
    assert b.num_graphs == 2 and b.x_s.shape == (6, 1) and b.x_t.shape == (4, 2)
    from harness import canonical_edges
    assert torch.equal(b.edge_index, canonical_edges(2, 3, 2))


def test_engine_param_order_is_reference_order():
    from pfsgnn.engine import param_names
    from oracle.ref_gnn import GNN
    for B in (1, 3):
        for normed in (True, False):
            m = GNN(B=B, Fdim=10, T=12, F_s=1, F_t=2, normed=normed)
            assert [n for n, _ in m.named_parameters()] == param_names(B, normed)


def test_noise_reference_is_uniform():
    from noise_ref import uniform_numpy
    u = uniform_numpy(7, 200000)
    assert u.min() >= 0.0 and u.max() < 1.0
    assert abs(u.mean() - 0.5) < 0.005 and abs(u.var() - 1 / 12) < 0.002
    assert (uniform_numpy(7, 10) == u[:10]).all() and (uniform_numpy(8, 10) != u[:10]).any()


def test_edge_grid_query_is_host_only(lib):
    from pfsgnn import native
    g = native.edge_grid(16, 2394, 128)
    # tail-aware split count: KS=5 fills the last dispatch round at the bench shape
    assert g == dict(KS=5, CPS=26, nblocks=3040, NFG=38)
    assert native.edge_grid(256, 2394, 16)["KS"] == 1


def test_tensor_cache_keys_on_object_not_address():
    """A freed tensor's cache entry must never serve a new tensor, even one the
    allocator places at the same address; in-place writes invalidate."""
    import gc
    from pfsgnn.gnn import _TensorCache
    c = _TensorCache(4)
    a = torch.zeros(1000)
    c.put(a, ("k",), "A")
    assert c.get(a, ("k",)) == "A"
    assert c.get(a, ("other",)) is None
    a.add_(1)                                    # bumps _version
    assert c.get(a, ("k",)) is None
    c.put(a, ("k",), "A2")
    ptr = a.data_ptr()
    del a
    gc.collect()
    for _ in range(50):                          # try to land on the same block
        b = torch.zeros(1000)
        if b.data_ptr() == ptr:
            break
    assert c.get(b, ("k",)) is None
    for i in range(10):                          # capacity: dead entries purged first
        t = torch.zeros(3)
        c.put(t, (), i)
    assert len(c.d) <= 4


def test_oversize_reduction_fails_loudly(lib):
    """a reduction wider than the packed 40-byte descriptor (rows >
    65535, cols > 32767) is refused with a non-zero return and an error text,
    before anything is launched (host-only: the pointers are never touched),
    instead of being skipped with success reported."""
    import ctypes
    from pfsgnn import native
    for rows, cols in ((70000, 4), (4, 40000)):
        r = native.Red(part=0x1000, nb=3, plen=rows * cols, ldp=cols, rows=rows, cols=cols,
                       out=0x2000, ldo=cols, add=0, scale=1.0)
        rc = lib.pfsgnn_reduce_batch(ctypes.byref(r), 1, None)
        assert rc != 0
        assert "packed descriptor" in lib.pfsgnn_last_error().decode()
