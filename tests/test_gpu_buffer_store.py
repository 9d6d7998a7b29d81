"""Edge-row store forms on the GPU (tests/native/buf_store.hip, the product's
own row map, offsets and loads from pfsgnn_mfma_core.h; 100 fibers x 7 classes
at Fdim 10, so lane group 3 holds one row and two masked slots, and 28 lanes
of the second block have no fiber).

* variants 2 (global stores under per-row exec masks), 3 and 4 (buffer
  stores, masked or with invalid offsets moved past the range, the row value
  copied to a float before its bit-cast) and 5 (the product's st_frows, the
  edge kernels' stores since round 4: variant 4's form) store every row
  exactly and nothing else;
* variants 0 and 1 (the same buffer stores with
  __builtin_bit_cast(unsigned int, v[r]) of the vector element itself) store
  row 0's value to all of a lane's rows: the compiler defect pinned on the
  CPU by tests/test_bitcast_vector_element.py -- the cause of round 3's
  "buffer-store miscompile", which was not the buffer stores.
"""
import ctypes
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

LIB = os.path.join(os.path.dirname(os.path.abspath(__file__)), "native", "libbufstore.so")
F, NF, NC = 10, 100, 7
SENT = -12345.0


def rows_of_lane(g):
    """Feature rows of lane group g at Fdim 10 (GM<10>: 3 slots per group)."""
    return [g * 3 + s for s in range(3) if g * 3 + s < F]


def run(x, variant):
    lib = ctypes.CDLL(LIB)
    y = np.full_like(x, SENT)
    p = lambda a: a.ctypes.data_as(ctypes.c_void_p)  # noqa: E731
    assert lib.buf_store_run(p(x), p(y), NF, NC, variant) == 0
    return y


def test_edge_row_store_forms():
    import torch
    torch.cuda.init()
    rng = np.random.default_rng(11)
    x = rng.standard_normal((F, NC * NF)).astype(np.float32)      # [F][E], e = c*NF + f
    want = (x.astype(np.float64) * 2 + 1).astype(np.float32)   # = fmaf(x, 2, 1): 2x is exact
    for v in (2, 3, 4, 5):
        y = run(x, v)
        assert np.array_equal(y, want), f"variant {v}"
    # the defect's signature: every row of a lane holds its first row's value
    bcast = np.empty_like(x)
    for g in range(4):
        rows = rows_of_lane(g)
        bcast[rows] = want[rows[0]]
    for v in (0, 1):
        y = run(x, v)
        print(f"variant {v}: rows equal to the lane's row 0: "
              f"{np.mean(y == bcast):.3f}; equal to the true rows: {np.mean(y == want):.3f}")
        assert np.array_equal(y, bcast), f"variant {v} no longer shows the defect"
