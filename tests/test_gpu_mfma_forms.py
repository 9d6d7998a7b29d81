"""MFMA form mixing on gfx950 (DESIGN.md §MFMA form mixing).

Round 2 recorded that an accumulation chain of v_mfma_f32_16x16x32_bf16
finished on the SAME accumulator by a v_mfma_f32_16x16x16_bf16 gave wrong sums
in its edge kernels, and kept every chain on one form.  This test isolates the
transition (tests/native/mfma_mix.hip): the mixed chain as hipcc schedules it
(no wait states between the two forms; hipcc even writes the first MFMA's
result over its own A operand registers), the same with 16 wait states forced
between the forms, and the other order, each against a float64 reference of
the same products (bf16 products are exact in fp32; sums of 48 of them per
element, compared at 1e-6 of their scale).  All three are exact on gfx950
(measured: 8e-8, 8e-8, 1e-7 of scale), so the hardware and hipcc's hazard
handling of the form change are not the cause; the round-2 failure lay in that
round's own operand construction for the unpaired K-tile (code that no longer
exists: every bf16 chain of pfsgnn_mfma.hip is now on the 16x16x32 form by
construction, LayerB3 / LayerB6).  The test pins that finding.
"""
import ctypes
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

LIB = os.path.join(os.path.dirname(os.path.abspath(__file__)), "native", "libmfmamix.so")


def bf16_bits(x):
    u = np.asarray(x, dtype=np.float32).view(np.uint32)
    return ((u + 0x7FFF + ((u >> 16) & 1)) >> 16).astype(np.uint16)


def bf16_val(b):
    return (b.astype(np.uint32) << 16).view(np.float32).astype(np.float64)


def reference(A, B, A2, B2):
    """D[i][j] = sum_k A[i][k] B[k][j] over the operand layouts: lane (g, i)
    holds A[i][k] for its k block, lane (g, j) B[k][j]; the x32 form's lane
    group g covers k = 8g..8g+7, the x16 form's k = 4g..4g+3."""
    D = np.zeros((16, 16))
    for t in range(2):
        a = bf16_val(A[t].reshape(4, 16, 8))      # [g][i][q]
        b = bf16_val(B[t].reshape(4, 16, 8))      # [g][j][q]
        D += np.einsum("giq,gjq->ij", a, b)
    a2 = bf16_val(A2.reshape(4, 16, 4))
    b2 = bf16_val(B2.reshape(4, 16, 4))
    D += np.einsum("giq,gjq->ij", a2, b2)
    return D


def run(A, B, A2, B2, variant):
    lib = ctypes.CDLL(LIB)
    out = np.zeros((64, 4), dtype=np.float32)
    p = lambda a: a.ctypes.data_as(ctypes.c_void_p)  # noqa: E731
    rc = lib.mfma_mix_run(p(A), p(B), p(A2), p(B2), p(out), ctypes.c_int(variant))
    assert rc == 0
    # lane (g, j) holds D[4g + r][j] in register r
    D = np.zeros((16, 16))
    for lane in range(64):
        g, j = lane >> 4, lane & 15
        for r in range(4):
            D[4 * g + r, j] = out[lane, r]
    return D


def test_mfma_form_mixing():
    import torch
    torch.cuda.init()
    rng = np.random.default_rng(3)
    A = np.ascontiguousarray(bf16_bits(rng.standard_normal((2, 64, 8))))
    B = np.ascontiguousarray(bf16_bits(rng.standard_normal((2, 64, 8))))
    A2 = np.ascontiguousarray(bf16_bits(rng.standard_normal((64, 4))))
    B2 = np.ascontiguousarray(bf16_bits(rng.standard_normal((64, 4))))
    ref = reference(A, B, A2, B2)
    scale = np.abs(ref).max()
    errs = {v: np.abs(run(A, B, A2, B2, v) - ref).max() / scale for v in (0, 1, 2)}
    print("MFMA form mixing: max |err| / scale per variant", errs)
    # every variant -- as scheduled, with forced wait states, other order --
    # is exact to fp32 rounding
    assert all(e < 1e-6 for e in errs.values()), errs
