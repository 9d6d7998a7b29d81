"""The loss kernels' two forms against the fp64 oracle.

LOSS_FAST (the library default, csrc/pfsgnn_loss.hip) computes softfloor's
sin / cos(2 pi x) (train.py:24-27) as sincospi(2x) and the two divisions by
T_i as one reciprocal; torch's fp32 form rounds the product 2 pi x first, so
the two differ by up to 2^-24 |2 pi x| rad in the angle, growing with the
visit count x = time / T_i.  The exact form (LOSS_FAST=0) is built as
tests/native/libpfsgnn_lossexact.so.  Both run one training step at
x ~ 10..63 visits (decoder bias raised) and every loss / gradient is held to
test_gpu_parity's bar against the fp64 oracle -- the reference's arithmetic
without fp32 rounding, which neither form reproduces bit for bit."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
EXACT = os.path.join(HERE, "native", "libpfsgnn_lossexact.so")


def run_case(libpath=None):
    env = dict(os.environ)
    env.pop("PFSGNN_LIB_VARIANT", None)
    if libpath:
        env["PFSGNN_LIB_PATH"] = libpath
    r = subprocess.run([sys.executable, os.path.join(HERE, "loss_form_case.py")], env=env,
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    line = [l for l in r.stdout.splitlines() if l.startswith("{")][-1]
    return json.loads(line)


def test_loss_fast_and_exact_forms_match_oracle():
    assert os.path.exists(EXACT), "build it: make -C pfs-neural-net_amd"
    fast, exact = run_case(), run_case(EXACT)
    assert fast["lib"] == "libpfsgnn.so" and exact["lib"] == "libpfsgnn_lossexact.so"
    print("LOSSFORM fast", fast["worst"], f"{fast['worst_ratio']:.3f}",
          "loss ratio", f"{fast['ratios']['loss']:.3f}")
    print("LOSSFORM exact", exact["worst"], f"{exact['worst_ratio']:.3f}",
          "loss ratio", f"{exact['ratios']['loss']:.3f}")
    for r in (fast, exact):
        assert r["worst_ratio"] <= 1.0, r
