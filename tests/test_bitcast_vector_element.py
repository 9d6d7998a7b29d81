"""The compiler defect behind round 3's "buffer-store miscompile" (CPU: hipcc
only, nothing runs).

Round 3 saw the edge kernels store ONE row's value to all of a lane's rows
when the row stores were buffer stores (DESIGN.md §Edge-row stores).  The
cause is not the buffer stores: __builtin_amdgcn_raw_buffer_store_b32 takes
its data as an unsigned int, and handing it a float element of a floatx4
(ext_vector_type) as ``__builtin_bit_cast(unsigned int, v[r])`` makes this
hipcc (ROCm 7.2 clang) read element 0 of the vector for EVERY r: the
bit-cast of a vector-element subscript is emitted as a load from the
vector's own address.  tests/native/bitcast_elem.hip is the minimal form
(no buffers at all); here its LLVM IR shows the broadcast of element 0
(``k_elem``) next to the correct per-element extraction once the element is
copied to a float first (``k_temp``).  tests/test_gpu_buffer_store.py runs
the edge-row store forms on the GPU.  If a later compiler fixes the defect,
the first assertion fails and says so: the product's workaround (a float
temporary, or the global-store form st_frows) stays correct either way.
"""
import os
import re
import shutil
import subprocess

import pytest

HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
SRC = os.path.join(os.path.dirname(os.path.abspath(__file__)), "native", "bitcast_elem.hip")


def kernel_ir(ir, name):
    m = re.search(r"define[^\n]*@" + name + r"[^\n]*\{\n(.*?)\n\}", ir, re.S)
    assert m, name
    return m.group(1)


@pytest.mark.skipif(not (os.path.exists(HIPCC) or shutil.which("hipcc")), reason="no hipcc")
def test_bitcast_of_vector_element_reads_element_zero(tmp_path):
    out = tmp_path / "bc.ll"
    subprocess.run([HIPCC, "-O3", "--offload-arch=gfx950", "--cuda-device-only", "-S",
                    "-emit-llvm", "-o", str(out), SRC], check=True, capture_output=True)
    ir = out.read_text()
    elem = kernel_ir(ir, "_Z6k_elemPKDv4_fPj")
    temp = kernel_ir(ir, "_Z6k_tempPKDv4_fPj")
    # k_temp: the whole vector is loaded and every lane of it stored
    assert "load <4 x i32>" in temp and "<i32 2, i32 3>" in temp, temp
    # k_elem: only element 0 is loaded, and broadcast to every output
    assert "load <1 x i32>" in elem and "zeroinitializer" in elem, (
        "hipcc no longer broadcasts element 0 for __builtin_bit_cast of a vector "
        "element (the defect is fixed in this compiler):\n" + elem)
