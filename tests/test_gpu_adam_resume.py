"""Resume from the reference's optimizer state on the HIP library
(tests/test_adam_resume.py has the CPU version and the description): the
real pfsgnn.GNN step on the device, FusedAdam (pfsgnn_adam) in both modes
against torch.optim.Adam on the same device (its default device kernels,
whose rounding FusedAdam follows: moments and parameters bitwise equal)."""
import pytest
import torch

pytestmark = pytest.mark.gpu

from test_adam_resume import check_resume, run_resume  # noqa: E402


@pytest.mark.parametrize("capturable", [False, True])
def test_gpu_resume_from_reference_adam_state(capturable):
    import pfsgnn
    wp, wm = check_resume(*run_resume(pfsgnn, "cuda", capturable), max_ulp=0)
    print(f"capturable={capturable}: worst difference vs torch.optim.Adam on the device: "
          f"parameters {wp:.2f} ulp, moments {wm:.2f} ulp")
