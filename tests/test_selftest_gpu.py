import pytest
import torch

pytestmark = pytest.mark.gpu


def test_xor_lane_exchanges(cuda_device, native):
    out = torch.full((6 * 64,), -1, dtype=torch.int32, device=cuda_device)
    native.xor_lane_selftest(int(out.data_ptr()), int(torch.cuda.current_stream().cuda_stream))
    torch.cuda.synchronize()
    got = out.view(6, 64).cpu()
    for j in range(6):
        J = 1 << j
        exp = torch.tensor([l ^ J for l in range(64)], dtype=torch.int32)
        assert torch.equal(got[j], exp), f"xor {J}: {got[j].tolist()}"
