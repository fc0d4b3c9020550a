"""Consumer for tests/test_cli.py::test_calibrate_on_read_cpu: reads every frame of a
--calibrate_on_read session through DataReader and checks it against the golden calibration."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402
import torch  # noqa: E402


def main(addr, n_prod, det, run):
    from psana_ray_amd.config import CommonModeParams
    from psana_ray_amd.data_reader import DataReader, EndOfStream
    from psana_ray_amd.ops import reference
    from psana_ray_amd.source import SyntheticRun

    cm = CommonModeParams.parse("default")
    srcs = [SyntheticRun("synthetic", run, det, rank=r, size=n_prod, gen_device="cpu") for r in range(n_prod)]
    n = 0
    with DataReader(addr, device="cpu", timeout_s=60) as reader:
        assert reader.calibrator is not None, "expected a calibrate_on_read session"
        cal_cm = reader.calibrator.cm
        while True:
            try:
                item = reader.read(timeout=1.0)
            except EndOfStream:
                break
            if item is None:
                continue
            rank, idx, data, pe = item
            src = srcs[rank]
            raw = torch.from_numpy(src.pool[idx % src.pool_frames].astype(np.int32))[None]
            mask = src.create_bad_pixel_mask()
            exp = reference.calibrate_reference(raw, src.consts, mask, cal_cm)[0]
            assert data.dtype == torch.float32 and tuple(data.shape) == tuple(exp.shape), (data.dtype, data.shape)
            assert torch.equal(data, exp), f"frame {rank}/{idx} differs from the golden calibration"
            n += 1
    assert cm.flags == cal_cm.flags
    print(f"COR_OK {n}")


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]), sys.argv[3], int(sys.argv[4]))
