"""Consumer for tests/test_panel_shards.py: reads the panel shards of a --panel_shards session,
regroups them with the ShardAssembler and checks every whole frame against the golden
calibration of the unsharded detector."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402
import torch  # noqa: E402


def main(addr, n_groups, det, run, device):
    from psana_ray_amd.config import CommonModeParams
    from psana_ray_amd.data_reader import DataReader, EndOfStream
    from psana_ray_amd.ops import reference
    from psana_ray_amd.source import SyntheticRun

    cm = CommonModeParams.parse("default")
    srcs = [SyntheticRun("synthetic", run, det, rank=g, size=n_groups, gen_device="cpu") for g in range(n_groups)]
    n, shards = 0, 0
    with DataReader(addr, device=device, timeout_s=60) as reader:
        G = reader.panel_shards
        asm = reader.shard_assembler()
        while True:
            try:
                items = reader.read_batch(8, timeout=1.0)
            except EndOfStream:
                break
            for it in items:
                lo, hi = reader.panel_range(it)
                assert (lo, hi) == ((it.rank % G) * it.data.shape[0], (it.rank % G + 1) * it.data.shape[0])
            shards += len(items)
            for fr in asm.add(items):
                src = srcs[fr.gevt % n_groups]
                k = fr.gevt // n_groups
                raw = torch.from_numpy(src.pool[k % src.pool_frames].astype(np.int32))[None]
                exp = reference.calibrate_reference(raw, src.consts, src.create_bad_pixel_mask(),
                                                    CommonModeParams(cm.flags, cm.thr, cm.maxcorr, cm.npix_min,
                                                                     src.spec.bank_cols))[0]
                got = fr.data.cpu()
                assert tuple(got.shape) == tuple(exp.shape), (got.shape, exp.shape)
                if device == "cpu":
                    assert torch.equal(got, exp), f"event {fr.gevt} differs from the golden calibration"
                else:
                    torch.testing.assert_close(got, exp, rtol=1e-5, atol=2e-3)
                n += 1
        assert asm.pending == 0, f"{asm.pending} events incomplete"
    print(f"SHARD_OK {n} {shards} G={G}")


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]), sys.argv[3], int(sys.argv[4]), sys.argv[5])
