"""Consumer for tests/test_psana_wrapper.py: reads every frame of a session through DataReader
until the end of the stream and saves it as <outdir>/<rank>_<idx>.npy (+ photon energies)."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main(addr, outdir, device):
    from psana_ray_amd.data_reader import DataReader, EndOfStream

    os.makedirs(outdir, exist_ok=True)
    pe = {}
    with DataReader(addr, device=None if device == "auto" else device, as_numpy=True, timeout_s=120) as reader:
        while True:
            try:
                item = reader.read(timeout=1.0)
            except EndOfStream:
                break
            if item is None:
                continue
            rank, idx, data, photon_energy = item
            import numpy as np

            np.save(os.path.join(outdir, f"{rank}_{idx}.npy"), np.asarray(data))
            pe[f"{rank}_{idx}"] = photon_energy
    with open(os.path.join(outdir, "pe.json"), "w") as f:
        json.dump(pe, f)
    print(f"PSANA_CONSUMER_OK {len(pe)}")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2], sys.argv[3])
