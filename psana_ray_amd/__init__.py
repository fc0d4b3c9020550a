"""psana_ray_amd -- an MI355X-native detector-frame streaming framework with the capabilities of
carbonscott/psana-ray: MPI-launched producers calibrate LCLS detector frames with hand-written
gfx950 HIP kernels and stream them through an elastic queue of HBM rings (independent
producer -> consumer links, HIP IPC peer copies over xGMI) to ``DataReader`` consumers.

Layout: ``models`` (detectors, constants, geometry, calibration pipeline), ``ops`` (HIP kernel
wrappers + fp32 golden models), ``queue`` (HBM ring / session / endpoint / CPU queue),
``parallel`` (launch env, rendezvous), ``source`` (synthetic / raw-run / psana), ``utils``.
"""
__version__ = "0.1.0"

from .config import CommonModeParams, PeakFinderParams, QueueConfig  # noqa: E402
from .models.detector import ImageRetrievalMode, Mode  # noqa: E402

__all__ = ["CommonModeParams", "PeakFinderParams", "QueueConfig", "Mode", "ImageRetrievalMode", "__version__"]
