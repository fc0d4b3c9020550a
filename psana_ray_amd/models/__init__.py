"""Detector models: specs, geometry, calibration constants and the calibration pipeline."""
from .calibrator import Calibrator
from .constants import CalibConstants, run_seed
from .detector import (EPIX10K2M, EPIX10KA, JUNGFRAU4M, JUNGFRAU16M, PLAIN256, TINY_EPIX, TINY_JUNGFRAU,
                       TINY_PLAIN, DetectorSpec, ImageRetrievalMode, Mode, get_detector, list_detectors)
from .geometry import Geometry, make_geometry

__all__ = ["Calibrator", "CalibConstants", "run_seed", "DetectorSpec", "Mode", "ImageRetrievalMode",
           "get_detector", "list_detectors", "Geometry", "make_geometry", "EPIX10K2M", "EPIX10KA",
           "JUNGFRAU16M", "JUNGFRAU4M", "PLAIN256", "TINY_EPIX", "TINY_JUNGFRAU", "TINY_PLAIN"]
