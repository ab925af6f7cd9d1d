"""StereoConfiguration (reference stereo_vision/src/stereo_configuration.cpp:4-46): the calibration
written by cv::FileStorage (``%YAML:1.0`` with ``!!opencv-matrix`` nodes, config/stereo.yaml).

loadFromFile(path) reads imageWidth/imageHeight, both camera matrices and distortion vectors,
R, T, E, F, R1, R2, P1, P2 and Q, and fails (returns False) on a missing file, a non-positive
image size or a missing essential matrix -- the reference's checks.
"""
from __future__ import annotations

import os
import re

import numpy as np
import yaml

_FIELDS = ("cameraMatrixLeft", "distCoeffsLeft", "cameraMatrixRight", "distCoeffsRight", "R", "T",
           "E", "F", "R1", "R2", "P1", "P2", "Q")
_ESSENTIAL = ("cameraMatrixLeft", "cameraMatrixRight", "R1", "R2", "P1", "P2", "Q")


class _Loader(yaml.SafeLoader):
    pass


def _opencv_matrix(loader, node):
    m = loader.construct_mapping(node, deep=True)
    dt = {"d": np.float64, "f": np.float32, "i": np.int32, "u": np.uint8, "s": np.int16, "w": np.uint16}
    return np.asarray(m["data"], dtype=dt.get(m.get("dt", "d"), np.float64)).reshape(m["rows"], m["cols"])


_Loader.add_constructor("tag:yaml.org,2002:opencv-matrix", _opencv_matrix)


def read_opencv_yaml(path: str) -> dict:
    """Parses a cv::FileStorage YAML file (the %YAML:1.0 directive is not accepted by PyYAML)."""
    with open(path) as f:
        text = f.read()
    text = re.sub(r"^%YAML:1\.0\s*\n", "", text)
    return yaml.load(text, Loader=_Loader) or {}


class StereoConfiguration:
    def __init__(self):
        self.imageSize = (0, 0)  # (width, height), cv::Size order
        for n in _FIELDS:
            setattr(self, n, None)

    def loadFromFile(self, filename: str) -> bool:
        if not os.path.exists(filename):
            return False
        d = read_opencv_yaml(filename)
        w, h = int(d.get("imageWidth", 0) or 0), int(d.get("imageHeight", 0) or 0)
        if w <= 0 or h <= 0:
            return False
        self.imageSize = (w, h)
        for n in _FIELDS:
            v = d.get(n)
            setattr(self, n, None if v is None else np.asarray(v, np.float64))
        return all(getattr(self, n) is not None and getattr(self, n).size for n in _ESSENTIAL)
