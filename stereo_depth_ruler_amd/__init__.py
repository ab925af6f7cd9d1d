"""stereo_depth_ruler_amd -- MI355X-native drop-in for the stereo hot path of
Amar-Aliaga/Stereo_Depth_Ruler: cv::StereoSGBM::compute + cv::reprojectImageTo3D as hand-written
HIP/CDNA4 kernels behind a C ABI (include/sdr/sdr.h), with an OpenCV-shaped Python surface.
"""
from ._lib import SDRError, SgbmParams, WlsParams, LIB_PATH  # noqa: F401
from .sgbm import (  # noqa: F401
    MODE_HH, MODE_HH4, MODE_SGBM, MODE_SGBM_3WAY, StereoSGBM, createRightMatcher,
    cvt_bgr2gray, disparity_to_float, filterSpeckles, host_empty, reprojectImageTo3D, resize_area_half,
)
from . import cloud  # noqa: F401
from . import display  # noqa: F401
from .display import COLORMAP_JET, COLORMAP_TURBO, Display, colormap_lut  # noqa: F401
from .ximgproc import (  # noqa: F401
    DisparityWLSFilter, createDisparityWLSFilter, fastGlobalSmootherFilter,
)
from .stereo_disparity import StereoDisparity  # noqa: F401

__all__ = [
    "SDRError", "SgbmParams", "StereoSGBM", "createRightMatcher", "reprojectImageTo3D",
    "disparity_to_float", "filterSpeckles", "cvt_bgr2gray", "resize_area_half",
    "MODE_SGBM", "MODE_HH", "MODE_SGBM_3WAY", "MODE_HH4", "WlsParams", "DisparityWLSFilter",
    "createDisparityWLSFilter", "fastGlobalSmootherFilter", "StereoDisparity", "Display",
    "colormap_lut", "COLORMAP_JET", "COLORMAP_TURBO", "host_empty",
]
