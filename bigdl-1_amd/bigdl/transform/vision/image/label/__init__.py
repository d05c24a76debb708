"""ROI labels and label-aware transforms (``DL/transform/vision/image/label/roi``)."""
from .roi import RoiLabel, RoiNormalize, RoiHFlip, RoiResize, RoiProject, BboxUtil

__all__ = ["RoiLabel", "RoiNormalize", "RoiHFlip", "RoiResize", "RoiProject", "BboxUtil"]
