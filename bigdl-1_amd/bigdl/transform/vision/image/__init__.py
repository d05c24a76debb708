"""Vision image pipeline: ImageFeature/ImageFrame, augmentations, convertors, ROI labels
(``DL/transform/vision/image``)."""
from .image_feature import (ImageFeature, ImageFrame, LocalImageFrame, DistributedImageFrame, FeatureTransformer,
                            ChainedFeatureTransformer, Pipeline)
from .augmentation import (BatchSampler, RandomSampler, PixelNormalize, Brightness, Contrast, Saturation, Hue, ChannelOrder, ColorJitter, ChannelNormalize,
                           ChannelScaledNormalizer, PixelNormalizer, HFlip, Resize, AspectScale, RandomAspectScale,
                           RandomResize, ScaleResize, Crop, CenterCrop, RandomCrop, FixedCrop, DetectionCrop,
                           RandomCropper, RandomAlterAspect, Expand, FixExpand, Filler, RandomTransformer, resize_mat,
                           bgr_to_hsv, hsv_to_bgr)
from .convertor import (BytesToMat, PixelBytesToMat, MatToFloats, MatToTensor, ImageFrameToSample,
                        ImageFeatureToMiniBatch, MTImageFeatureToBatch, decode_bytes)
from .label import RoiLabel, RoiNormalize, RoiHFlip, RoiResize, RoiProject, BboxUtil

from ....dataset.seqfile import SeqFileFolder  # noqa: E402,F401  (pyspark image.SeqFileFolder)
