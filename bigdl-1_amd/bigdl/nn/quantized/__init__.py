"""int8 quantized inference (``DL/nn/quantized``)."""
from .layers import Linear, SpatialConvolution, SpatialDilatedConvolution
from .quantizer import quantize, register

__all__ = ["Linear", "SpatialConvolution", "SpatialDilatedConvolution", "quantize", "register"]
