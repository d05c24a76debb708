from .tensor import Tensor
from .sparse import SparseTensor
from .quantized import QuantizedTensor
from .storage import Storage
