"""Model zoo (``DL/models/**`` and the example models): same topology and initialisation."""
from .lenet import LeNet5  # noqa: F401
from .resnet import ResNet  # noqa: F401
from .vgg import VggForCifar10, Vgg_16, Vgg_19  # noqa: F401
from .rnn import PTBModel, SimpleRNN  # noqa: F401
from .inception import (Inception_Layer_v1, Inception_Layer_v2, Inception_v1, Inception_v1_NoAuxClassifier,  # noqa: F401
                        Inception_v2, Inception_v2_NoAuxClassifier)
from .autoencoder import Autoencoder  # noqa: F401
from .maskrcnn import MaskRCNN, MaskRCNNParams  # noqa: F401
