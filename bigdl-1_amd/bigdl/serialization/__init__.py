"""Model formats: ``.bigdl`` protobuf (module_serializer), checkpoints, Torch7 ``.t7`` (torch_file),
Caffe prototxt/caffemodel (caffe_loader / caffe_persister), TensorFlow / Keras / ONNX importers."""
from .module_serializer import save_module, load_module, save_definition, load_definition, register_module
from .checkpoint import save_checkpoint, load_latest_checkpoint, save_optim_method, load_optim_method
