"""Native host runtime (``runtime/csrc``, built into ``runtime/lib/libbigdl_runtime.so`` by
``bigdl.ops.build.build_runtime``): components the reference runs on the JVM that sit on the hot
path around the GPU — currently the multi-threaded minibatch assembler."""
from .loader import NativeBatchLoader, runtime_library  # noqa: F401
