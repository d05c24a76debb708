"""Layer library, grouped by family (see each module's docstring for the reference citations)."""
from .conv import *  # noqa: F401,F403
from .normalization import *  # noqa: F401,F403
from .activation import *  # noqa: F401,F403
from .linear import *  # noqa: F401,F403
from .pooling import *  # noqa: F401,F403
from .shape import *  # noqa: F401,F403
from .table_ops import *  # noqa: F401,F403
from .math_ops import *  # noqa: F401,F403
from .dropout import *  # noqa: F401,F403
from .embedding import *  # noqa: F401,F403
from .recurrent import *  # noqa: F401,F403
from .attention import Attention, FeedForwardNetwork, Transformer, SequenceBeamSearch  # noqa: F401
from .detection import (Anchor, Nms, Proposal, RegionProposal, PriorBox, DetectionOutputSSD,  # noqa: F401
                        DetectionOutputFrcnn, Pooler, FPN, BoxHead, MaskHead, nms, box_iou, roi_align)
from .tree_lstm import TreeLSTM, BinaryTreeLSTM, TensorTree  # noqa: F401
from .sparse import DenseToSparse, SparseJoinTable  # noqa: F401
