"""rankops — MI355X-native CTR feature-interaction engine.

Drop-in `nn.Module`s for the reference's ranking models whose eval forward runs on
hand-written HIP kernels (gfx950) through the C ABI in include/rankops.h:

    DCNModel, cross_layer                  algorithm/DCN/dcn.py
    DeepFM                                 algorithm/DeepFM/deepfm.py
    DIN, Dice, din_attention               algorithm/DIN/din.py
    AFM, create_feature_columns            algorithm/AFM/afm.py
    DeepCrossingModel, residual_unit       algorithm/DeepCrossing/deepcrossing.py
    BSTModel, BSTTransformer               algorithm/BST/bst.py
    FwFM                                   algorithm/FwFM/fwfm.py

`rankops.sharded.ShardedDeepFM` adds the table-sharded multi-GPU DeepFM lookup (RCCL
all-to-all); `rankops.loader` (Vocabulary, BatchAssembler, wechat_vocabularies) replaces the
reference's Dataset bucketing + collate with C++ column bucketing and one H2D copy per batch;
`rankops.metrics` (EvalAccumulator, roc_auc) computes evaluate()'s loss / accuracy / AUC on the GPU;
`rankops.train` holds the HIP backward (train-mode forwards return autograd-connected outputs)
and `rankops.Adam`, a one-launch torch.optim.Adam.
Import order matters: torch first, so librankops binds to torch's HIP runtime.
"""
import torch  # noqa: F401

from ._lib import RankOpsError, error_flags, load as load_library  # noqa: F401
from .afm import AFM, create_feature_columns  # noqa: F401
from .bst import BSTModel, BSTTransformer  # noqa: F401
from .dcn import DCNModel, cross_layer  # noqa: F401
from .deepcrossing import DeepCrossingModel, residual_unit  # noqa: F401
from .deepfm import DeepFM  # noqa: F401
from .din import DIN, Dice, din_attention, din_attention_gather  # noqa: F401
from .fwfm import FwFM  # noqa: F401
from .loader import BatchAssembler, Vocabulary, label_encode, wechat_vocabularies  # noqa: F401
from .metrics import EvalAccumulator, roc_auc  # noqa: F401
from .train import Adam  # noqa: F401

__all__ = [
    "AFM", "BSTModel", "BSTTransformer", "BatchAssembler", "DCNModel", "DIN", "DeepCrossingModel", "DeepFM",
    "Dice", "FwFM", "RankOpsError", "Vocabulary", "create_feature_columns", "cross_layer", "din_attention", "din_attention_gather",
    "error_flags", "load_library", "residual_unit", "wechat_vocabularies", "EvalAccumulator", "roc_auc",
    "label_encode", "Adam",
]
