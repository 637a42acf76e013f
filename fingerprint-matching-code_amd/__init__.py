"""fpm — MI355X-native GNN graph-matching forward of the fingerprint QAP matcher.

Import as ``import fpm`` (root-level shim; this directory's name has hyphens).
Public surface mirrors the reference: ``Net`` (src/model/ngm.py); ``fpm.parallel.ShardedNet``
(pair-sharded forward over several GPUs of one process, in place of src/parallel's DataParallel);
the reference-signature operators ``fpm.ops.Sinkhorn`` / ``soft_topk`` / ``greedy_perm`` /
``hungarian`` (src/model/sinkhorn.py, src/model/soft_topk.py, utils/hungarian.py) beside the raw
kernel wrappers in ``fpm.ops``; ``fpm.sparse_torch`` / ``fpm.fgm`` / ``fpm.gconv`` for the
reference's CSX containers, factorised graph matching and Gconv.
"""
from . import config  # noqa: F401
from . import params  # noqa: F401

__version__ = "0.1.0"


def __getattr__(name):
    # lazy: importing the package must not require torch.cuda or the built library
    if name == "Net":
        from .model import Net
        return Net
    if name == "DeviceBatch":
        from .batch import DeviceBatch
        return DeviceBatch
    raise AttributeError(name)
