"""fpm — MI355X-native GNN graph-matching forward of the fingerprint QAP matcher.

Import as ``import fpm`` (root-level shim; this directory's name has hyphens).
Public surface mirrors the reference: ``Net`` (src/model/ngm.py), plus the op wrappers in
``fpm.ops`` and the host-side Hungarian/greedy helpers in ``fpm.lap``.
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
