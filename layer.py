"""Drop-in replacement for the reference's ``layer.py``.

Put this repository ahead of the reference on ``sys.path`` and the reference's
``trainer.py`` (``from layer import GCN``, trainer.py:25) trains on the
gfx950 kernels without any other change.  See INTEGRATION.md.
"""
from gcn_amd import GCN, GraphConvolution  # noqa: F401

__all__ = ["GraphConvolution", "GCN"]
