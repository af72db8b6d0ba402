"""Drop-in `stransfer` package: the reference's module names
(tupini07/StyleTransfer stransfer/__init__.py) backed by styletransfer_amd."""
from styletransfer_amd import c_logging, constants, dataset, img_utils, network

__all__ = ["c_logging", "constants", "dataset", "img_utils", "network"]
