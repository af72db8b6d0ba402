"""Alias of styletransfer_amd.img_utils (drop-in module name)."""
import sys as _sys

from styletransfer_amd import img_utils as _m

_sys.modules[__name__] = _m
