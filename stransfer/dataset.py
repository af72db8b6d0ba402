"""Alias of styletransfer_amd.dataset (drop-in module name)."""
import sys as _sys

from styletransfer_amd import dataset as _m

_sys.modules[__name__] = _m
