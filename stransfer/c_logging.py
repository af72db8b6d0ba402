"""Alias of styletransfer_amd.c_logging (drop-in module name)."""
import sys as _sys

from styletransfer_amd import c_logging as _m

_sys.modules[__name__] = _m
