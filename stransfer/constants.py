"""Alias of styletransfer_amd.constants (drop-in module name)."""
import sys as _sys

from styletransfer_amd import constants as _m

_sys.modules[__name__] = _m
