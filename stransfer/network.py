"""Alias of styletransfer_amd.network (drop-in module name)."""
import sys as _sys

from styletransfer_amd import network as _m

_sys.modules[__name__] = _m
