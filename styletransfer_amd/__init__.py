"""styletransfer_amd — MI355X-native engine for the tupini07/StyleTransfer hot path.

Host code (this package) mirrors the reference `stransfer` API; arithmetic runs in
libstx.so (hand-written HIP for gfx950, C ABI in include/stx.h)."""
__version__ = "0.1.0"
