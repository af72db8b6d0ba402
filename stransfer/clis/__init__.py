"""Alias of styletransfer_amd.clis."""
from styletransfer_amd.clis import cli, fast_st, gatys_st, video_st  # noqa: F401
