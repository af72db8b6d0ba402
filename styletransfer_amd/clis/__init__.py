"""`python -m stransfer` command groups (mirror of stransfer/clis/__init__.py)."""
import click

from . import fast_st, gatys_st, video_st


@click.group(commands={
    "video_st": video_st.video_st,
    "fast_st": fast_st.fast_st,
    "gatys_st": gatys_st.gatys_st,
})
def cli():
    """Style Transfer (MI355X)"""
