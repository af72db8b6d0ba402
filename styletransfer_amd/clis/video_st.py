"""`video_st` commands (mirror of stransfer/clis/video_st.py).  Video I/O needs
imageio, which this image lacks; the per-frame network is VideoTransformNet
(a "next" row)."""
import click


@click.group()
def video_st():
    """Video Style Transfer"""


def _need_imageio():
    try:
        import imageio  # noqa: F401
    except ImportError as e:
        raise click.ClickException("video_st needs imageio (not installed in this image)") from e


@video_st.command()
@click.argument("style-image-path")
@click.option("-e", "--epochs", default=50)
@click.option("-b", "--batch-size", default=4)
@click.option("-cw", "--content-weight", default=1)
@click.option("-sw", "--style-weight", default=100_000)
@click.option("-tw", "--temporal-weight", default=0.8)
@click.option("--use-pretrained-fast-st", is_flag=True)
def train(style_image_path, epochs, batch_size, content_weight, style_weight, temporal_weight,
          use_pretrained_fast_st):
    """Train the video style transfer network."""
    _need_imageio()
    raise click.ClickException("video_st train is not implemented yet (SURVEY.md §8f row 1)")


@video_st.command()
@click.argument("video-path")
@click.argument("style-name")
@click.option("-o", "--out-dir", default="results/")
@click.option("--fps", default=24.0)
def convert_video(video_path, style_name, out_dir, fps):
    """Convert a video with a pretrained video network (stransfer/clis/video_st.py).
    VIDEO_PATH: a video file (needs imageio), a directory of frames or a .npy array."""
    import torch

    from .. import network
    sty = network.VideoTransformNet(torch.rand([3, 255, 255]))  # as the reference CLI
    out = sty.process_video(video_path=video_path, style_name=style_name, out_dir=out_dir,
                            fps=fps)
    click.echo(f"stylised video: {out}")
