"""`video_st` commands (mirror of stransfer/clis/video_st.py:11-87).  Decoding
video files needs imageio, which this image lacks; frame directories and .npy
frame arrays work without it."""
import click


@click.group()
def video_st():
    """Video Style Transfer"""


@video_st.command()
@click.argument("style-image-path")
@click.option("-e", "--epochs", default=50)
@click.option("-b", "--batch-size", default=4)
@click.option("-cw", "--content-weight", default=1)
@click.option("-sw", "--style-weight", default=100_000)
@click.option("-tw", "--temporal-weight", default=0.8)
@click.option("--use-pretrained-fast-st", is_flag=True)
@click.option("--synthetic", default=0, type=int,
              help="Train on N synthetic clips instead of data/video/ (no network here)")
def train(style_image_path, epochs, batch_size, content_weight, style_weight, temporal_weight,
          use_pretrained_fast_st, synthetic):
    """Train the video style transfer network (checkpoint per epoch in data/models/).

    Videos come from data/video/: video files (need imageio), directories of frames
    or .npy [T, H, W, 3] uint8 arrays."""
    import os

    from .. import c_logging, constants, dataset, img_utils, network
    log = c_logging.get_logger()
    style_name = style_image_path.split("/")[-1]
    log.info("Training video style transfer network with style name: %s", style_name)
    ft = None
    if use_pretrained_fast_st:
        log.info("Trying to load pretrained fast ST weights")
        try:
            ft = network._load_latest_model_weigths("fast_st", style_name)
        except AssertionError:
            log.warning("Couldn't load pretrained weights")
    style_image = img_utils.image_loader(os.path.join(constants.PROJECT_ROOT_PATH,
                                                      style_image_path))
    net = network.VideoTransformNet(style_image, batch_size, fast_transfer_dict=ft)
    loader = None
    if synthetic:
        clips = [dataset.synthetic_video(16, constants.IMSIZE, seed=i) for i in range(synthetic)]
        loader = dataset.VideoDataset(videos=clips, batch_size=batch_size)
    net.video_train(style_name=style_name, epochs=epochs, style_weight=style_weight,
                    content_weight=content_weight, temporal_weight=temporal_weight,
                    video_loader=loader)


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
