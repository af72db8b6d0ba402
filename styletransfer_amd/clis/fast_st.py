"""`fast_st` commands (mirror of stransfer/clis/fast_st.py:11-63)."""
import os

import click
import torch

from .. import c_logging, constants, dataset, img_utils, network

LOGGER = c_logging.get_logger()


@click.group()
def fast_st():
    """Fast Style Transfer"""


@fast_st.command()
@click.argument("style-image-path")
@click.option("-e", "--epochs", default=50, help="How many epochs the training will take")
@click.option("-b", "--batch-size", default=4, help="Batch size for training")
@click.option("-cw", "--content-weight", default=1,
              help="The weight we will assign to the content loss during the optimization")
@click.option("-sw", "--style-weight", default=100_000,
              help="The weight we will assign to the style loss during the optimization")
@click.option("--synthetic", default=0, type=int,
              help="Train on N synthetic images instead of local COCO (no network here)")
def train(style_image_path, epochs, batch_size, content_weight, style_weight, synthetic):
    """Train the fast style transfer network (checkpoint per epoch in data/models/)."""
    from .. import distributed
    distributed.from_env()  # torchrun: one rank per GPU, bound before anything allocates
    style_name = style_image_path.split("/")[-1]
    LOGGER.info("Training fast style transfer network with style name: %s", style_name)
    style_image = img_utils.image_loader(
        os.path.join(constants.PROJECT_ROOT_PATH, style_image_path))
    net = network.ImageTransformNet(style_image, batch_size)
    loaders = ((lambda shard: dataset.get_synthetic_loader(batch_size, n_train=synthetic,
                                                            shard=shard))
               if synthetic else None)
    net.static_train(style_name=style_name, epochs=epochs, style_weight=style_weight,
                     content_weight=content_weight, loaders=loaders)


@fast_st.command()
@click.argument("image-path")
@click.argument("style-name")
@click.option("-o", "--out-dir", default="results/",
              help="The results directory where the converted image will be saved")
def convert_image(image_path, style_name, out_dir):
    """Convert IMAGE-PATH with the network pretrained on STYLE-NAME (data/models/)."""
    sty = network.ImageTransformNet(torch.rand([3, 255, 255]))
    sty.process_image(image_path=image_path, style_name=style_name, out_dir=out_dir)
