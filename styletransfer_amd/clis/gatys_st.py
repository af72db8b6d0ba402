"""`gatys_st` command (mirror of stransfer/clis/gatys_st.py:10-49)."""
import os

import click

from .. import c_logging, constants, img_utils, network

LOGGER = c_logging.get_logger()


@click.command()
@click.argument("content-image-path")
@click.argument("style-image-path")
@click.option("-n", "--out-name", default="gatys_converted.png",
              help="The name of the result file (transformed image)")
@click.option("-s", "--steps", default=300,
              help="How many iterations should the optimization go through.")
@click.option("-cw", "--content-weight", default=1,
              help="The weight we will assign to the content loss during the optimization")
@click.option("-sw", "--style-weight", default=100_000,
              help="The weight we will assign to the style loss during the optimization")
@click.option("--optimizer", type=click.Choice(["lbfgs", "adam"]), default="lbfgs",
              help="lbfgs = the reference's train_gatys; adam = one hipGraph replay per iteration")
def gatys_st(content_image_path, style_image_path, out_name, steps, content_weight, style_weight,
             optimizer):
    """Run the original Gatys style transfer (slow)."""
    style_image = img_utils.image_loader(
        os.path.join(constants.PROJECT_ROOT_PATH, style_image_path))
    content_image = img_utils.image_loader(
        os.path.join(constants.PROJECT_ROOT_PATH, content_image_path))
    net = network.StyleNetwork(style_image, content_image)
    train = net.train_gatys if optimizer == "lbfgs" else net.train_gatys_adam
    converted = train(style_image=style_image, content_image=content_image,
                      style_weight=style_weight, content_weight=content_weight, steps=steps)
    out_dir = os.path.join(constants.PROJECT_ROOT_PATH, "results")
    os.makedirs(out_dir, exist_ok=True)
    out_file = os.path.join(out_dir, out_name)
    img_utils.imshow(converted, path=out_file)
    LOGGER.info("Done! Transformed image has been saved to: %s", out_file)
