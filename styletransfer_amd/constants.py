"""Constants (mirror of stransfer/constants.py).

Differences from the reference (stransfer/constants.py:20-30):
  * the reference calls `torch.set_default_tensor_type(torch.cuda.FloatTensor)`
    at import; this package does not change torch's global defaults — every
    entry point moves its inputs to `DEVICE` itself;
  * `IMSIZE` can be overridden with $STX_IMSIZE (the 512x512 Gatys config).
"""
import os

import torch

RUNS_PATH = "runs/"
LOG_PATH = os.path.join(RUNS_PATH, "runtime.log")

IMAGENET_MEAN = [0.485, 0.456, 0.406]
IMAGENET_STD = [0.229, 0.224, 0.225]

# device_count() (not is_available()) so that importing the package does not initialise
# the HIP runtime: launchers (bench.py --gpus N, the DP tests) spawn their GPU ranks from
# a parent that must never touch the GPU
DEVICE = torch.device("cuda" if torch.cuda.device_count() > 0 else "cpu")

IMSIZE = int(os.environ.get("STX_IMSIZE", "256"))

PROJECT_ROOT_PATH = os.environ.get(
    "STX_PROJECT_ROOT",
    os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
