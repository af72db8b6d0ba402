"""video_st per-frame path on libstx (BASELINE.json config 5).

Reference: `VideoTransformNet.process_video` (stransfer/network.py:1071-1158): every
decoded frame is conditioned like an image (`dataset.iterate_on_video_batches`,
stransfer/dataset.py:280-310 -> `img_utils.image_loader_transform`: centre crop,
resize to IMSIZE, ImageNet normalisation), concatenated with the previous stylised
frame along channels (`torch.cat([frame, old], dim=1)`, the first frame with
itself) and run through the 6-channel ImageTransformNet; the output becomes the
next frame's `old`.  `get_temporal_loss` (:885-903) is ||dy|| / (||dx|| + 1).

`FrameEngine` makes one frame one hipGraph replay: the frame is copied into
channels 0-2 of a static [1, 6, H, W] input whose channels 3-5 hold the previous
output, the ITN forward runs on the HIP kernels, the output is copied back into
channels 3-5, and the temporal-loss norms of the step are reduced on the device
(the reference computes them only in training; here they are the per-frame
"temporal loss" of BASELINE config 5).
"""
from __future__ import annotations

import os
from typing import Iterator

import numpy as np
import torch

from . import constants, img_utils, ops

VIDEO_EXTS = (".mp4", ".avi", ".mov", ".mkv", ".gif", ".webm")
FRAME_EXTS = (".png", ".jpg", ".jpeg", ".bmp")


def iterate_raw_frames(source, max_frames=90 * 24) -> Iterator[np.ndarray]:
    """Decoded frames of a video as HxWx3 uint8 arrays (the sources of iterate_frames)."""
    from PIL import Image
    if isinstance(source, np.ndarray):
        frames = iter(source)
    elif isinstance(source, str) and source.endswith(".npy"):
        frames = iter(np.load(source, allow_pickle=False, mmap_mode="r"))
    elif isinstance(source, str) and os.path.isdir(source):
        def key(name):
            stem = os.path.splitext(name)[0]
            digits = "".join(ch for ch in stem if ch.isdigit())
            return (int(digits) if digits else -1, name)
        names = sorted((n for n in os.listdir(source) if n.lower().endswith(FRAME_EXTS)), key=key)
        frames = (np.asarray(Image.open(os.path.join(source, n)).convert("RGB")) for n in names)
    elif isinstance(source, str) and source.lower().endswith(VIDEO_EXTS):
        try:
            import imageio
        except ImportError as e:
            raise RuntimeError(f"decoding {source} needs imageio (not installed); pass a "
                               "directory of frames or a .npy frame array instead") from e
        reader = imageio.get_reader(source)

        def gen():
            try:
                while True:
                    yield np.asarray(reader.get_next_data())
            except IndexError:
                return
        frames = gen()
    else:
        raise ValueError(f"unsupported video source {source!r}")
    for i, f in enumerate(frames):
        if i >= max_frames:
            break
        f = np.ascontiguousarray(f, dtype=np.uint8)
        if f.ndim == 3 and f.shape[2] == 4:
            f = np.ascontiguousarray(f[:, :, :3])  # RGBA frame: .convert("RGB") drops alpha
        elif f.ndim == 2:
            f = np.repeat(f[:, :, None], 3, axis=2)  # grayscale: PIL "L" -> "RGB" copies
        yield f


def iterate_frames(source, max_frames=90 * 24, imsize=None) -> Iterator[torch.Tensor]:
    """Conditioned frames [1, 3, IMSIZE, IMSIZE] of a video (stransfer/dataset.py:280-310),
    through the host-side PIL transforms (img_utils.image_loader_transform).

    `source`: a video file (decoded with imageio when it is installed, as the
    reference does), a directory of frame images (sorted by the integer in their
    name, then by name), a `.npy` array [T, H, W, 3] uint8 (loaded with
    allow_pickle=False), or an in-memory uint8 array of that shape."""
    from PIL import Image
    for f in iterate_raw_frames(source, max_frames):
        yield img_utils.image_loader_transform(Image.fromarray(f), imsize)


class FrameEngine:
    """One stylised frame = one hipGraph replay of the VideoTransformNet forward.

    raw_hw=(H, W): frames arrive as decoded HxWx3 uint8 (`step_raw`) and the graph
    also holds their conditioning (centre crop, Pillow-exact resize to the engine's
    size, normalisation: img_utils.FixedConditioner) written straight into the
    frame channels of the 6-channel input -- the per-frame path of
    process_video (stransfer/network.py:1117-1131) with no host-side resize."""

    def __init__(self, net, shape, device=None, graph=True, raw_hw=None):
        self.net = net
        self.dev = torch.device(device or constants.DEVICE)
        n, c, h, w = shape
        assert c == 3 and n == 1, shape  # the reference converts one video (batch 1)
        self.x6 = torch.zeros((n, 6, h, w), device=self.dev, dtype=torch.float32)
        self.frame = self.x6[:, :3]
        self.prev = self.x6[:, 3:]
        self.prev_frame = torch.zeros((n, 3, h, w), device=self.dev, dtype=torch.float32)
        self.out = None
        # device scalars: temporal loss (weight 1), ||y_t - y_{t-1}||, ||x_t - x_{t-1}||
        self.scal = torch.zeros(4, device=self.dev, dtype=torch.float32)
        self.graph = None
        self.use_graph = graph
        self.started = False
        self.cond = None
        if raw_hw is not None:
            assert h == w, "frames are conditioned to IMSIZE x IMSIZE"
            self.cond = img_utils.ImageConditioner(h, self.dev).fixed(*raw_hw, out=self.frame)

    def _forward(self):
        if self.cond is not None:
            self.cond.run()                # uint8 frame -> normalised frame channels
        with torch.no_grad():
            y = self.net(self.x6)
        if self.out is None:
            self.out = torch.empty_like(y)
        # temporal-loss terms of this step (stransfer/network.py:885-903): one fused
        # pass, [loss(w=1), ||y - y_prev||, ||x - x_prev||]
        ops.temporal_loss(y, self.prev, self.frame, self.prev_frame, 1.0,
                          out=self.scal[:3])
        self.out.copy_(y)
        self.prev.copy_(y)                 # next step's "old stylised" channels
        self.prev_frame.copy_(self.frame)

    def step(self, frame: torch.Tensor) -> torch.Tensor:
        """Stylise one conditioned frame [n, 3, H, W]; returns the (static) output."""
        if self.cond is not None:
            raise RuntimeError("FrameEngine(raw_hw=...) takes uint8 frames: use step_raw")
        self.frame.copy_(frame)
        if not self.started:
            self.prev.copy_(frame)         # first frame: old = the frame itself
            self.prev_frame.copy_(frame)
            self.started = True
        return self._run()

    def step_raw(self, frame_u8) -> torch.Tensor:
        """Stylise one decoded HxWx3 uint8 frame (host array or device tensor)."""
        if self.cond is None:
            raise RuntimeError("FrameEngine without raw_hw takes conditioned frames: use step")
        self.cond.load(frame_u8)
        if not self.started:
            self.cond.run()                # first frame: old = the frame itself
            self.prev.copy_(self.frame)
            self.prev_frame.copy_(self.frame)
            self.started = True
        return self._run()

    def _run(self):
        if self.graph is not None:
            self.graph.replay()
        elif self.use_graph and self.out is not None:
            # the first frame ran eagerly (allocations, prepped-weight caches); capture
            # records without executing, then replay runs this frame
            self.graph = torch.cuda.CUDAGraph()
            with ops.graph_capture(self.graph):
                self._forward()
            self.graph.replay()
        else:
            self._forward()
        return self.out

    def temporal_loss(self, temporal_weight=1.0) -> float:
        """||y_t - y_{t-1}|| / (||x_t - x_{t-1}|| + 1) * w of the last step."""
        return float(self.scal[0]) * temporal_weight


def process_video(net, video_path, style_name="nsp", working_dir="workdir/", out_dir="results/",
                  fps=24.0, graph=True, max_frames=90 * 24) -> str:
    """VideoTransformNet.process_video (stransfer/network.py:1071-1158) on FrameEngine."""
    working_dir = os.path.join(constants.PROJECT_ROOT_PATH, working_dir)
    out_dir = os.path.join(constants.PROJECT_ROOT_PATH, out_dir)
    import shutil
    shutil.rmtree(working_dir, ignore_errors=True)
    os.makedirs(working_dir, exist_ok=True)
    os.makedirs(out_dir, exist_ok=True)
    eng = None
    S = constants.IMSIZE
    for i, frame in enumerate(iterate_raw_frames(video_path, max_frames)):
        # decoded uint8 frames go to the GPU as they are; crop, resize and normalisation
        # run inside the per-frame graph (bit-identical to image_loader_transform)
        if eng is None or eng.cond.h != frame.shape[0] or eng.cond.w != frame.shape[1]:
            if eng is not None:  # a clip whose frame size changes: a new engine, as the
                prev = eng.out.clone()  # reference, but keep the recurrence going
            eng2 = FrameEngine(net, (1, 3, S, S), constants.DEVICE, graph=graph,
                               raw_hw=frame.shape[:2])
            if eng is not None:
                eng2.prev.copy_(prev)
                eng2.prev_frame.copy_(eng.prev_frame)
                eng2.started = True
            eng = eng2
        y = eng.step_raw(frame)
        img_utils.imshow(y[0], path=os.path.join(working_dir, f"{i}.png"))
    final = os.path.join(out_dir, f"video_st_{style_name}.mp4")
    try:
        import imageio
    except ImportError:
        return working_dir  # frames only: no encoder in this image
    from PIL import Image
    writer = imageio.get_writer(final, fps=fps)
    names = sorted(os.listdir(working_dir), key=lambda x: int(x.split(".")[0]))
    for nm in names:
        writer.append_data(np.array(Image.open(os.path.join(working_dir, nm))))
    writer.close()
    return final
