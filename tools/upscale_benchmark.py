#!/usr/bin/env python3
"""Upscale benchmark (reference tools/upscale_benchmark.py).

Reference flow: extract a clip to PNG -> realesrgan-ncnn-vulkan x{2,3,4} -> encode, printing
JSON timings.  MI355X flow, all on one GPU and without touching disk for frames:

    extract (source reader, optional bwdif deinterlace on the GPU)
      -> upscale x{2,3,4}: ``lanczos`` (HIP k_resize) or ``srnet`` (an ESPCN-style conv net on
         the luma plane in bf16, channels-last, PyTorch-ROCm/MIOpen; chroma by Lanczos)
      -> scale to the target height -> HEVC encode on the GPU engine (batched GOPs)

The SR net is random-initialised (no pretrained weights are available offline), so it
measures throughput, not quality.  Output keys follow the reference: extract/upscale/encode/
total_elapsed_s, upscale_fps, total_fps, output_size_bytes.

    python tools/upscale_benchmark.py input.y4m --frames 120 --target-height 1080 --scale 2
    python tools/upscale_benchmark.py synth:640x360:120 --engine srnet --target-height 1080
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def open_input(spec: str):
    from thinvids_amd.models import media

    if spec.startswith("synth:"):
        _, wh, n = spec.split(":")
        w, h = (int(x) for x in wh.split("x"))
        return media.SynthSource(spec={"width": w, "height": h, "frames": int(n), "fps": 30, "seed": 7})
    return media.open_source(spec)


class SRNet:
    """ESPCN-style x`scale` luma super-resolution: 5x5 conv(64) -> 3x3 conv(32) x2 -> 3x3 conv(s^2)
    -> pixel shuffle, residual over a bicubic-free nearest upsample."""

    def __init__(self, scale: int, device, dtype):
        import torch

        torch.manual_seed(0)
        nn = torch.nn
        self.scale = scale
        self.net = nn.Sequential(
            nn.Conv2d(1, 64, 5, padding=2), nn.Tanh(), nn.Conv2d(64, 32, 3, padding=1), nn.Tanh(),
            nn.Conv2d(32, 32, 3, padding=1), nn.Tanh(), nn.Conv2d(32, scale * scale, 3, padding=1),
            nn.PixelShuffle(scale)).to(device=device, dtype=dtype).to(memory_format=torch.channels_last).eval()
        self.dtype = dtype

    def __call__(self, y):  # y: (N, 1, H, W) uint8 tensor
        import torch

        with torch.inference_mode():
            x = y.to(self.dtype).contiguous(memory_format=torch.channels_last) / 255.0
            base = torch.nn.functional.interpolate(x, scale_factor=self.scale, mode="nearest")
            out = base + 0.05 * self.net(x)
            return (out.clamp(0, 1) * 255.0).round().to(torch.uint8)


def main() -> int:
    ap = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    ap.add_argument("input")
    ap.add_argument("--start-frame", type=int, default=0)
    ap.add_argument("--frames", type=int, default=120)
    ap.add_argument("--target-height", type=int, default=1080, choices=(720, 1080, 1440, 2160))
    ap.add_argument("--scale", type=int, choices=(2, 3, 4))
    ap.add_argument("--engine", choices=("lanczos", "srnet"), default="lanczos")
    ap.add_argument("--batch-frames", type=int, default=8, help="frames per upscale launch")
    ap.add_argument("--deinterlace", choices=("auto", "none", "bwdif"), default="auto")
    ap.add_argument("--qp", type=int, default=23)
    ap.add_argument("--gop", type=int, default=32)
    ap.add_argument("--output", default="upscaled_sample.mp4")
    ap.add_argument("--software-encode", action="store_true")
    a = ap.parse_args()

    import torch

    from thinvids_amd.models import hevc
    from thinvids_amd.ops.deint import deinterlace_frames
    from thinvids_amd.ops.resize import resize_plane
    from thinvids_amd.worker.encoder import EncodeSpec, EngineCache, encode_parts
    from thinvids_amd.worker.helpers import output_geometry

    gpu = torch.cuda.is_available()
    dev = torch.device("cuda", 0) if gpu else torch.device("cpu")
    t_total = time.monotonic()
    src = open_input(a.input)
    scale = a.scale or max(2, min(4, round(a.target_height / src.height)))
    t0 = time.monotonic()
    frames = src.read(a.start_frame, a.frames)
    deint = a.deinterlace == "bwdif" or (a.deinterlace == "auto" and src.height in (480, 576))
    if deint:
        frames = deinterlace_frames(frames)
    extract_s = time.monotonic() - t0
    ow, oh = output_geometry(src.width * scale, src.height * scale, a.target_height)

    t0 = time.monotonic()
    up = []
    net = SRNet(scale, dev, torch.bfloat16 if gpu else torch.float32) if a.engine == "srnet" else None
    for i in range(0, len(frames), a.batch_frames):
        chunk = frames[i:i + a.batch_frames]
        planes = [[torch.from_numpy(np.ascontiguousarray(f[c])).to(dev) for f in chunk] for c in range(3)]
        if net is not None:
            ys = net(torch.stack(planes[0])[:, None])[:, 0]
            ys = [resize_plane(y, oh, ow) if y.shape != (oh, ow) else y for y in ys]
        else:
            ys = [resize_plane(y, oh, ow) for y in planes[0]]
        us = [resize_plane(u, oh // 2, ow // 2) for u in planes[1]]
        vs = [resize_plane(v, oh // 2, ow // 2) for v in planes[2]]
        if gpu:
            torch.cuda.synchronize()
        up.extend((y.cpu().numpy(), u.cpu().numpy(), v.cpu().numpy()) for y, u, v in zip(ys, us, vs))
    upscale_s = time.monotonic() - t0

    t0 = time.monotonic()
    spec = EncodeSpec(ow, oh, qp=a.qp, gop=a.gop, software=a.software_encode or not gpu)
    cache = None if spec.software else EngineCache(batch=8)
    annexb = encode_parts([up], spec, cache)[0]
    with open(a.output, "wb") as f:
        f.write(hevc.mux_mp4(annexb, ow, oh, src.fps_num, src.fps_den))
    encode_s = time.monotonic() - t0
    total_s = time.monotonic() - t_total
    print(json.dumps({
        "input": a.input, "engine": a.engine, "scale": scale, "weights": "random-init" if net else "n/a",
        "deinterlace": bool(deint), "source": f"{src.width}x{src.height}", "output_geometry": f"{ow}x{oh}",
        "frames_extracted": len(frames), "frames_upscaled": len(up),
        "extract_elapsed_s": round(extract_s, 3), "upscale_elapsed_s": round(upscale_s, 3),
        "encode_elapsed_s": round(encode_s, 3), "total_elapsed_s": round(total_s, 3),
        "upscale_fps": round(len(up) / upscale_s, 3) if upscale_s else 0,
        "total_fps": round(len(up) / total_s, 3) if total_s else 0,
        "output_size_bytes": os.path.getsize(a.output), "device": str(dev),
    }, indent=2, sort_keys=True))
    if cache:
        cache.close()
    return 0


if __name__ == "__main__":
    sys.exit(main())
