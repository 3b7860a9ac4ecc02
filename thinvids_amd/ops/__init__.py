"""Pre-processing ops of the transcode pipeline (HIP kernels in csrc/gpu/k_ops.hip).

* :mod:`.resize`  — Lanczos plane/frame resampling (``scale=-2:H``);
* :mod:`.color`   — RGB/P010 -> I420 conversion, HDR10 PQ -> SDR tone mapping;
* :mod:`.overlay` — frame-number stamping (``drawtext text=%{n}``).

Each op takes either numpy arrays (float64 reference path) or torch tensors; a GPU tensor
always runs the HIP kernel and raises if the native library is unavailable.
"""
from .color import p010_to_i420, rgb_to_i420, tonemap_pq  # noqa: F401
from .overlay import label_mask, stamp_frames_gpu, stamp_ref  # noqa: F401
from .resize import filter_table, resize_frame, resize_plane  # noqa: F401
