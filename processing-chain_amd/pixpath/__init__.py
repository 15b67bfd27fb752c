"""pixpath -- MI355X-native raw-frame pixel path of the P.NATS / AVHD-AS
processing chain (pnats2avhd/processing-chain).

Layers:
  _native   ctypes binding of libpixpath.so (HIP kernels, C ABI include/pixpath.h)
  frames    device frame batches (HBM layout)
  ops       scaler plans, pad, v210, stall compositing, SI/TI, fps map
  ffmpeg    drop-in for the reference's lib/ffmpeg.py command builders
  siti      SRC_analysis / complexity_classification hooks (P.910 SI/TI)
"""
from . import formats  # noqa: F401

__version__ = "0.1.0"
