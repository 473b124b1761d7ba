"""lbic -- MI355X-native block-level masked-convolution codec (host side).

The hot path (the raster closed-loop encode/decode of ``BlockBasedImgCompLossyNetv9``,
graphs/models/BlockBasedImgCompLossy_net.py:319-452 in the reference) runs in HIP kernels inside
``liblbic.so``; this package is the Python mirror of the reference's model / agent interface that
calls it through the C ABI declared in ``include/lbic.h``.
"""
from .arch import Arch, arch_from_config  # noqa: F401
