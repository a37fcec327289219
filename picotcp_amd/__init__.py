"""picotcp_amd -- MI355X-native drop-in for picoTCP's Internet-checksum path.

The product is libpicocsum.so (C ABI, include/pico_csum.h): HIP kernels for
gfx950 behind picoTCP's pico_checksum / pico_dualbuffer_checksum surface plus
batched entry points.  `picotcp_amd.batch` calls it on torch device tensors.
"""
from ._lib import LIB_PATH, EXPORTED, load  # noqa: F401

__all__ = ["LIB_PATH", "EXPORTED", "load"]
