"""curve_amd -- MI355X-native chunk-checksum engine for Curve's per-page CRC32C path.

Product = libcurvecrc.so (HIP kernels for gfx950 + the C ABI in include/curve_crc.h).
This package is the host-side mirror of the reference's operator surface:
  crc      -- CRC32 primitive + device page CRC / verify / fold   (src/common/crc32.h)
  scan     -- ScanMap slices and digests                          (op_request.cpp, scan_manager.cpp)
"""
from . import _lib
from .crc import CRC32, CurveCrcError, combine, shift, zeros  # noqa: F401

__all__ = ["CRC32", "CurveCrcError", "combine", "shift", "zeros", "crc"]
