"""fluidframework_amd — MI355X-native batch merge engine for Fluid Framework op replay.

The product is the C-ABI library `libfmt.so` (include/fmt.h) built from `csrc/` for gfx950. The
Python modules here are the host side of the drop-in boundary: stream packing (`streams`), the
ctypes binding that fails loudly when the HIP library is missing (`native`), and the
processMessagesCore-shaped adapters for SharedMap and SharedString (`map`, `sequence`).
"""
__all__ = ["streams"]
