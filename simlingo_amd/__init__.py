"""SimLingo VLA hot path, MI355X-native (gfx950 HIP kernels behind a C-ABI)."""
__version__ = "0.1.0"
