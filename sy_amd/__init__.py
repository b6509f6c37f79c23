"""sy_amd — MI355X-native delta-sync hot path of nijaru/sy (src/delta).

``sy_amd.delta`` mirrors src/delta's public API; ``sy_amd.device`` exposes the
device-resident kernels; both sit on libsydelta.so (include/sydelta.h) and
raise ImportError when it is missing (no CPU fallback).  ``sy_amd.build``
compiles the library and must stay importable without it.
"""

__all__ = ["delta", "device", "build"]
