"""koordinator_amd — MI355X-native batched Filter/Score engine for koord-scheduler.

The hot path (LoadAwareScheduling + NodeResourcesFit Filter/Score over pods × nodes, and the
sequential placement cycle) runs as hand-written HIP kernels for gfx950 behind the C-ABI in
include/koord_gpu.h; this package is the host-side glue (object model → rows, engine handle,
plugin mirror, multi-GPU sharding).
"""
__all__ = ["objects", "config", "engine", "synth", "plugins"]
