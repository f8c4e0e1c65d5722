"""janus_amd: MI355X-native batched Prio3 preparation + aggregation for Janus's aggregate-init path.

The product is the HIP library `janus_amd/lib/libprio3gpu.so` behind the C ABI in
`include/prio3gpu.h`; `janus_amd.prio3` is the host-side mirror of prio's Aggregator surface.
"""
from ._lib import Prio3GpuError, build, lib  # noqa: F401

__all__ = ["Prio3GpuError", "build", "lib"]
