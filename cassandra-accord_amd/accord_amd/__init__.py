"""accord_amd — MI355X-native batched dependency calculation for Apache Cassandra Accord.

The compute path is libaccord_amd.so (hand-written HIP for gfx950 behind the C ABI in
include/accord_amd.h); this package is the thin host mirror used by tests and the bench.
"""
from . import workload  # noqa: F401

__all__ = ["workload", "deps"]


def __getattr__(name):
    if name == "deps":
        from . import deps
        return deps
    raise AttributeError(name)
