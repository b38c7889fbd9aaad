"""disq_amd -- MI355X-native BAM read path for Disq.

The compute path is libdisq_gpu.so (hand-written HIP kernels for gfx950) behind a C ABI
(include/disq_gpu.h).  This package holds its ctypes binding and a host-side mirror of Disq's
HtsjdkReadsRddStorage read API.
"""
from .storage import (HtsjdkReadsRdd, HtsjdkReadsRddStorage, HtsjdkReadsTraversalParameters,
                      Interval, ValidationStringency)

__all__ = ["HtsjdkReadsRdd", "HtsjdkReadsRddStorage", "HtsjdkReadsTraversalParameters",
           "Interval", "ValidationStringency"]
