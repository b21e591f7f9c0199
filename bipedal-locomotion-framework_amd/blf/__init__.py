"""blf — MI355X-native batched DCM-MPC planning path (bipedal-locomotion-framework drop-in).

The compute lives in lib/libblf.so (hand-written gfx950 HIP kernels behind the C ABI in
include/blf/blf_c.h); this package is the Python-side binding (`blf.native`) and the synthetic
workload generator (`blf.problems`).  The C++17 mirror of the reference's interfaces
(Advanceable, ForwardEuler, ConvexHullHelper, ContactList, ...) is in host/ (lib/libblf_host.so).
"""
from . import native, problems  # noqa: F401

__all__ = ["native", "problems"]
