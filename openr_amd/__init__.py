"""openr_amd — MI355X-native Decision SPF engine (LinkState / SpfSolver).

The HIP engine lives in libopenr_spf.so (C ABI: include/openr_spf.h); the
C++ LinkState / SpfSolver re-implementation is exposed to Python as
openr_amd._openr_spf.  Nothing here falls back to a CPU path.
"""
