"""MI355X-native per-pixel ray tracer: the hot path of D4rkFr4g/Ray_Tracer_Fragment_Shader
(rayTraceScreen -> rayTraceRay, Hw4/MySdlApplication.cpp:1184-1324) as HIP kernels behind a C ABI
(include/rt_api.h, built into lib/librt_amd.so)."""
from . import abi, scenes  # noqa: F401
