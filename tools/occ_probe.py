#!/usr/bin/env python3
"""Runtime occupancy of the render kernels (rt_diag_kernel_occupancy) at the LDS the launches use."""
import ctypes
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402,F401

from ray_tracer_fragment_shader_amd import abi  # noqa: E402

L = abi.lib()
torch.zeros(1, device="cuda")
out = {}
for depth in (0, 1, 2, 3):
    for variant in (0, 1):
        for lds in (0, 3 * 24 * 64, 4 * 24 * 64, 5 * 24 * 64, 8192, 16384):
            n = ctypes.c_int(0)
            rc = L.rt_diag_kernel_occupancy(depth, variant, lds, ctypes.byref(n))
            out[f"B{depth}v{variant}lds{lds}"] = n.value if rc == 0 else f"rc{rc}"
print(json.dumps(out))
