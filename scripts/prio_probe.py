#!/usr/bin/env python3
"""What the HIP runtime reports for stream priorities (the READY / pull gates' safety check)."""
import ctypes

import torch

torch.cuda.init()
hip = ctypes.CDLL("libamdhip64.so")
lo, hi = ctypes.c_int(7), ctypes.c_int(7)
print("hipDeviceGetStreamPriorityRange rc", hip.hipDeviceGetStreamPriorityRange(ctypes.byref(lo), ctypes.byref(hi)),
      "least", lo.value, "greatest", hi.value)
for name, st in (("null", None), ("torch current", torch.cuda.current_stream().cuda_stream),
                 ("torch high", torch.cuda.Stream(priority=-1).cuda_stream)):
    p = ctypes.c_int(7)
    rc = hip.hipStreamGetPriority(ctypes.c_void_p(st), ctypes.byref(p))
    print(f"hipStreamGetPriority({name}) rc {rc} priority {p.value}")
s = ctypes.c_void_p()
rc = hip.hipStreamCreateWithPriority(ctypes.byref(s), 1, hi.value)
p = ctypes.c_int(7)
print("created with greatest: rc", rc, "get rc", hip.hipStreamGetPriority(s, ctypes.byref(p)), "priority", p.value)
