"""Probe: external event records inside HIP stream capture, engine loaded (diagnostic)."""
import ctypes as C
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from __graft_entry__ import load_package  # noqa: E402

pkg = load_package()
hip = C.CDLL("libamdhip64.so")
L = pkg.lib()


def probe(tag):
    s = C.c_void_p()
    hip.hipStreamCreateWithFlags(C.byref(s), 1)
    e = C.c_void_p()
    hip.hipEventCreate(C.byref(e))
    r0 = hip.hipStreamBeginCapture(s, 1)
    r1 = hip.hipEventRecordWithFlags(e, s, 1)
    g = C.c_void_p()
    r2 = hip.hipStreamEndCapture(s, C.byref(g))
    print(tag, "begin", r0, "record_external", r1, "end", r2, flush=True)


probe("torch+engine loaded")
torch.zeros(1, device="cuda")
probe("after torch cuda init")
L.ngp_profiler_enable(1)
probe("after profiler enable (8192 events)")
L.ngp_profiler_enable(0)
