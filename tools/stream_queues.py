"""Which hardware queue does each stream land on?  One tiny kernel per
stream (torch pool streams, raw HIP streams, high-priority pool streams);
run under rocprofv3 --kernel-trace and read Queue_Id / Stream_Id."""
import ctypes
import sys

import torch

dev = torch.device("cuda", 0)
hip = ctypes.CDLL("libamdhip64.so")
x = torch.ones(1 << 16, device=dev)
out = []
for i in range(4):
    s = torch.cuda.Stream(device=dev)
    out.append(("pool", s))
for i in range(4):
    h = ctypes.c_void_p()
    assert hip.hipStreamCreateWithFlags(ctypes.byref(h), ctypes.c_uint(1)) == 0
    out.append(("raw", torch.cuda.ExternalStream(h.value, device=dev)))
for i in range(2):
    out.append(("prio", torch.cuda.Stream(device=dev, priority=-1)))
for k, (kind, s) in enumerate(out):
    with torch.cuda.stream(s):
        for _ in range(k + 1):   # k + 1 launches: the stream's index in the trace
            x.add_(1)
torch.cuda.synchronize()
for k, (kind, s) in enumerate(out):
    print(k, kind, hex(s.cuda_stream), k + 1, "launches", flush=True)
sys.exit(0)
