import sys, ctypes
sys.path.insert(0, '.')
import torch
from sy_amd._lib import lib
n = ctypes.c_int()
print("count rc", lib.sydelta_device_count(ctypes.byref(n)), n.value, lib.sydelta_last_error())
from sy_amd import wire
src = bytes(range(256)) * 10
d = torch.frombuffer(bytearray(src), dtype=torch.uint8).cuda()
try:
    out = wire.delta_to_json_device([1], [0], [len(src)], len(src), 4096, d)
    print("ok", len(out))
except Exception as e:
    print("ERR", e)
