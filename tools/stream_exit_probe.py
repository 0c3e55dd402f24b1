"""Diagnostic: which HwStream teardown sequence exits cleanly (round-4 abort at interpreter exit)."""
import sys
import torch
sys.path.insert(0, ".")
import tinyraytracerinrust_amd as T

mode = sys.argv[1]
dev = torch.device("cuda", 0)
x = torch.zeros(16, device=dev)
s = T.HwStream(0)
if mode in ("use", "use_close", "use_close_del"):
    with torch.cuda.stream(s.torch):
        x += 1
    ev = torch.cuda.Event()
    ev.record(s.torch)
    torch.cuda.synchronize()
if mode in ("close", "use_close", "use_close_del"):
    s.close()
if mode == "use_close_del":
    del s
print("end", mode, flush=True)
