"""Diagnostic: when does each workgroup of a tail-bound ordered deferred launch start and end?  A
-DRT_DIAG_ENTRY_TIMES build records wall-clock ticks (10 ns) per dispatched entry; this renders rank
0's share of the 4K globes frame at N ranks (cyclic 8-row bands) -- calibration, then ordered
launches -- and prints the launch span, the dispatch-time profile and the entries that end last.
usage: python tools/entry_times_probe.py LIB [--world N] [--depth D]"""
import argparse
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
S = os.path.join(ROOT, "tests", "golden", "scenes")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("lib")
    ap.add_argument("--world", type=int, default=8)
    ap.add_argument("--depth", type=int, default=10)
    ap.add_argument("--size", default="3840x2160")
    a = ap.parse_args()
    import torch
    W, H = (int(v) for v in a.size.split("x"))
    L = ctypes.CDLL(os.path.abspath(a.lib))
    text = open(os.path.join(S, "globes.scene")).read().encode()
    sc, cx = ctypes.c_void_p(), ctypes.c_void_p()
    assert L.rt_scene_compile(text, S.encode(), ctypes.c_double(0.0), W, H, ctypes.byref(sc)) == 0
    assert L.rt_ctx_create(0, ctypes.byref(cx)) == 0
    assert L.rt_ctx_upload(cx, sc) == 0
    band, n = 8, a.world
    n_bands = len(range(0, -(-H // band), n))
    rows = n_bands * band
    out = torch.empty((rows, W, 4), dtype=torch.uint8, device="cuda")
    st = torch.cuda.current_stream().cuda_stream
    for _ in range(4):
        assert L.rt_render_row_bands(cx, 0, band, band * n, n_bands, a.depth, ctypes.c_void_p(out.data_ptr()),
                                     ctypes.c_size_t(W * 4), ctypes.c_void_p(st)) == 0
        torch.cuda.synchronize()
    v = ctypes.c_float()
    L.rt_ctx_last_kernel_ms(cx, ctypes.byref(v))
    tiles = ((W + 7) // 8) * ((rows + 7) // 8)
    cap = tiles * 4
    t = np.zeros((cap, 2), np.uint64)
    order = np.zeros(cap, np.int32)
    rc = L.rt_diag_entry_times(cx, ctypes.c_void_p(t.ctypes.data), ctypes.c_void_p(order.ctypes.data),
                               ctypes.c_size_t(cap))
    used = t[:, 1] > 0
    n_ent = int(np.nonzero(used)[0].max()) + 1 if used.any() else 0
    t, order = t[:n_ent].astype(np.int64), order[:n_ent]
    t0 = t[:, 0].min()
    st_us, en_us = (t[:, 0] - t0) / 100.0, (t[:, 1] - t0) / 100.0
    dur = en_us - st_us
    print(f"N={n} share: {tiles} tiles, {n_ent} entries (rc {rc}), last launch {v.value:.4f} ms (events), "
          f"span by ticks {en_us.max():.1f} us")
    for q in (0.1, 0.5, 0.9, 0.99, 1.0):
        k = min(n_ent - 1, int(q * n_ent))
        print(f"  entry #{k:6d} ({q:4.0%} of the order): starts {st_us[k]:7.1f} us")
    print(f"  durations: p50 {np.median(dur):.1f}  p99 {np.percentile(dur, 99):.1f}  max {dur.max():.1f} us")
    print("  entries ending last: idx start dur end  tile part/P")
    for i in np.argsort(-en_us)[:20]:
        e = int(order[i]) if rc == 0 else -1
        print(f"    {i:6d} {st_us[i]:7.1f} {dur[i]:7.1f} {en_us[i]:7.1f}  {e & 0xFFFFF:6d} {(e >> 20) & 15}/{1 << ((e >> 24) & 7)}")
    busy = np.zeros(int(en_us.max()) + 2)
    for s0, e0 in zip(st_us.astype(int), en_us.astype(int)):
        busy[s0:e0 + 1] += 1
    for us in range(0, len(busy), max(1, len(busy) // 15)):
        print(f"  t={us:5d} us: {int(busy[us]):6d} waves resident")


if __name__ == "__main__":
    sys.exit(main())
