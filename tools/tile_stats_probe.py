"""Diagnostic: per-tile phase times of the deferred-shadow kernel from a RT_TILE_STATS build
(make diag NAME=stats DIAG=-DRT_TILE_STATS): the calibration launch of a geometry records, per
8x8 tile, the chain-phase and shadow-phase wall times (10 ns ticks), the longest chain in the
wave, the shadow rounds and the wave's total hits.  Prints the distribution and the slowest tiles.
usage: python tools/tile_stats_probe.py LIB [--size WxH] [--depth D] [--world N]"""
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
    ap.add_argument("--size", default="3840x2160")
    ap.add_argument("--depth", type=int, default=10)
    ap.add_argument("--world", type=int, default=1)
    ap.add_argument("--scene", default="globes")
    a = ap.parse_args()
    import torch
    W, H = (int(v) for v in a.size.split("x"))
    L = ctypes.CDLL(os.path.abspath(a.lib))
    text = open(os.path.join(S, a.scene + ".scene")).read().encode()
    sc, cx = ctypes.c_void_p(), ctypes.c_void_p()
    assert L.rt_scene_compile(text, S.encode(), ctypes.c_double(0.0), W, H, ctypes.byref(sc)) == 0
    assert L.rt_ctx_create(0, ctypes.byref(cx)) == 0
    assert L.rt_ctx_upload(cx, sc) == 0
    band, n = 8, a.world
    n_bands = len(range(0, -(-H // band), n)) if n > 1 else 1
    rows = n_bands * band if n > 1 else H
    out = torch.empty((rows, W, 4), dtype=torch.uint8, device="cuda")
    st = torch.cuda.current_stream().cuda_stream
    if n > 1:
        rc = L.rt_render_row_bands(cx, 0, band, band * n, n_bands, a.depth, ctypes.c_void_p(out.data_ptr()),
                                   ctypes.c_size_t(W * 4), ctypes.c_void_p(st))
    else:
        rc = L.rt_render_rows(cx, 0, H, a.depth, ctypes.c_void_p(out.data_ptr()), ctypes.c_size_t(W * 4),
                              ctypes.c_void_p(st))
    assert rc == 0
    torch.cuda.synchronize()
    v = ctypes.c_float()
    L.rt_ctx_last_kernel_ms(cx, ctypes.byref(v))
    tiles = ((W + 7) // 8) * ((rows + 7) // 8)
    buf = np.zeros((tiles, 4), np.uint32)
    assert L.rt_diag_tile_stats(ctypes.c_void_p(buf.ctypes.data), ctypes.c_size_t(tiles)) == 0
    p1, p2 = buf[:, 0] / 100.0, buf[:, 1] / 100.0              # 10 ns ticks -> us
    mx, rounds, hits = buf[:, 2] & 255, buf[:, 2] >> 8, buf[:, 3]
    tot = p1 + p2
    print(f"{a.scene} {W}x{H} d={a.depth} world={n}: {tiles} tiles, calibration launch {v.value:.4f} ms")
    for name, arr in (("chain phase us", p1), ("shadow phase us", p2), ("total us", tot)):
        q = np.percentile(arr, [50, 90, 99, 99.9, 100])
        print(f"  {name:16s} p50 {q[0]:8.1f}  p90 {q[1]:8.1f}  p99 {q[2]:8.1f}  p99.9 {q[3]:8.1f}  max {q[4]:8.1f}")
    print(f"  longest chain per wave: p50 {np.median(mx):.0f}, max {mx.max()}; hits per wave p50 {np.median(hits):.0f}")
    order = np.argsort(-tot)[:25]
    tx = (W + 7) // 8
    print("  slowest tiles: tile (tx,ty) total chain shadow maxchain rounds hits")
    for t in order:
        print(f"    {t:7d} ({t % tx:4d},{t // tx:4d}) {tot[t]:8.1f} {p1[t]:8.1f} {p2[t]:8.1f} {mx[t]:3d} {rounds[t]:3d} {hits[t]:5d}")
    # chain-length vs time: mean total per max-chain bucket
    for c in sorted(set(mx.tolist())):
        sel = mx == c
        print(f"  maxchain {c:2d}: {sel.sum():7d} tiles, mean chain {p1[sel].mean():7.1f} us, shadow {p2[sel].mean():7.1f} us")


if __name__ == "__main__":
    sys.exit(main())
