"""Headless driver: compile -> upload -> render -> (gather) -> PNG.

    python -m tinyraytracerinrust_amd render SCENE [--size WxH] [--time T | --frame F]
                                          [--depth D] [--gpus N] [-o out.png]

Replaces the reference's entry point and its GUI load path for this purpose: ``main()`` only
starts the GTK application (src/main.rs:7-9), which builds a RayTracer per frame with
``time = frame / 300`` (src/raydebugger/debug_window.rs:53-62, gui.rs:20) and renders it row by
row into a cairo surface (debug_window.rs:74-87, 147-164).  Here the frame is rendered by the HIP
kernels and written as a PNG of exactly the bytes the GUI would show, ``(c * 255.0) as u8``
(easy_pixbuf.rs:46-53).  SCENE is a .scene path; texture names resolve against its directory
(``--assets`` overrides), like the reference's CWD-relative ``texture("worldmap.png")``.

``--gpus N`` (N > 1) renders the frame row-tiled over N GPUs, one process per GPU, assembled by one
RCCL all-gather (tinyraytracerinrust_amd/distributed.py); started without torch.distributed.run it
launches its own N ranks.  Phase times go to stderr as one JSON line.  There is no CPU path: without
a HIP device the command fails.
"""
from __future__ import annotations

import argparse
import json
import os
import socket
import subprocess
import sys
import time


def _parse(argv):
    ap = argparse.ArgumentParser(prog="python -m tinyraytracerinrust_amd", description=__doc__.split("\n")[0])
    sub = ap.add_subparsers(dest="cmd", required=True)
    r = sub.add_parser("render", help="render one frame of a .scene file to a PNG")
    r.add_argument("scene", help="path of a .scene file")
    r.add_argument("--size", default="480x360", help="WxH (the GUI default is 480x360, gui.rs:17-18)")
    g = r.add_mutually_exclusive_group()
    g.add_argument("--time", type=float, default=None, help="the scene's global `time` (default 0)")
    g.add_argument("--frame", type=int, default=None, help="GUI frame number: time = frame / 300")
    r.add_argument("--depth", type=int, default=-1, help="max_depth (default: the scene's, 10)")
    r.add_argument("--gpus", type=int, default=1)
    r.add_argument("--layout", default="cyclic", choices=["cyclic", "contiguous"])
    r.add_argument("--band", type=int, default=8)
    r.add_argument("--assets", default=None, help="directory textures resolve against (default: the scene's)")
    r.add_argument("--channels", type=int, default=3, choices=[3, 4], help="PNG channels (RGB or RGBA)")
    r.add_argument("-o", "--output", default="out.png")
    a = ap.parse_args(argv)
    try:
        w, h = a.size.lower().split("x")
        a.width, a.height = int(w), int(h)
    except ValueError:
        ap.error(f"--size must be WxH, not {a.size!r}")
    if a.width <= 0 or a.height <= 0:
        ap.error("--size must be positive")
    if a.gpus < 1:
        ap.error("--gpus must be >= 1")
    if a.band < 1:
        ap.error("--band must be >= 1")
    a.t = a.frame / 300.0 if a.frame is not None else (a.time or 0.0)
    return a


def _self_launch(argv, gpus: int) -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={gpus}",
           "--master-addr", "127.0.0.1", "--master-port", str(port), "-m", "tinyraytracerinrust_amd"] + list(argv)
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    return subprocess.call(cmd, env=env)


def render(a) -> dict:
    import numpy as np
    import torch
    import torch.distributed as dist
    from . import distributed as D
    from .raytracer import Scene, Renderer, write_png

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != a.gpus:
        raise SystemExit(f"--gpus {a.gpus} but WORLD_SIZE={world}")
    if not torch.cuda.is_available():
        raise SystemExit("no HIP device: the render path has no CPU fallback")
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        dist.init_process_group("nccl", device_id=dev)
    times = {}
    t0 = time.perf_counter()
    with open(a.scene) as f:
        text = f.read()
    assets = a.assets or os.path.dirname(os.path.abspath(a.scene))
    scene = Scene.compile(text, a.t, a.width, a.height, asset_dir=assets, strict=False)
    if scene.status:
        print(f"scene parse error (rendering the default scene, as the reference does): {scene.error}",
              file=sys.stderr)
    times["compile_ms"] = (time.perf_counter() - t0) * 1e3
    t0 = time.perf_counter()
    r = Renderer(local)
    r.upload(scene)
    torch.cuda.synchronize(dev)
    times["upload_ms"] = (time.perf_counter() - t0) * 1e3
    W, H = a.width, a.height
    t0 = time.perf_counter()
    if world == 1:
        frame = r.render_rows(0, H, max_depth=a.depth)
        torch.cuda.synchronize(dev)
        times["render_ms"] = (time.perf_counter() - t0) * 1e3
    else:
        band = a.band if a.layout == "cyclic" else -(-H // world)
        slot = torch.zeros((D.rows_per_rank(H, world, a.layout, band), W, 3), dtype=torch.uint8, device=dev)   # packed RGB8
        y_first, band_rows, pitch, n_bands = D.band_params(H, world, rank, a.layout, band)
        if n_bands:
            r.render_row_bands(y_first, band_rows, pitch, n_bands, slot, max_depth=a.depth)
        torch.cuda.synchronize(dev)
        times["render_ms"] = (time.perf_counter() - t0) * 1e3
        t0 = time.perf_counter()
        gath = torch.empty((world * slot.shape[0], W, 3), dtype=torch.uint8, device=dev)
        dist.all_gather_into_tensor(gath, slot)
        frame = D.assemble(gath, H, world, a.layout, band)
        torch.cuda.synchronize(dev)
        times["gather_assemble_ms"] = (time.perf_counter() - t0) * 1e3
    if rank == 0:
        t0 = time.perf_counter()
        host = frame.cpu().numpy()
        times["d2h_ms"] = (time.perf_counter() - t0) * 1e3
        t0 = time.perf_counter()
        write_png(a.output, np.ascontiguousarray(host), channels=a.channels)
        times["png_ms"] = (time.perf_counter() - t0) * 1e3
    if world > 1:
        dist.destroy_process_group()
    return {"output": a.output, "width": W, "height": H, "time": a.t, "gpus": world,
            **{k: round(v, 3) for k, v in times.items()}}


def main(argv=None) -> int:
    argv = sys.argv[1:] if argv is None else argv
    a = _parse(argv)
    if a.gpus > 1 and "WORLD_SIZE" not in os.environ:
        return _self_launch(argv, a.gpus)      # before this process touches the GPU
    info = render(a)
    if int(os.environ.get("RANK", "0")) == 0:
        print(json.dumps(info), file=sys.stderr)
    return 0


if __name__ == "__main__":
    sys.exit(main())
