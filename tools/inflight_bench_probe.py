"""Diagnostic (round 5): why bench.py's `inflight4` phase (4 frames in flight on
own-queue streams, N = 1) ran 14.5 % slower per frame than its lone frames.  Renders the headline
workload (4K globes.scene d10, specialised kernels, timing events off, like bench.py) under several
stream / kernel arrangements, interleaved over `--rounds` rounds after a 300 ms settle, and prints the
wall time per frame of each.

arrangements:
  k1_cur    one frame at a time on torch's current stream, the library's kernel choice (bench `value`)
  k1_hw     one frame at a time on one own-queue stream (rt_stream_create)
  kK_hw     K frames in flight on K own-queue streams, context with RT_KERNEL_MEGA (bench `inflight4`)
  kK_hwauto K own-queue streams, the auto context (no kernel switch, no re-calibration)
  kK_pool   K torch pool streams (shared hardware queues)
  kK_hwser  K own-queue streams, but each frame waits for the previous one (events): queue switching
            without any overlap
usage: python tools/inflight_bench_probe.py [--frames 60] [--rounds 3] [--ks 2,4]"""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
S = os.path.join(ROOT, "tests", "golden", "scenes")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=60)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--ks", default="2,4")
    ap.add_argument("--config", default="globes4k", choices=["globes4k", "globes1080d5", "sphere1080d0"])
    ap.add_argument("--specialize", type=int, default=1)
    a = ap.parse_args()
    import torch
    import tinyraytracerinrust_amd as T
    scene, W, H, depth = {"globes4k": ("globes", 3840, 2160, 10), "globes1080d5": ("globes", 1920, 1080, 5),
                          "sphere1080d0": (None, 1920, 1080, 0)}[a.config]
    text = open(os.path.join(S, scene + ".scene")).read() if scene else "draw(sphere(<0, 0, 0>, 30, red))"
    sc = T.Scene.compile(text, 0.0, W, H, asset_dir=S)
    dev = torch.device("cuda", 0)

    def renderer(kernel):
        r = T.Renderer(0)
        r.upload(sc)
        r.set_timing(False)
        if a.specialize:
            r.set_specialize(1)
        r.set_kernel(kernel)
        return r
    r_auto, r_mega = renderer("auto"), renderer("mega")
    ks = [int(k) for k in a.ks.split(",")]
    K = max(ks)
    bufs = [torch.zeros((H, W, 4), dtype=torch.uint8, device=dev) for _ in range(K)]
    hw = [T.HwStream(0) for _ in range(K)]
    hws = [h.torch for h in hw]
    pool = [torch.cuda.Stream(dev) for _ in range(K)]
    cur = torch.cuda.current_stream(dev)
    whole = r_auto.render_rows(0, H, max_depth=depth)          # calibrates r_auto's order
    r_mega.render_rows(0, H, max_depth=depth, out=bufs[0])     # calibrates r_mega's order
    torch.cuda.synchronize()

    def run(name, r, streams, k, serial=False, n=None):
        n = n or a.frames
        ev = [torch.cuda.Event() for _ in range(k)] if serial else None
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for i in range(n):
            s = streams[i % k]
            if serial and i:
                s.wait_event(ev[(i - 1) % k])
            r.render_rows(0, H, max_depth=depth, out=bufs[i % k], stream=s)
            if serial:
                ev[i % k].record(s)
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) * 1e3 / n

    arr = [("k1_cur", r_auto, [cur], 1, False), ("k1_hw", r_auto, hws[:1], 1, False)]
    for k in ks:
        arr += [(f"k{k}_hw", r_mega, hws[:k], k, False), (f"k{k}_hwauto", r_auto, hws[:k], k, False),
                (f"k{k}_pool", r_mega, pool[:k], k, False), (f"k{k}_hwser", r_mega, hws[:k], k, True)]
    ts = time.perf_counter()                                   # settle, as bench.py
    while (time.perf_counter() - ts) < 0.3:
        run("settle", r_auto, [cur], 1, n=8)
    res = {name: [] for name, *_ in arr}
    for rd in range(a.rounds):
        for name, r, streams, k, serial in arr:
            run(name, r, streams, k, serial, n=2 * k + 2)      # warm this arrangement's streams
            res[name].append(run(name, r, streams, k, serial))
        print(f"round {rd}: " + "  ".join(f"{n} {v[-1]:.4f}" for n, v in res.items()), flush=True)
    for b in bufs[:K]:
        if not torch.equal(b, whole):
            raise SystemExit("a frame buffer differs from the single-launch render")
    print(f"{a.config} spec={a.specialize}: ms per frame, median of {a.rounds} rounds of {a.frames} frames "
          f"({r_auto.kernel_info()})")
    for name, v in res.items():
        v = sorted(v)
        print(f"  {name:10s} {v[len(v) // 2]:.4f}   (all: {' '.join(f'{x:.4f}' for x in res[name])})")
    for h in hw:
        h.close()


if __name__ == "__main__":
    main()
