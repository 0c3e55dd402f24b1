"""Offline: algorithmic work of a workload, counted by the CPU oracle's counting build.

Writes tests/golden/flops_<scene>_<W>x<H>_t<time>_d<depth>.json with per-row flop counts (the
reference algorithm's f64 add/sub/mul/div/sqrt + libm calls, oracle/rt_oracle.c FL()/TR()) and
frame totals of every event counter.  bench.py sums the rows a launch renders to get the
algorithmic flops per launch for its roofline (DESIGN.md "Roofline").  Test infrastructure only.
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from oracle import oracle as O  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scene", default="globes")
    ap.add_argument("--width", type=int, default=3840)
    ap.add_argument("--height", type=int, default=2160)
    ap.add_argument("--time", type=float, default=0.0)
    ap.add_argument("--depth", type=int, default=10)
    ap.add_argument("--threads", type=int, default=8)
    ap.add_argument("--text", default="",
                    help="scene text instead of tests/golden/scenes/<scene>.scene (e.g. BASELINE config 2's one-line "
                         "sphere scene, written as flops_sphere_*.json with --scene sphere)")
    ap.add_argument("--frames", type=int, default=0,
                    help="animation mode: per-frame totals of frames f = 0..F-1 at time f/F (BASELINE config 5)")
    a = ap.parse_args()
    scenes = os.path.join(ROOT, "tests", "golden", "scenes")
    O.register_texture_file("worldmap.png", os.path.join(scenes, "worldmap.png"))
    text = a.text or open(os.path.join(scenes, a.scene + ".scene")).read()
    if a.frames:
        return animation(a, text)
    sc = O.OracleScene(text, a.time, a.width, a.height, max_depth=a.depth, counting=True)
    rows, totals = [], {}
    for y in range(a.height):
        _, _, c = sc.render(y, y + 1, threads=a.threads, u8=False)
        rows.append(c["flop"])
        for k, v in c.items():
            totals[k] = totals.get(k, 0) + v
    out = {
        "scene": a.text or a.scene + ".scene", "width": a.width, "height": a.height, "time": a.time,
        "max_depth": a.depth, "flop_definition": "f64 add/sub/mul/div/sqrt and libm acos/sin calls as the "
        "reference evaluates them (oracle/rt_oracle.c FL/TR); negation, comparisons, clamps not counted",
        "totals": totals, "row_flops": rows,
    }
    path = os.path.join(ROOT, "tests", "golden", f"flops_{a.scene}_{a.width}x{a.height}_t{a.time:g}_d{a.depth}.json")
    with open(path, "w") as f:
        json.dump(out, f)
    print(path, totals["flop"], "flops,", totals["flop"] / (a.width * a.height), "per pixel")


def animation(a, text):
    """Per-frame totals of an F-frame animation (time = f / F), whole frames."""
    frames, totals = [], {}
    for f in range(a.frames):
        sc = O.OracleScene(text, f / a.frames, a.width, a.height, max_depth=a.depth, counting=True)
        _, _, c = sc.render(0, a.height, threads=a.threads, u8=False)
        frames.append(c["flop"])
        for k, v in c.items():
            totals[k] = totals.get(k, 0) + v
        print(f"frame {f}: {c['flop']} flops", flush=True)
    out = {
        "scene": a.scene + ".scene", "width": a.width, "height": a.height, "frames": a.frames,
        "time": "f / frames", "max_depth": a.depth, "flop_definition": "as flops_globes_*.json",
        "totals": totals, "frame_flops": frames,
    }
    path = os.path.join(ROOT, "tests", "golden", f"flops_{a.scene}_{a.width}x{a.height}_anim{a.frames}_d{a.depth}.json")
    with open(path, "w") as f:
        json.dump(out, f)
    print(path, totals["flop"], "flops")


if __name__ == "__main__":
    main()
