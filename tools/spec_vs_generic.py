"""Lone-frame kernel time of one scene through the generic kernels (RT_OPT_SPECIALIZE 0) and through its
scene-specialised program (1, after rt_ctx_spec_wait), interleaved in one process; each context calibrates
on its first launch, then REPS ordered launches per round, median over ROUNDS (diagnostic: the resource
guard's bounds).  Prints the kernel info (resources) of both and checks both frames are
byte-identical.
usage: python tools/spec_vs_generic.py (SCENE | PATH.scene | fuzz:SEED) WxH TIME DEPTH [REPS] [ROUNDS]"""
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402
import tinyraytracerinrust_amd as T  # noqa: E402

S = os.path.join(ROOT, "tests", "golden", "scenes")


def main():
    scene, size, t, depth = sys.argv[1], sys.argv[2], float(sys.argv[3]), int(sys.argv[4])
    reps = int(sys.argv[5]) if len(sys.argv) > 5 else 10
    rounds = int(sys.argv[6]) if len(sys.argv) > 6 else 5
    W, H = (int(v) for v in size.split("x"))
    if scene.startswith("fuzz:"):
        from tests.scene_fuzz import random_scene
        text = random_scene(int(scene[5:]))
    elif os.path.exists(scene):                                # a scene file's path
        text = open(scene).read()
    else:
        text = open(os.path.join(S, scene + ".scene")).read()
    rs = {}
    for level in (0, 1):
        r = T.Renderer(0, specialize=0)
        r.upload(T.Scene.compile(text, t, W, H, asset_dir=S))
        r.set_kernel("mega")
        if level:
            r.set_specialize(1, wait=True)
        out = r.render_rows(0, H, max_depth=depth)            # calibration
        torch.cuda.synchronize()
        rs[level] = (r, out, [])
    for _ in range(rounds):
        for level, (r, out, ms) in rs.items():
            v = []
            for _ in range(reps):
                r.render_rows(0, H, max_depth=depth, out=out)
                v.append(r.last_kernel_ms())
            ms.append(statistics.median(v))
    for level, (r, out, ms) in rs.items():
        print(f"{scene} {W}x{H} t={t} d={depth} {'specialised' if level else 'generic'}: median {statistics.median(ms):.4f} ms "
              f"(rounds {' '.join(f'{m:.4f}' for m in ms)}) -- {r.kernel_info()}", flush=True)
    same = bool(torch.equal(rs[0][1], rs[1][1]))
    print(f"frames identical: {same}", flush=True)
    return 0 if same else 1


if __name__ == "__main__":
    sys.exit(main())
