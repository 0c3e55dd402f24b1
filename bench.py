#!/usr/bin/env python
"""bench.py -- Mrays/s of the MI355X render path on the BASELINE workload.

Workload (BASELINE.json metric "Mrays/sec at 3840x2160 globes.scene"; configs[3]):
globes.scene at t=0, 3840x2160, max_depth 10 (the reference's hard-coded depth,
raytracer.rs:65), default test light, RGBA8 output.  One step = one frame:

* N = 1: one kernel launch renders all 2160 rows into an HBM framebuffer;
* N > 1: one process per GPU (torchrun); rank r renders its rows -- 8-row bands dealt
  round-robin (``--layout cyclic``, default: balances cheap sky rows against floor rows with
  reflection chains; ``contiguous`` = one tile per rank) -- and one RCCL all_gather_into_tensor
  over xGMI assembles the frame on every rank, followed by one local permute copy for the cyclic
  layout.  Frame k's gather overlaps frame k+1's render (double-buffered; ``--no-overlap``
  serialises).  Total work is fixed as N grows: scaling "strong".

value = W*H primary rays per frame * K frames / (max over ranks of the timed wall time), in
millions.  The scene blob and texture are uploaded before the timed region (inputs resident in
HBM).  rank 0 prints ONE JSON line with two extra objects:

* roofline -- the render kernel against the FP64 vector roofline (this path has no dense
  contraction and ~0.1 B/flop, see DESIGN.md "Roofline"): algorithmic flops per launch (the
  reference algorithm's f64 ops for the rows the launch renders, counted by the oracle's counting
  build: tests/golden/flops_*.json) / the kernel's mean duration measured here with HIP events on
  the launch stream; traffic = HBM bytes per launch from the committed rocprofv3 PMC summary
  (profiles/) when it exists for this workload, else null.  ``roofline_hbm`` restates the same
  launch against HBM bandwidth, as the north star asks.
* cpu_baseline -- the CPU oracle (a faithful C restatement of the reference loop; the Rust
  reference cannot be built here) timed on this host on rank 0 at N=1 only, on every core this
  process may run on (sched_getaffinity, capped by the cgroup CPU quota), as the reference's
  threadpool is sized to num_cpus (src/raydebugger/gui.rs:49-51), plus a 1-thread sample.

Launching: ``python bench.py --gpus N`` with N > 1 outside torch.distributed.run starts N rank
processes itself (a torch.distributed.run child, before this process touches the GPU) and exits
with its status; rank 0's JSON line is the child's stdout.  ``--launcher-check`` runs the same
N-rank machinery on CPU under gloo with a synthetic per-pixel pattern instead of rendering (no
GPU, no measurement): band layout, all-gather and assembly are checked (tests/test_bench_launcher.py).
"""
from __future__ import annotations

import argparse
import json
import math
import os
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)
SCENES = os.path.join(ROOT, "tests", "golden", "scenes")

FP64_VECTOR_PEAK_TFLOPS = 78.6     # MI355X spec, FMA counted as 2 flops
FP64_NO_FMA_TFLOPS = 39.3          # one add or mul per lane per cycle: the parity-bound ceiling
HBM_PEAK_GBS = 8000.0              # MI355X_MICROARCH.md chip table (spec)

CONFIGS = {
    # name: (scene, width, height, time, max_depth)
    "globes4k": ("globes", 3840, 2160, 0.0, 10),
    "globes1080d5": ("globes", 1920, 1080, 0.0, 5),
    "sphere1080d0": (None, 1920, 1080, 0.0, 0),
}
# Default timed steps per config: a timed region of >= ~14 ms, as the headline's 50 x 0.27 ms.  The
# sphere's 50 frames took 0.77 ms, in which the region's fixed cost (the synchronisations that bracket
# it, ~35 us) was 5 % of the time (profiles/r09r_*: 50 steps 0.0154 ms/step, 1000 steps 0.0147).
DEFAULT_STEPS = {"globes4k": 50, "globes1080d5": 200, "sphere1080d0": 1000, "anim120": 50}
SPHERE_SCENE = "draw(sphere(<0, 0, 0>, 30, red))"      # BASELINE config 2
# BASELINE config 5: the 120-frame spinning_globes animation at 1920x1080, time = f / 120,
# frames dealt round-robin over the ranks (replicas, no collective).
ANIM = {"anim120": ("spinning_globes", 1920, 1080, 120, 10)}


def parse():
    ap = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=None,
                    help="timed steps (default: the config's DEFAULT_STEPS, a timed region of >= ~14 ms)")
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--config", default="globes4k", choices=sorted(CONFIGS) + sorted(ANIM),
                    help="globes4k = the headline workload; anim120 = BASELINE config 5 (one step = the "
                         "whole 120-frame animation)")
    ap.add_argument("--layout", default="cyclic", choices=["contiguous", "cyclic"],
                    help="row tiling for N > 1 (cyclic 8-row bands balance sky vs floor rows)")
    ap.add_argument("--band", type=int, default=8)
    ap.add_argument("--gather", default="rgb", choices=["rgb", "rgba"],
                    help="N > 1: ranks render their bands as packed RGB8 and the all-gather moves 3 bytes per "
                         "pixel (the assembly writes the RGBA8 frame, A = 255); rgba gathers RGBA8 rows")
    ap.add_argument("--no-overlap", action="store_true",
                    help="N > 1: do not overlap frame k's all-gather with frame k+1's render")
    ap.add_argument("--force-collective", action="store_true",
                    help="exercise the N > 1 path (process group, bands, all-gather) even at N = 1")
    ap.add_argument("--rehearse-one-gpu", action="store_true",
                    help="diagnostic, not a measurement: run the N ranks' whole frame pipeline (HIP band renders, "
                         "frames in flight, gathers, assembly kernel, per-rank frame checks) on ONE GPU -- every "
                         "rank on device 0, the all-gather over gloo staged through host memory (RCCL refuses two "
                         "ranks on one device).  The line carries no value")
    ap.add_argument("--cpu-threads", type=int, default=0,
                    help="CPU-baseline threads (0 = every core available to this process)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-extra", action="store_true",
                    help="skip the extra phase after the timed region (N = 1: 4 frames in flight; N > 1: one "
                         "frame at a time), which reports the other half of the scaling picture")
    ap.add_argument("--inflight", type=int, default=0,
                    help="frames whose renders may overlap, each on a stream with its own hardware queue "
                         "(0 = 1 at N = 1, so the roofline's kernel time and the rocprof trace are of one launch "
                         "alone; 4 at N > 1).  A frame's tail is its costliest tiles, so a lone frame leaves the "
                         "GPU partly idle at its end; overlapping frames fill it (N = 1, --inflight 4: 4K globes "
                         "+2.5 %%, 1080p d5 +37 %%, the sphere +52 %%, profiles/r02bg_inflight_n1.txt)")
    ap.add_argument("--specialize", type=int, default=1, choices=[0, 1],
                    help="compile the scene's own row kernels before the timed region (hipRTC, rt_ctx_set_option "
                         "RT_OPT_SPECIALIZE; the compile time is reported as spec_compile_ms); 0 = the generic kernels. "
                         "anim120: the frames' scenes registered as scene families (rt_spec_family_register: one "
                         "program per family of frames of the same structure, compiled before the timed region)")
    ap.add_argument("--chunks", type=int, default=4,
                    help="N > 1, the single-frame phase: the frame as this many sub-frames, each gathered and assembled "
                         "as soon as its bands are rendered, cheapest first (1 = render, then one gather, then assembly)")
    ap.add_argument("--rccl-priority", default="normal", choices=["high", "normal"],
                    help="priority of RCCL's stream (the all-gathers) relative to the render streams")
    ap.add_argument("--pool-streams", action="store_true",
                    help="diagnostic: frames in flight on torch pool streams instead of own-queue streams")
    ap.add_argument("--streams", type=int, default=2,
                    help="anim120: frames dealt round-robin over this many HIP streams so independent "
                         "frames' kernels overlap (one 1080p frame does not fill the GPU to its end); "
                         "specialised (scene families) 1 / 2 / 4 / 8 streams: 14152 / 14781 / 14452 / 13828 Mrays/s "
                         "(profiles/r05x_tuning.txt); generic 1 / 2 / 3 / 4: 8226 / 8786 / 8901 / 8913 "
                         "(profiles/r02cu_anim120_streams.txt)")
    ap.add_argument("--kernel", default="auto", choices=["auto", "mega", "deferred"],
                    help="anim120: the renderers' RT_OPT_KERNEL (auto: the library's choice per launch)")
    ap.add_argument("--settle-ms", type=float, default=300.0,
                    help="before the warmup steps, render untimed frames for this long so the GPU reaches its "
                         "sustained clocks (reported as `settle` in the line; 0 disables).  Measured: 20 steps after "
                         "5 warmup steps alone run 0.675 ms/frame, 100 steps 0.603 (profiles/r02l_same_box.txt)")
    ap.add_argument("--png", default="", help="write the rendered frame (rank 0) to this PNG")
    ap.add_argument("--launcher-check", action="store_true",
                    help="CPU/gloo check of the N-rank launcher, band layout, all-gather and assembly with a "
                         "synthetic pixel pattern (no GPU, no rendering, no measurement)")
    a = ap.parse_args()
    if a.steps is None:
        a.steps = DEFAULT_STEPS.get(a.config, 50)
    return a


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def self_launch(a) -> int:
    """N > 1 without a launcher: run N ranks under torch.distributed.run as a CHILD process (this
    process has not touched the GPU) and return its exit status.  Rank 0's stdout -- the one JSON
    line -- is inherited."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={a.gpus}",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    env.setdefault("OMP_NUM_THREADS", "1")
    return subprocess.call(cmd, env=env)


def host_cpus():
    """(cores this process may use, CPU model, affinity count, cgroup quota or None)."""
    aff = len(os.sched_getaffinity(0))
    quota = None
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, per = f.read().split()[:2]
            if q != "max":
                quota = int(q) / int(per)
    except (OSError, ValueError):
        pass
    model = "unknown"
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    cores = aff if quota is None else max(1, min(aff, int(math.ceil(quota))))
    return min(cores, 256), model, aff, quota


def owned_rows(H, world, rank, layout, band):
    from tinyraytracerinrust_amd import distributed as D
    return D.owned_rows(H, world, rank, layout, band)


def load_flops(scene, W, H, t, depth):
    path = os.path.join(ROOT, "tests", "golden", f"flops_{scene}_{W}x{H}_t{t:g}_d{depth}.json")
    if not os.path.exists(path):
        return None
    with open(path) as f:
        return json.load(f)


def load_pmc(config, world, layout):
    """The committed PMC summary entry of this config (profiles/pmc_summary.json, written by
    tools/pmc_summary.py from rocprofv3 --pmc passes of this bench command), or {}."""
    path = os.path.join(ROOT, "profiles", "pmc_summary.json")
    if not os.path.exists(path):
        return {}
    with open(path) as f:
        d = json.load(f)
    key = f"{config}/n{world}/{layout}"
    return d.get(key) or (d.get(f"{config}/n1/contiguous") if world == 1 else None) or {}


def load_traffic(config, world, layout):
    """HBM bytes per launch of the render kernel from the committed PMC summary (or None)."""
    return load_pmc(config, world, layout).get("hbm_bytes_per_launch")


def issue_model(config, world, layout, kernel_ms, n_cu=256, clock_ghz=2.4):
    """Where the render kernel's cycles go, from the committed PMC counters of this config
    (profiles/pmc_summary.json) over THIS run's kernel time.  SIMD issue cycles per wave64 VALU
    instruction: FP64 add/mul/fma 4 (16 lanes per cycle: the 78.6 TFLOP/s FP64 peak), FP64
    transcendental (rcp/rsq/sqrt) 8, every other VALU instruction 2 (32 lanes per cycle, the f32
    rate; MI355X_MICROARCH.md cycle constants).  valu_issue_fill = those cycles / (SIMDs x kernel
    time x clock); wait_any_share = SQ_WAIT_ANY / SQ_WAVE_CYCLES (waves parked on s_waitcnt);
    valu_active_share = SQ_ACTIVE_INST_VALU / SQ_WAVE_CYCLES."""
    c = load_pmc(config, world, layout).get("counters")
    if not c or not kernel_ms or "SQ_INSTS_VALU" not in c:
        return None
    f64 = sum(c.get(k, 0.0) for k in ("SQ_INSTS_VALU_ADD_F64", "SQ_INSTS_VALU_MUL_F64", "SQ_INSTS_VALU_FMA_F64"))
    trans = c.get("SQ_INSTS_VALU_TRANS_F64", 0.0)
    other = c["SQ_INSTS_VALU"] - f64 - trans
    cyc = 4.0 * f64 + 8.0 * trans + 2.0 * other
    avail = n_cu * 4 * kernel_ms * 1e-3 * clock_ghz * 1e9
    out = {"valu_issue_fill": round(cyc / avail, 4), "valu_insts": c["SQ_INSTS_VALU"], "fp64_insts": f64,
           "fp64_trans_insts": trans, "clock_ghz_assumed": clock_ghz,
           "cycle_model": "FP64 add/mul/fma 4, FP64 trans 8, other VALU 2 SIMD cycles per wave64 instruction"}
    if c.get("SQ_WAVE_CYCLES"):
        out["wait_any_share"] = round(c.get("SQ_WAIT_ANY", 0.0) / c["SQ_WAVE_CYCLES"], 4)
        if "SQ_ACTIVE_INST_VALU" in c:
            out["valu_active_share"] = round(c["SQ_ACTIVE_INST_VALU"] / c["SQ_WAVE_CYCLES"], 4)
        if "SQ_WAIT_INST_ANY" in c:
            out["wait_inst_share"] = round(c["SQ_WAIT_INST_ANY"] / c["SQ_WAVE_CYCLES"], 4)
    return out


def lib_sha16():
    """sha256 (16 hex digits) of the loaded librt_mi355x.so: the binary a PMC block must come from."""
    import hashlib
    from tinyraytracerinrust_amd import _lib
    with open(_lib.LIB_PATH, "rb") as f:
        return hashlib.sha256(f.read()).hexdigest()[:16]


def executed_fp64(config, world, layout, kernel_ms, variant=None):
    """The EXECUTED FP64 rate: (ADD + MUL + 2 FMA) wave-instructions x 64 per launch from the PMC
    summary over this run's kernel time -- the hardware's view (`roofline.frac`), next to the reference
    algorithm's flops (`frac_algorithmic`, of which exact culling skips about 70 %).  The block names
    the session and the library binary the counters were measured on, and whether that binary (and
    kernel variant) is the one this run loaded."""
    e = load_pmc(config, world, layout)
    fl = e.get("executed_fp64_flops_per_launch")
    if not fl or not kernel_ms:
        return None
    tf = fl / (kernel_ms * 1e-3) / 1e12
    sha = lib_sha16()
    same = e.get("so_sha16") == sha and (variant is None or e.get("variant", "generic") == variant)
    return {"tflops": round(tf, 3), "frac": round(tf / FP64_VECTOR_PEAK_TFLOPS, 4),
            "flops_per_launch": fl, "pmc_tag": e.get("tag"), "pmc_so_sha16": e.get("so_sha16"),
            "pmc_variant": e.get("variant", "generic"), "this_so_sha16": sha, "pmc_matches_binary": same,
            "valu_insts_per_wave": e.get("valu_insts_per_wave")}


def roofline_block(achieved_alg, ex, traffic, extra):
    """`roofline` of a bench line.  `frac` is a HARDWARE fraction: the FP64 flops the render kernel
    executes (PMC: (ADD + MUL + 2 FMA) x 64 per launch, `executed_fp64`) per second of this run's
    kernel time over the 78.6 TFLOP/s FP64 peak.  The reference algorithm's flop count (the oracle's
    counting build) over the same time is `achieved_algorithmic` / `frac_algorithmic`: it exceeds what
    the GPU executes, because exact culling skips most of the reference's work, so it says how fast
    the reference's computation is delivered, not how busy the hardware is (round-3 VERDICT)."""
    hw = ex["tflops"] if ex else None
    out = {
        "bound": "fp64-valu",
        "achieved": hw,
        "peak": FP64_VECTOR_PEAK_TFLOPS,
        "unit": "TFLOP/s",
        "frac": round(hw / FP64_VECTOR_PEAK_TFLOPS, 4) if hw else None,
        "frac_basis": "executed FP64 flops (PMC, executed_fp64) / this run's kernel time / FP64 peak",
        "traffic": traffic,
        "achieved_algorithmic": round(achieved_alg, 3) if achieved_alg else None,
        "frac_algorithmic": round(achieved_alg / FP64_VECTOR_PEAK_TFLOPS, 4) if achieved_alg else None,
        "frac_of_no_fma_ceiling": round(achieved_alg / FP64_NO_FMA_TFLOPS, 4) if achieved_alg else None,
        "no_fma_ceiling": FP64_NO_FMA_TFLOPS,
        "executed_fp64": ex,
    }
    out.update(extra)
    return out


def cpu_baseline(text, W, H, t, depth, threads, target_s=1.0):
    """Time the CPU oracle: `threads` threads (default: every available core) on whole frames,
    repeated until ~target_s of wall time (at least one frame), and 1 thread on a row sample."""
    from oracle import oracle as O
    cores, model, aff, quota = host_cpus()
    threads = threads or cores
    O.register_texture_file("worldmap.png", os.path.join(SCENES, "worldmap.png"))
    sc = O.OracleScene(text, t, W, H, max_depth=depth)
    frames = 0
    t0 = time.perf_counter()
    while True:
        sc.render(0, H, threads=threads, u8=True)
        frames += 1
        if time.perf_counter() - t0 >= target_s or frames >= 50:
            break
    dt_all = (time.perf_counter() - t0) / frames
    step = 27
    rows = len(range(0, H, step))
    t0 = time.perf_counter()
    sc.render(0, H, row_step=step, threads=1, u8=True)
    dt_one = time.perf_counter() - t0
    return {
        "value": round(W * H / dt_all / 1e6, 3),
        "unit": "Mrays/s",
        "cores": threads,
        "kind": "port",
        "cpu_model": model,
        "host_cpus_affinity": aff,
        "cgroup_cpu_quota": quota,
        "sample": f"{frames} whole {W}x{H} frame(s), rows interleaved over {threads} threads "
                  f"({dt_all * frames * threads:.1f} thread-s of CPU work); oracle/rt_oracle.c -O2 -ffp-contract=off",
        "single_thread_value": round(rows * W / dt_one / 1e6, 3),
        "single_thread_sample": f"every {step}th row ({rows} rows x {W} px) on 1 thread",
    }


def main():
    a = parse()
    launched = "WORLD_SIZE" in os.environ or "LOCAL_RANK" in os.environ
    if a.gpus > 1 and not launched:
        sys.exit(self_launch(a))         # before anything here touches the GPU
    # Exactly one JSON line on stdout: libraries (RCCL prints a version banner at communicator
    # creation) write to fd 1 as well, so route fd 1 to stderr and keep a private copy for the line.
    json_out = os.fdopen(os.dup(1), "w")
    os.dup2(2, 1)
    if a.launcher_check:
        return launcher_check(a, json_out)
    import torch
    import torch.distributed as dist
    import tinyraytracerinrust_amd as T
    from tinyraytracerinrust_amd import distributed as D

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != a.gpus:
        raise SystemExit(f"--gpus {a.gpus} but WORLD_SIZE={world}: one rank per GPU")
    rehearse = a.rehearse_one_gpu
    if rehearse:
        if not launched:
            raise SystemExit("--rehearse-one-gpu: under a launcher (--gpus N > 1 starts one)")
        local = 0                        # every rank on the one GPU
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    multi = world > 1 or a.force_collective or rehearse
    if rehearse:
        dist.init_process_group("gloo")
    elif multi:
        # The gathers run on RCCL's stream while later frames' renders fill every CU.  A
        # high-priority RCCL stream (--rccl-priority high) measured 7 % slower per step on the RCCL
        # path at world 1 (0.625 vs 0.582 ms, profiles/r02bw_rccl_priority.txt): normal by default.
        opts = dist.ProcessGroupNCCL.Options()
        opts.is_high_priority_stream = a.rccl_priority == "high"
        dist.init_process_group("nccl", device_id=dev, pg_options=opts)

    if a.config in ANIM:
        return anim_main(a, json_out, rank, world, local, dev, multi, rehearse)
    scene, W, H, t, depth = CONFIGS[a.config]
    text = open(os.path.join(SCENES, scene + ".scene")).read() if scene else SPHERE_SCENE
    scene = scene or "sphere"
    rt = T.RayTracer(W, H, device=local)
    rt.load_scene(text, t, asset_dir=SCENES)
    t_up = time.perf_counter()
    # the upload: the scene blob + texture to HBM, and (the library's default, RT_OPT_SPECIALIZE 1) the
    # request for the scene's specialised program, compiled by the library's pool in the background
    rend = rt.renderer
    # bench times the launches with its own events on the launch stream: the library's per-launch
    # event pair (rt_ctx_last_kernel_ms) is off, as a host that does not read it would run
    # (RT_OPT_TIMING: each timed event costs the stream ~5 us, profiles/r02dc_launch_events.txt)
    rend.set_timing(False)
    if not a.specialize:
        rend.set_specialize(0)
    frame0 = rend.render_rows(0, H, max_depth=depth)     # the host's first frame: at once, whatever is loaded
    torch.cuda.synchronize(dev)
    first_frame_ms = round((time.perf_counter() - t_up) * 1e3, 1)
    first_kernel = rend.kernel_info().split("last launch: ")[-1]
    spec_ms = spec = None
    if a.specialize:
        rend.spec_wait()                                  # setup: before the settle / warmup / timed steps
        spec_ms = round((time.perf_counter() - t_up) * 1e3, 1)
        spec = {"request_to_loaded_ms": spec_ms, "first_frame_ms": first_frame_ms, "first_frame_kernel": first_kernel,
                "generic_ms_per_frame": generic_frame_ms(T, text, t, W, H, depth, local, dev) if world == 1 else None,
                "note": "RT_OPT_SPECIALIZE 1 (the library default) compiles in a background pool: upload and the first "
                        "frames return at once on the generic kernels, the specialised kernels take over when loaded "
                        "(request_to_loaded_ms, the compile plus the load; ~0 with the on-disk or comgr cache warm)"}
    del frame0

    layout = a.layout if multi else "contiguous"
    band = a.band if layout == "cyclic" else -(-H // world)
    slot_rows = D.rows_per_rank(H, world, layout, band)
    mine = owned_rows(H, world, rank, layout, band)
    y_first, band_rows, pitch, n_bands = D.band_params(H, world, rank, layout, band)
    frame = torch.zeros((H, W, 4), dtype=torch.uint8, device=dev)
    stream = torch.cuda.current_stream(dev)
    overlap = multi and not a.no_overlap
    # Up to K frames' renders overlap, each frame on its own HIP stream: a frame (or a rank's
    # share of it) ends with its costliest tiles running alone (DESIGN.md "Multi-GPU"), so a lone
    # frame leaves the GPU partly idle.  N > 1: frame k's all-gather (RCCL stream) also runs under
    # later frames' renders.  Every frame is still fully rendered (gathered and assembled) inside
    # the timed region.
    K = a.inflight if a.inflight > 0 else (1 if world == 1 else 4)
    if multi and not overlap:
        K = 1
    nbuf = K + 1 if multi else K     # N = 1: buffer b is only ever written on stream b
    # With several frames in flight the launches overlap, so no launch's tail leaves the GPU idle:
    # the per-lane megakernel then beats the deferred-shadow kernel that the library picks for a
    # lone tail-bound launch (a rank's share at N = 4 / 8 with K = 4: 0.148 / 0.076 ms against
    # 0.182 / 0.093 ms, profiles/r02x_inflight_*.txt).
    if K >= 3:
        rend.set_kernel("mega")
    # Each in-flight frame on a stream with a hardware queue of its own (rt_stream_create): torch's
    # pool streams share the process's 4 hardware queues, and two renders whose streams land on
    # one queue serialise -- a rank's N = 8 share with K = 4 measured 0.072 or 0.118 ms depending
    # on which pool streams it got, 0.075-0.079 every time on own-queue streams
    # (profiles/r02ba_streams.txt).
    hw = [] if K == 1 or a.pool_streams else [T.HwStream(local) for _ in range(K)]
    rstreams = [stream] if K == 1 else [h.torch for h in hw] if hw else [torch.cuda.Stream(dev) for _ in range(K)]
    ch = 3 if a.gather == "rgb" else 4
    slots = [torch.zeros((slot_rows, W, ch), dtype=torch.uint8, device=dev) for _ in range(nbuf)] if multi else []
    gath = [torch.zeros((world * slot_rows, W, ch), dtype=torch.uint8, device=dev) for _ in range(nbuf)] if multi else []
    frames = [frame] + [torch.zeros_like(frame) for _ in range(nbuf - 1)]
    free_ev = [None] * nbuf    # buffer b's last gather and assembly are done once this event fires
    pending = []               # (work, buffer) of gathers not yet assembled, oldest first
    # Assemblies run on a stream of their own: on a render stream an assembly would queue behind
    # that stream's NEXT render, and the render after it (which waits for the buffer the assembly
    # frees) could not start before the previous render ended -- the renders would serialise.
    ahw = T.HwStream(local) if K > 1 and not a.pool_streams else None    # kept alive with the stream
    astream = stream if K == 1 else (ahw.torch if ahw else torch.cuda.Stream(dev))

    def finish(p):
        work, b = p
        with torch.cuda.stream(astream):
            work.wait()                                   # astream waits for the gather
            D.assemble(gath[b], H, world, layout, band, out=frames[b])
            free_ev[b] = torch.cuda.Event()
            free_ev[b].record(astream)

    # N = 1: each (buffer, stream) pair's launch pre-bound (Renderer.rows_launcher): one ctypes call per
    # frame, as a native host's FFI call, not the Python wrapper's per-call argument handling
    launchers = [rend.rows_launcher(0, H, frames[b], max_depth=depth, stream=rstreams[b % K]) for b in range(nbuf)] \
        if not multi else []

    def step(i, ev0=None, ev1=None):
        b = i % nbuf
        s = rstreams[i % K]
        if not multi and free_ev[b] is None:
            if ev0 is not None:
                ev0.record(s)
            launchers[b]()
            if ev1 is not None:
                ev1.record(s)
            return
        with torch.cuda.stream(s):
            if free_ev[b] is not None:
                s.wait_event(free_ev[b])                  # slot / gather / frame buffers reusable
            if ev0 is not None:
                ev0.record(s)
            if not multi:
                rend.render_rows(0, H, max_depth=depth, out=frames[b], stream=s)
            else:
                rend.render_row_bands(y_first, band_rows, pitch, n_bands, slots[b], max_depth=depth, stream=s)
            if ev1 is not None:
                ev1.record(s)
            if multi:
                work = (HostGather(gath[b], slots[b], s) if rehearse else
                        dist.all_gather_into_tensor(gath[b], slots[b], async_op=True))   # after s's render
        if multi:
            pending.append((work, b))
            while len(pending) > (K if overlap else 0):
                finish(pending.pop(0))

    def drain():
        while pending:
            finish(pending.pop(0))

    # settle (setup, untimed, not a step): the first launch of the geometry calibrates the tile
    # order; then frames render until the GPU has run `settle_ms` at sustained clocks
    settle_frames, ts = 0, time.perf_counter()
    while settle_frames < 1 or (time.perf_counter() - ts) * 1e3 < a.settle_ms:
        if multi:
            rend.render_row_bands(y_first, band_rows, pitch, n_bands, slots[0], max_depth=depth, stream=stream)
        else:
            rend.render_rows(0, H, max_depth=depth, out=frames[0], stream=stream)
        settle_frames += 1
        if settle_frames % 8 == 0 or settle_frames == 1:
            torch.cuda.synchronize(dev)
    torch.cuda.synchronize(dev)
    settle = {"frames": settle_frames, "ms": round((time.perf_counter() - ts) * 1e3, 1)}
    if multi:
        dist.barrier()
    for i in range(a.warmup):
        step(i)
    drain()
    torch.cuda.synchronize(dev)
    # One launch stream (N = 1, one frame at a time): ONE event pair on that stream brackets the
    # timed region, and the kernel time per launch is its span / K -- a timed event costs the
    # stream ~5 us (profiles/r02dc_launch_events.txt), so events around every launch would slow the
    # launches they measure.  Otherwise (several streams, or the collective path) a pair per step.
    # With frames in flight (K > 1) the roofline is taken over wall time and per-step events would
    # only add their cost to every render stream: none are recorded then.
    region = K == 1 and not multi
    per_step = K == 1 and multi
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(a.steps)] \
        if per_step else []
    reg = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
    if multi:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    if region:
        reg[0].record(stream)
    for i in range(a.steps):
        step(a.warmup + i, *(evs[i] if evs else (None, None)))
    if region:
        reg[1].record(stream)
    drain()
    torch.cuda.synchronize(dev)
    if multi:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if multi:
        e = torch.tensor([elapsed], dtype=torch.float64, device="cpu" if rehearse else dev)
        dist.all_reduce(e, op=dist.ReduceOp.MAX)
        elapsed = float(e.item())
    kernel_ms = ([s.elapsed_time(e) for s, e in evs] if evs else
                 [reg[0].elapsed_time(reg[1]) / a.steps] if region else [elapsed * 1e3 / a.steps])
    mean_kernel_ms = sum(kernel_ms) / len(kernel_ms)
    rows_per_rank = None
    # outside the timed region: every frame buffer holds one of the last frames (assembled, at
    # N > 1); each must equal a single-launch render of the whole frame on the default stream
    # (catches any stream-ordering or buffer-reuse mistake)
    whole = rend.render_rows(0, H, max_depth=depth)
    torch.cuda.synchronize(dev)
    used = min(nbuf, a.warmup + a.steps)
    bad = [b for b in range(used) if not torch.equal(frames[b], whole)]
    if bad:
        raise SystemExit(f"rank {rank}: frame buffer(s) {bad} differ from the single-launch render")
    frame_check = f"all {used} frame buffers == single-launch render" + (", on every rank" if multi else "")
    if multi:
        counts = [None] * world
        dist.all_gather_object(counts, sum(y1 - y0 for y0, y1 in mine))
        rows_per_rank = counts
    busy_ms = mean_kernel_ms if K == 1 else elapsed * 1e3 / a.steps

    # One definition of scaling (DESIGN.md "Multi-GPU"): the line carries BOTH the latency and the
    # throughput figure at every N, measured after the timed region (they are not `value`):
    # N = 1: `inflight4` -- the same frames with 4 in flight on own-queue streams (the N > 1 default);
    # N > 1: `single_frame` -- one frame at a time, fully serialised, with events on the launch stream
    #        around the rank's band render, the all-gather (as seen by the assembly: render end ->
    #        gather done, so it includes waiting for the slowest rank) and the assembly kernel.
    extra_steps = max(4, min(a.steps, 20))
    single = infl = None
    if multi and overlap and not a.no_extra:
        fl0 = load_flops(scene, W, H, t, depth)
        single = single_frame_phase(a, T, rend, dist, D, stream, dev, slots[0], gath[0], frames[0], whole,
                                    (y_first, band_rows, pitch, n_bands), H, W, world, layout, band, depth,
                                    rehearse, extra_steps, fl0["row_flops"] if fl0 else None)
    elif not multi and K == 1 and not a.no_extra:
        infl = inflight_phase(T, rend, stream, dev, frames[0], whole, H, W, depth, local, 4, max(20, a.steps),
                              a.settle_ms)
    if rank == 0 and a.png:
        T.write_png(a.png, frames[(a.warmup + a.steps - 1) % nbuf].cpu().numpy())

    if rank != 0:
        for h in hw + ([ahw] if ahw else []):
            h.close()
        if multi:
            dist.destroy_process_group()
        return

    rows_rendered = [y for (y0, y1) in mine for y in range(y0, y1)]
    fl = load_flops(scene, W, H, t, depth)
    flops_launch = sum(fl["row_flops"][y] for y in rows_rendered) if fl else None
    achieved = flops_launch / (busy_ms * 1e-3) / 1e12 if flops_launch else None
    traffic = load_traffic(a.config, world, layout)
    ex = executed_fp64(a.config, world, layout, busy_ms, rend.kernel_variant())
    # algorithmic bytes of one launch: its RGBA8 rows written + scene blob + the texture once
    alg_bytes = len(rows_rendered) * W * 4 + 1024 * 568 * 4 + 16 * 1024
    line = {
        "metric": "Mrays/sec at 3840x2160 globes.scene" if a.config == "globes4k" else f"Mrays/sec {a.config}",
        "config_name": a.config,
        "value": round(W * H * a.steps / elapsed / 1e6, 2),
        "unit": "Mrays/s",
        "n_gpus": world,
        "steps": a.steps,
        "warmup": a.warmup,
        "ms_per_step": round(elapsed * 1e3 / a.steps, 4),
        "higher_is_better": True,
        "scaling": "strong",
        "vs_baseline": None,
        "dtype": "f64",
        "data": ("synthetic: the reference's own globes.scene + worldmap.png, deterministic (no RNG)"
                 if scene == "globes" else f"synthetic: the one-line scene `{SPHERE_SCENE}`, deterministic"),
        "config": {
            "workload": (f"{scene}.scene" if scene == "globes" else "single red sphere r30, default camera + test light")
                        + f" {W}x{H} t={t:g} max_depth {depth}, one frame per step",
            "scene": f"{scene}.scene" if scene == "globes" else SPHERE_SCENE, "width": W, "height": H, "time": t, "max_depth": depth,
            "parallelism": f"rowtile{world}" + ("" if not multi else f"-{layout}" + (f"{band}" if layout == "cyclic" else "")),
            "collective": None if not multi else f"all_gather_into_tensor (RCCL) of {a.gather.upper()}8 band slots" + (
                ", overlapped with later frames" if overlap else ""),
            "frames_in_flight": K,
            "streams": "current stream" if K == 1 else f"{K} torch pool streams" if a.pool_streams else
                       f"{K} streams, each with its own hardware queue (rt_stream_create)",
            "kernel": "megakernel (rt_ctx_set_option)" if K >= 3 else "library's choice (auto)",
            "frame_bytes": W * H * 4,
        },
        "rays": rays_line(fl, W * H * a.steps / elapsed),
        "roofline": roofline_block(achieved, ex, traffic, {
            "kernel": rend.kernel_info(),
            "kernel_ms_mean": round(mean_kernel_ms, 4),
            "achieved_basis": ("kernel time: one event pair over the K back-to-back launches on the launch stream / K"
                               if region else "kernel event time per launch" if K == 1
                               else f"step wall time ({K} frames in flight; no per-step events)"),
            "kernel_ms_min": round(min(kernel_ms), 4) if per_step else None,
            "algorithmic_flops_per_launch": flops_launch,
            "issue": issue_model(a.config, world, layout, busy_ms),
        }),
        "roofline_hbm": {
            "bound": "hbm",
            "achieved": round(alg_bytes / (busy_ms * 1e-3) / 1e9, 2),
            "peak": HBM_PEAK_GBS,
            "unit": "GB/s",
            "frac": round(alg_bytes / (busy_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 5),
            "algorithmic_bytes_per_launch": alg_bytes,
            "traffic": traffic,
        },
        "cpu_baseline": None,
        "frame_check": frame_check,
        "settle": settle,
        "kernel_code": rend.kernel_info(),
        "spec_compile_ms": spec_ms,
        "specialisation": spec,
    }
    if spec and spec.get("generic_ms_per_frame"):
        g, sp = spec["generic_ms_per_frame"], line["ms_per_step"]
        spec["specialised_ms_per_frame"] = sp
        spec["frames_rendered_generic_meanwhile"] = int(spec_ms / g) if g else None
        spec["break_even_frames_if_blocking"] = int(spec_ms / (g - sp)) if g > sp else None
    if rehearse:
        line.update({"metric": "one-GPU rehearsal of the N-rank pipeline (not a measurement)", "value": None,
                     "vs_baseline": None, "roofline": None, "roofline_hbm": None, "rays": None})
        line["config"]["collective"] = "all_gather_into_tensor (gloo, staged through host memory) of " \
                                       f"{a.gather.upper()}8 band slots; every rank on device 0"
    if multi:
        line["distributed"] = {"backend": dist.get_backend(), "world_size_seen": dist.get_world_size(),
                               "rows_per_rank": rows_per_rank, "layout": layout, "band_rows": band,
                               "frames_in_flight": K, "gather": a.gather,
                               "kernel": "megakernel (rt_ctx_set_option)" if K >= 3 else "library's choice (auto)",
                               "frame_check": frame_check}
    if single is not None:
        line["single_frame"] = single
        if line["value"] is not None and not rehearse:
            single["value"] = round(W * H / (single["ms_per_step"] * 1e-3) / 1e6, 2)
    if infl is not None:
        line["inflight4"] = infl
    if world == 1 and not multi and not a.no_cpu_baseline:
        cb = cpu_baseline(text, W, H, t, depth, a.cpu_threads)
        cb["gpu_over_cpu"] = round(line["value"] / cb["value"], 1)
        line["cpu_baseline"] = cb
    json_out.write(json.dumps(line) + "\n")
    json_out.flush()
    for h in hw + ([ahw] if ahw else []):
        h.close()
    if multi:
        dist.destroy_process_group()


def generic_frame_ms(T, text, t, W, H, depth, local, dev, frames=10):
    """Setup, untimed: the generic kernels' wall ms per frame (a context of its own with RT_OPT_SPECIALIZE
    0; calibration + 3 warm frames first) -- what a host renders at until the specialised program is
    loaded; with the lines' spec_compile_ms it gives the break-even of a BLOCKING compile."""
    import torch
    r = T.Renderer(local, specialize=0)
    r.upload(T.Scene.compile(text, t, W, H, asset_dir=SCENES))
    r.set_timing(False)
    out = torch.empty((H, W, 4), dtype=torch.uint8, device=dev)
    for _ in range(4):
        r.render_rows(0, H, max_depth=depth, out=out)
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(frames):
        r.render_rows(0, H, max_depth=depth, out=out)
    torch.cuda.synchronize(dev)
    ms = (time.perf_counter() - t0) * 1e3 / frames
    r.free()
    return round(ms, 4)


def inflight_phase(T, rend, stream, dev, frame, whole, H, W, depth, local, K, steps, settle_ms):
    """N = 1: `steps` frames with K in flight, each stream on a hardware queue of its own and writing
    only its own buffer, the megakernel (as the N > 1 pipeline runs); checked against `whole`."""
    import torch
    hw = [T.HwStream(local) for _ in range(K)]
    ss = [h.torch for h in hw]
    bufs = [torch.zeros_like(frame) for _ in range(K)]
    rend.set_kernel("mega")
    rend.render_rows(0, H, max_depth=depth, out=bufs[0], stream=stream)      # calibrates this kernel's order
    torch.cuda.synchronize(dev)
    # settle, as before the timed region: the calibration's host sort and the set-up above leave the GPU
    # idle for tens of ms, and a short warm-up then left the clock ramp inside this phase's few timed
    # frames -- round 4's `inflight4` ran 0.371 ms per frame against 0.324 for lone frames, while the
    # same arrangement after a settle measures 0.3243 vs 0.3242 (profiles/r07a_inflight_probe.txt)
    i, ts = 0, time.perf_counter()
    while i < 2 * K or (time.perf_counter() - ts) * 1e3 < settle_ms:
        rend.render_rows(0, H, max_depth=depth, out=bufs[i % K], stream=ss[i % K])
        i += 1
        if i % (8 * K) == 0:
            torch.cuda.synchronize(dev)
    torch.cuda.synchronize(dev)
    launch = [rend.rows_launcher(0, H, bufs[k], max_depth=depth, stream=ss[k]) for k in range(K)]
    t0 = time.perf_counter()
    for i in range(steps):
        launch[i % K]()
    torch.cuda.synchronize(dev)
    el = time.perf_counter() - t0
    bad = [b for b in range(K) if not torch.equal(bufs[b], whole)]
    if bad:
        raise SystemExit(f"inflight phase: frame buffer(s) {bad} differ from the single-launch render")
    rend.set_kernel("auto")
    for h in hw:                 # synchronise and destroy them now, not at the runtime's teardown
        h.close()
    return {"frames_in_flight": K, "steps": steps, "ms_per_step": round(el * 1e3 / steps, 4),
            "value": round(W * H * steps / el / 1e6, 2), "kernel": "megakernel (rt_ctx_set_option)",
            "frame_check": f"all {K} frame buffers == single-launch render",
            "note": "throughput at the N > 1 default of 4 frames in flight: the N > 1 lines' `value` divides by this"}


def single_frame_phase(a, T, rend, dist, D, stream, dev, slot, gath, frame, whole, geom, H, W, world, layout, band,
                       depth, rehearse, steps, row_cost=None):
    """N > 1: one frame at a time, fully serialised (barrier + synchronize around every frame), the
    library's kernel choice for a lone launch.  Returns the max over ranks of the mean per-step wall
    time and this rank's event means (rank 0's in the line).

    --chunks C > 1 (cyclic layout): the frame is C sub-frames (distributed.chunk_plan), cheapest
    first by the reference's per-row flop counts.  Each rank renders its bands of every chunk at once,
    one launch per chunk on its own hardware-queue stream; chunk j's all-gather is queued on RCCL's
    stream behind chunk j's render and its assembly behind that gather, so the cheap chunks' gathers
    and assemblies run while the costly chunk's tail still renders.  Latency = the last chunk's
    render end + its gather + its assembly.  C = 1: render, gather, assembly in series."""
    import torch
    y_first, band_rows, pitch, n_bands = geom
    rend.set_kernel("auto")
    C = a.chunks if layout == "cyclic" else 1
    plan = D.chunk_plan(H, world, band, C, row_cost) if C > 1 else [(0, H)]
    C = len(plan)
    rank = dist.get_rank()
    ch = slot.shape[-1]
    if C > 1:
        params = [D.chunk_band_params(y0, y1, world, rank, band) for y0, y1 in plan]
        cslots = [torch.zeros((p[4], W, ch), dtype=torch.uint8, device=dev) for p in params]
        cgath = [torch.zeros((world * p[4], W, ch), dtype=torch.uint8, device=dev) for p in params]
        hs = [T.HwStream(dev.index) for _ in range(C)]
        ahs = T.HwStream(dev.index)
    rec = []
    warm = 3
    for i in range(warm + steps):
        dist.barrier()
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        if C == 1:
            ev = [torch.cuda.Event(enable_timing=True) for _ in range(4)]
            ev[0].record(stream)
            rend.render_row_bands(y_first, band_rows, pitch, n_bands, slot, max_depth=depth, stream=stream)
            ev[1].record(stream)
            work = HostGather(gath, slot, stream) if rehearse else dist.all_gather_into_tensor(gath, slot, async_op=True)
            work.wait()
            ev[2].record(stream)
            D.assemble(gath, H, world, layout, band, out=frame)
            ev[3].record(stream)
            evs = {"render": [(ev[0], ev[1])], "gather": [(ev[0], ev[2])], "assemble": [(ev[0], ev[3])]}
        else:
            e0 = torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            works, er = [], []
            for j, p in enumerate(params):
                s = hs[j].torch
                s.wait_event(e0)
                with torch.cuda.stream(s):
                    rend.render_row_bands(p[0], p[1], p[2], p[3], cslots[j], max_depth=depth, stream=s)
                    e = torch.cuda.Event(enable_timing=True)
                    e.record(s)
                    er.append(e)
                    works.append(HostGather(cgath[j], cslots[j], s) if rehearse else
                                 dist.all_gather_into_tensor(cgath[j], cslots[j], async_op=True))
            eg, ea = [], []
            with torch.cuda.stream(ahs.torch):
                for j, (y0, y1) in enumerate(plan):
                    works[j].wait()                                  # the assembly stream waits for the gather
                    e = torch.cuda.Event(enable_timing=True)
                    e.record(ahs.torch)
                    eg.append(e)
                    D.assemble(cgath[j], y1 - y0, world, layout, band, out=frame[y0:y1])
                    e = torch.cuda.Event(enable_timing=True)
                    e.record(ahs.torch)
                    ea.append(e)
            evs = {"render": [(e0, e) for e in er], "gather": [(e0, e) for e in eg], "assemble": [(e0, e) for e in ea]}
        torch.cuda.synchronize(dev)
        dt = time.perf_counter() - t0
        if i >= warm:
            rec.append((dt, evs))
    if C > 1:
        for h in hs + [ahs]:
            h.close()
    if not torch.equal(frame, whole):
        raise SystemExit("single-frame phase: the assembled frame differs from the single-launch render")
    wall = sum(d for d, _ in rec) / len(rec)
    e = torch.tensor([wall], dtype=torch.float64, device="cpu" if rehearse else dev)
    dist.all_reduce(e, op=dist.ReduceOp.MAX)
    mean = lambda k, j: round(sum(ev[k][j][0].elapsed_time(ev[k][j][1]) for _, ev in rec) / len(rec), 4)
    out = {"frames_in_flight": 1, "steps": steps, "ms_per_step": round(float(e.item()) * 1e3, 4),
           "chunks": C, "kernel": "library's choice (auto) for a lone launch",
           "frame_check": "assembled frame == single-launch render, on every rank"}
    if C == 1:
        r, g, s = mean("render", 0), mean("gather", 0), mean("assemble", 0)
        out.update({"render_ms": r, "gather_ms": round(g - r, 4), "assemble_ms": round(s - g, 4), "frame_ms": s,
                    "basis": "wall time per serialised frame (max over ranks); render/gather/assemble: rank 0's events "
                             "on its launch stream (gather = render end -> all-gather done, incl. waiting for the "
                             "slowest rank)"})
    else:
        out.update({"chunk_rows": plan,
                    "chunk_render_end_ms": [mean("render", j) for j in range(C)],
                    "chunk_gather_done_ms": [mean("gather", j) for j in range(C)],
                    "chunk_assembled_ms": [mean("assemble", j) for j in range(C)],
                    "render_ms": max(mean("render", j) for j in range(C)),
                    "frame_ms": mean("assemble", C - 1),
                    "basis": "wall time per serialised frame (max over ranks); chunk_*: rank 0's events, ms from the "
                             "frame's start: each chunk's render end (its stream), all-gather done and assembly done "
                             "(the assembly stream), chunks cheapest first"})
        out["last_chunk_gather_ms"] = round(out["chunk_gather_done_ms"][-1] - out["chunk_render_end_ms"][-1], 4)
    return out


class HostGather:
    """--rehearse-one-gpu: the all-gather of one frame's band slots over gloo, staged through host
    memory, with the interface bench's pipeline uses of an async RCCL work handle.  The slot is
    copied out once the render stream `s` has finished it; wait() copies the gathered slots back to
    the device on the CURRENT stream (the assembly stream), as RCCL's wait() orders that stream."""

    def __init__(self, out, slot, s):
        import torch
        import torch.distributed as dist
        s.synchronize()
        self.out = out
        self.host = torch.empty(out.shape, dtype=out.dtype)
        self.work = dist.all_gather_into_tensor(self.host, slot.cpu(), async_op=True)

    def wait(self):
        self.work.wait()
        self.out.copy_(self.host)


def rays_line(fl, primary_per_s):
    """Primary + shadow + reflection + refraction rays of one frame, from the oracle's counters
    (the same ray definition as the reference's spawn sites, raytracer.rs:176,243,268)."""
    if not fl or "totals" not in fl:
        return None
    t = fl["totals"]
    n = {k: int(t.get("ray_" + k, 0)) for k in ("primary", "shadow", "reflect", "refract")}
    total = sum(n.values())
    frames = fl.get("frames", 1)
    return {"per_frame": {k: v // frames for k, v in n.items()}, "total_per_frame": total // frames,
            "total_Mrays_s": round(primary_per_s * total / n["primary"] / 1e6, 2) if n["primary"] else None,
            "source": "oracle event counters (tests/golden/flops_*.json)"}


def launcher_check(a, json_out):
    """The N-rank machinery without a GPU: gloo process group, this rank's band layout filled the
    way rt_render_row_bands fills it (output row r -> frame row y_first + (r / band_rows) *
    band_pitch + r % band_rows) with a per-pixel pattern, one all_gather_into_tensor, the frame
    assembly, and a check of the assembled frame on every rank."""
    import torch
    import torch.distributed as dist
    from tinyraytracerinrust_amd import distributed as D

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    dist.init_process_group("gloo")
    W, H = 97, 163                                   # odd sizes: padded slots, partial last band
    layout = a.layout
    band = a.band if layout == "cyclic" else -(-H // world)

    ch = 3 if a.gather == "rgb" else 4

    def pattern(ys, channels=4):
        ys = torch.as_tensor(ys, dtype=torch.int64).view(-1, 1).expand(-1, W)
        xs = torch.arange(W, dtype=torch.int64).view(1, -1).expand(len(ys), -1)
        a_ = torch.full_like(xs, 255) if channels == 4 and ch == 3 else xs >> 8    # RGB slots: assembled A = 255
        px = torch.stack([ys & 255, ys >> 8, xs & 255, a_], -1).to(torch.uint8)
        return px[..., :channels]

    slot_rows = D.rows_per_rank(H, world, layout, band)
    y_first, band_rows, pitch, n_bands = D.band_params(H, world, rank, layout, band)
    slot = torch.zeros((slot_rows, W, ch), dtype=torch.uint8)
    ys = [y_first + (r // band_rows) * pitch + r % band_rows for r in range(band_rows * n_bands)] if band_rows else []
    keep = [r for r, y in enumerate(ys) if y < H]
    if keep:
        slot[keep] = pattern([ys[r] for r in keep], ch)
    ok = True
    for _ in range(max(1, a.steps)):
        gath = torch.empty((world * slot_rows, W, ch), dtype=torch.uint8)
        dist.all_gather_into_tensor(gath, slot)
        frame = D.assemble(gath, H, world, layout, band)
        ok = ok and torch.equal(frame, pattern(range(H)))
    # the single-frame phase's chunks (distributed.chunk_plan): each sub-frame's bands gathered and
    # assembled on their own, in a cost order that is not the frame order
    chunks_ok = None
    if layout == "cyclic" and a.chunks > 1:
        plan = D.chunk_plan(H, world, band, a.chunks, row_cost=[(y * 7919) % 101 for y in range(H)])
        frame = torch.zeros((H, W, 4), dtype=torch.uint8)
        for y0, y1 in plan:
            f0, br, bp, nb, srows = D.chunk_band_params(y0, y1, world, rank, band)
            cslot = torch.zeros((srows, W, ch), dtype=torch.uint8)
            cys = [f0 + (r // br) * bp + r % br for r in range(br * nb)]
            ck = [r for r, y in enumerate(cys) if y < y1]
            if ck:
                cslot[ck] = pattern([cys[r] for r in ck], ch)
            cg = torch.empty((world * srows, W, ch), dtype=torch.uint8)
            dist.all_gather_into_tensor(cg, cslot)
            D.assemble(cg, y1 - y0, world, layout, band, out=frame[y0:y1])
        chunks_ok = len(plan) > 1 and sorted(plan) == [(c[0], c[1]) for c in sorted(plan)] and \
            torch.equal(frame, pattern(range(H)))
        ok = ok and chunks_ok
    flags = [None] * world
    dist.all_gather_object(flags, (ok, len(keep)))
    if rank == 0:
        line = {"metric": "launcher check (synthetic pattern, no rendering, no measurement)", "value": None,
                "n_gpus": world, "steps": a.steps, "warmup": 0,
                "distributed": {"backend": dist.get_backend(), "world_size_seen": dist.get_world_size(),
                                "rows_per_rank": [n for _, n in flags], "layout": layout, "band_rows": band,
                                "gather": a.gather, "frame_check": all(f for f, _ in flags),
                                "chunks": a.chunks if chunks_ok is not None else 1, "chunks_check": chunks_ok},
                "config": {"width": W, "height": H}}
        json_out.write(json.dumps(line) + "\n")
        json_out.flush()
    dist.destroy_process_group()
    if not all(f for f, _ in flags):
        sys.exit(1)


def anim_main(a, json_out, rank, world, local, dev, multi, rehearse=False):
    """BASELINE config 5: frames f = 0..F-1 of spinning_globes.scene at time f / F, rank r
    renders f = r (mod N) -- replicas, no collective (the reference's animate mode renders its
    frames as independent pool jobs, src/raydebugger/gui.rs:78-89, each with its own scene build,
    debug_window.rs:53-62).  Each owned frame's scene is compiled and uploaded once before the
    timed region (host compile + H2D upload are timed and reported separately, like the
    headline's); one step renders every frame of the animation into its own HBM framebuffer.
    After the timed region every rank compares EVERY owned frame buffer with a single-launch render
    of that frame on the default stream (catches stream-ordering and buffer-reuse mistakes of the
    overlapping streams).  ``--rehearse-one-gpu``: every rank on device 0, gloo process group, no
    value."""
    import torch
    import torch.distributed as dist
    import tinyraytracerinrust_amd as T

    scene, W, H, F, depth = ANIM[a.config]
    text = open(os.path.join(SCENES, scene + ".scene")).read()
    mine = list(range(rank, F, world))
    t0 = time.perf_counter()
    scenes = [T.Scene.compile(text, f / F, W, H, asset_dir=SCENES) for f in mine]
    prep_s = time.perf_counter() - t0
    spec_ms = None
    if a.specialize:
        # setup, as the headline's specialisation: the owned frames' families (one hipRTC program per
        # family of frames of the same structure; spinning_globes: two), each renderer loads its own
        t1 = time.perf_counter()
        T.Scene.register_family(scenes)
        spec_ms = round((time.perf_counter() - t1) * 1e3, 1)
    t0 = time.perf_counter()
    rends = []
    for sc in scenes:
        r = T.Renderer(local, specialize=1 if a.specialize else 0)
        r.upload(sc)                                      # the frame's family program (compiled above) or its own
        if a.specialize:
            r.spec_wait()
        r.set_timing(False)                               # bench's own events time the frames
        r.set_kernel(a.kernel)
        rends.append(r)
    torch.cuda.synchronize(dev)
    prep_ms = (prep_s + time.perf_counter() - t0) * 1e3 / max(1, len(mine))
    variants = sorted({r.kernel_variant() for r in rends})
    outs = [torch.zeros((H, W, 4), dtype=torch.uint8, device=dev) for _ in mine]
    K = max(1, a.streams)
    hw = [] if K == 1 else [T.HwStream(local) for _ in range(K)]      # own hardware queues (main())
    streams = [torch.cuda.current_stream(dev)] if K == 1 else [h.torch for h in hw]
    torch.cuda.synchronize(dev)

    launch = [r.rows_launcher(0, H, outs[j], max_depth=depth, stream=streams[j % K]) for j, r in enumerate(rends)]

    def step(evs=None):
        for j in range(len(rends)):
            stream = streams[j % K]
            if evs is not None:
                evs[j][0].record(stream)
            launch[j]()
            if evs is not None:
                evs[j][1].record(stream)

    settle_frames, ts = 0, time.perf_counter()          # untimed setup, as in main()
    while settle_frames < 1 or (time.perf_counter() - ts) * 1e3 < a.settle_ms:
        step()
        torch.cuda.synchronize(dev)
        settle_frames += len(rends)
    settle = {"frames": settle_frames, "ms": round((time.perf_counter() - ts) * 1e3, 1)}
    for _ in range(a.warmup):
        step()
    torch.cuda.synchronize(dev)
    # one stream: an event pair per frame gives the frames' kernel times; several streams: no events in
    # the timed region (each timed event costs its stream ~5 us, profiles/r02dc_launch_events.txt, and
    # the roofline is taken over wall time then) -- the per-frame times come from one untimed step after
    evs = [[(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in mine]
           for _ in range(a.steps if K == 1 else 1)]
    if multi:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for i in range(a.steps):
        step(evs[i] if K == 1 else None)
    torch.cuda.synchronize(dev)
    if multi:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if multi:
        e = torch.tensor([elapsed], dtype=torch.float64, device="cpu" if rehearse else dev)
        dist.all_reduce(e, op=dist.ReduceOp.MAX)
        elapsed = float(e.item())
    if K > 1:
        step(evs[0])                                      # untimed: the frames' kernel times
        torch.cuda.synchronize(dev)
    per_frame = [sum(evs[i][j][0].elapsed_time(evs[i][j][1]) for i in range(len(evs))) / len(evs)
                 for j in range(len(mine))]
    # outside the timed region: every owned frame buffer == a single-launch render of its frame
    bad = []
    for j, r in enumerate(rends):
        whole = r.render_rows(0, H, max_depth=depth)
        torch.cuda.synchronize(dev)
        if not torch.equal(outs[j], whole):
            bad.append(mine[j])
    if bad:
        raise SystemExit(f"rank {rank}: frame buffer(s) of frames {bad} differ from the single-launch render")
    frame_check = f"all {len(mine)} frame buffers == single-launch render" + (", on every rank" if multi else "")
    frames_per_rank = None
    if multi:
        counts = [None] * world
        dist.all_gather_object(counts, mine)
        frames_per_rank = counts
    for h in hw:
        h.close()
    if rank != 0:
        if multi:
            dist.destroy_process_group()
        return
    path = os.path.join(ROOT, "tests", "golden", f"flops_{scene}_{W}x{H}_anim{F}_d{depth}.json")
    fl = json.load(open(path)) if os.path.exists(path) else None
    achieved = None
    busy_frame_ms = (sum(per_frame) / len(per_frame)) if K == 1 else elapsed * 1e3 / a.steps / len(mine)
    if fl:
        # One stream: the frames' kernel time (events on the launch stream).  Several streams:
        # the kernels overlap, so the flops are divided by the step's wall time instead.
        busy_s = sum(per_frame) * 1e-3 if K == 1 else elapsed / a.steps
        achieved = sum(fl["frame_flops"][f] for f in mine) / busy_s / 1e12
    line = {
        "metric": f"Mrays/sec {scene}.scene {W}x{H} {F}-frame animation",
        "config_name": a.config,
        "value": round(F * W * H * a.steps / elapsed / 1e6, 2),
        "unit": "Mrays/s",
        "n_gpus": world,
        "steps": a.steps,
        "warmup": a.warmup,
        "ms_per_step": round(elapsed * 1e3 / a.steps, 4),
        "higher_is_better": True,
        "scaling": "strong",
        "vs_baseline": None,
        "dtype": "f64",
        "data": f"synthetic: the reference's own {scene}.scene, time = f / {F}, deterministic (no RNG)",
        "config": {
            "workload": f"{scene}.scene {W}x{H} max_depth {depth}, frames 0..{F - 1} at time f/{F}, "
                        f"one step = the whole animation",
            "scene": f"{scene}.scene", "width": W, "height": H, "frames": F, "max_depth": depth,
            "parallelism": f"frames round-robin over {world} rank(s) (replicas), {K} HIP stream(s) per rank",
            "kernel": a.kernel,
            "collective": None,
        },
        "roofline": roofline_block(achieved, executed_fp64(a.config, 1, "contiguous", busy_frame_ms,
                                                            rends[0].kernel_variant()),
                                   load_traffic(a.config, 1, "contiguous"), {
            "kernel": rends[0].kernel_info() + " (ray-chain scene; RT_OPT_KERNEL " + a.kernel + ")",
            "streams": K,
            "achieved_basis": "kernel event time" if K == 1 else "step wall time (frames overlap on the streams; "
                              "kernel_ms_*: one untimed step with events, overlapped)",
            "kernel_ms_mean": round(sum(per_frame) / len(per_frame), 4),
            "kernel_ms_min": round(min(per_frame), 4),
            "kernel_ms_max": round(max(per_frame), 4),
            "issue": issue_model(a.config, 1, "contiguous", busy_frame_ms),
        }),
        "rays": rays_line(fl, F * W * H * a.steps / elapsed),
        "host_compile_upload_ms_per_frame": round(prep_ms, 3),
        "kernel_code": "+".join(variants),
        "spec_compile_ms": spec_ms,
        "settle": settle,
        "cpu_baseline": None,
        "frame_check": frame_check,
    }
    if multi:
        line["distributed"] = {"backend": dist.get_backend(), "world_size_seen": dist.get_world_size(),
                               "frames_per_rank": [len(c) for c in frames_per_rank],
                               "frames_of_rank": frames_per_rank, "frame_check": frame_check}
    if rehearse:
        line.update({"metric": "one-GPU rehearsal of the N-rank animation (not a measurement)", "value": None,
                     "vs_baseline": None, "roofline": None, "rays": None})
    if world == 1 and not multi and not a.no_cpu_baseline:
        from oracle import oracle as O
        cores, model, aff, quota = host_cpus()
        threads = a.cpu_threads or cores
        sample = list(range(0, F, 30))
        t0 = time.perf_counter()
        for f in sample:
            O.OracleScene(text, f / F, W, H, max_depth=depth).render(0, H, threads=threads, u8=True)
        dt = time.perf_counter() - t0
        cb = {"value": round(len(sample) * W * H / dt / 1e6, 3), "unit": "Mrays/s", "cores": threads,
              "kind": "port", "cpu_model": model, "host_cpus_affinity": aff, "cgroup_cpu_quota": quota,
              "sample": f"frames {sample} (whole frames, rows interleaved over {threads} threads, "
                        f"{dt * threads:.1f} thread-s); oracle/rt_oracle.c -O2 -ffp-contract=off"}
        cb["gpu_over_cpu"] = round(line["value"] / cb["value"], 1)
        line["cpu_baseline"] = cb
    json_out.write(json.dumps(line) + "\n")
    json_out.flush()
    if multi:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
