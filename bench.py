#!/usr/bin/env python3
"""Benchmark of the hot path: Msamples/s of the reference's ray_colour loop on
the Book-1 final scene (scenes::simple), BASELINE.json configs[1]:
1200x800, 500 spp, max_depth 50, one MI355X per rank.  The headline runs the
f64 parity mode -- the reference's own f64 arithmetic,
bit-identical to the oracle, so the line is the creditable one;
`modes` adds the f32 speed modes as secondary single-GPU lines: hit64 (f32
with the reference's self-intersection decisions made in f64, within the
stated statistical f32 tolerance of DESIGN.md §2b) and plain f32.
`configs` adds BASELINE configs[2] (C3, 10k spheres, 1920x1080x1024 spp) and
configs[4] on one GPU (C5, 1M spheres, 1920x1080x256 spp: the HBM/MALL
roofline point), each in f64 and f32.

A step = one full render of the image (every pixel x every sample) from the
scene already resident in HBM; the image's 8x8 tiles are interleaved over
the ranks (tile T -> rank T % N), and for N > 1 the ranks' packed tiles are
gathered to rank 0 over RCCL and un-interleaved there inside the step.

    python bench.py [--gpus N] [--steps K] [--warmup W]
    torchrun --nproc-per-node N bench.py --gpus N ...   (one process per GPU)

`--gpus N` > 1 without torchrun renders on N GPUs from this one process
through the C-ABI's multi-device context (rtw_create_devices: one rank per
GPU, one RCCL gather); it exits non-zero when fewer than N GPUs are visible,
and under torchrun --gpus must equal WORLD_SIZE.

Rank 0 prints ONE JSON line (see DESIGN.md §Measurement for every field).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

import ray_tracing_weekend_amd as rtw  # noqa: E402
from ray_tracing_weekend_amd import sharding  # noqa: E402

SCENE_SEED = 0x5EED0001
W, H, SPP, DEPTH = 1200, 800, 500, 50
PEAK_FP32_TFLOPS = 157.3     # MI355X vector FP32 (MI355X_MICROARCH.md, chip table)
PEAK_FP64_TFLOPS = 78.6      # MI355X vector FP64
# Roofline flops.  `roofline.achieved` is the arithmetic the kernel EXECUTES,
# priced from its own counters (node visits, sphere tests, segments, Lambertian
# bounces) -- a fraction of the VALU peak.  The brute-force-
# equivalent rate of SURVEY.md §8d (every sphere's 23-flop discriminant per
# segment + the light loop, what the reference's algorithm would need) is
# reported beside it as `algorithmic_equiv_tflops`: the BVH skips most of that
# work, so that rate can exceed the peak and is not a roofline fraction.
ALG_SPHERE = 23              # flops to the discriminant
ALG_PLANE = 6
ALG_LAMBERT_BASE = 40
FLOP_SPHERE = 17             # oc (3) + half_b (5) + c = oc.oc - r^2 (6) + disc (3)
FLOP_BOX = 20                # one child slab test: 6 x (lo*inv - o*inv) + 6 min/max + 2 clamps
FLOP_PLANE = 6               # d.n (5) + compare
FLOP_LAMBERT_BASE = 40       # mixture sample + ONB + cosine pdf, per Lambertian bounce
FLOP_LIGHT = 17              # one light's Sphere::hit discriminant in HittablePdf::value
FLOP_CELL = 8                # one light-grid DDA step: 2 compares + exit_t (sub, fma, mul, max) + select
ACCEL_NAMES = {1: "brute_lds", 2: "bvh"}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--precision", choices=["f32", "f64"], default="f64",
                    help="f64: the parity mode, the reference's arithmetic, bit-identical to the oracle "
                         "(the headline; FP64 roofline); f32: the speed mode (hit64)")
    ap.add_argument("--cpu-row-step", type=int, default=100,
                    help="cpu_baseline sample: the fixed image rows step/2, 3 step/2, ... (every step-th row, "
                         "stratified; no pilot, so every run times the same samples)")
    ap.add_argument("--configs", default="C3,C5",
                    help="other BASELINE configs timed on one GPU after the headline (comma list of C3, "
                         "C5; 'none' to skip)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-modes", action="store_true",
                    help="skip the secondary single-GPU lines (f64 parity mode, f32 without f64 hit points)")
    ap.add_argument("--accel", choices=["auto", "brute", "bvh"], default="auto")
    ap.add_argument("--tuning", default="", help="rtw_set_tuning overrides, e.g. bvh_kind=1,auto_chunk=4")
    ap.add_argument("--balance", type=int, default=1,
                    help="N > 1: deal the tiles to the ranks by their counted costs (1, the default) or keep the "
                         "round robin (0)")
    return ap.parse_args()


def pmc_traffic(workload, kernel_name, isa_sha):
    """HBM bytes per render-kernel launch and the PMC fractions of the newest
    committed rocprofv3 PMC summary (tools/pmc_summary.py --traffic: FETCH_SIZE
    x2 + WRITE_SIZE, MI355X_MICROARCH.md "HBM") of this workload whose
    recorded ISA hash of `kernel_name` equals `isa_sha` -- the machine code
    that ran now -- or None (then the line prints null: no profile of this
    code exists)."""
    import glob
    import re
    best = None

    def version(f):   # profiles/r01_v11_traffic.json -> (1, 11): the newest profile wins
        m = re.search(r"r(\d+)_v(\d+)\w*_traffic", os.path.basename(f))
        return (int(m.group(1)), int(m.group(2))) if m else (0, 0)

    for f in sorted(glob.glob(os.path.join(ROOT, "profiles", "*_traffic.json")), key=version):
        with open(f) as fh:
            d = json.load(fh)
        if d.get("workload") == workload and "bytes_per_launch" in d and isa_sha and \
                d.get("isa_sha", {}).get(kernel_name) == isa_sha:
            best = dict(d, file=os.path.relpath(f, ROOT))
    return best


def kernel_identity(r, precision):
    """(rocprof name, ISA hash) of the render kernel the last render of `r`
    launched (rtw_last_kernel + the code object of the loaded librtw.so)."""
    from ray_tracing_weekend_amd import isa
    v = r.last_kernel()
    if v is None:
        return None, None
    return isa.render_kernel_name(precision, *v), isa.kernel_isa_sha(isa.render_kernel_symbol(precision, *v))


HBM_PEAK_GBS = 8000.0        # MI355X HBM3E (MI355X_MICROARCH.md)
MALL_GATHER_GBS = 8600.0     # Infinity Cache, uniformly random rows gathered (MI355X_MICROARCH.md "Indexed rows")
L2_GATHER_GBS = 17000.0      # an XCD's L2, rows shared by every workgroup (ibid., 16.8-18.8 TB/s)


def attach_pmc(roof, workload, kname, sha, chunk_sum_bytes=None, kernel_ms=None):
    """traffic + PMC fractions into a roofline dict, only from a profile of
    the same machine code (else null).  scratch_write_frac = (WRITE_SIZE -
    the chunk sums the kernel must write) / WRITE_SIZE: the share of the
    kernel's writes that is register spill (scratch write-back) or other
    waste; `chunk_sum_bytes` = n_chunks x pixels x 3 x element bytes.
    Beside the line's own `frac` it prints what the PMC says bounds the
    kernel: `valu_lane_frac` = VALU issue x lanes active
    (the share of the SIMDs' lane-cycles doing VALU work), the measured HBM
    rate of `traffic` against 8 TB/s, and `bound_pmc` -- "latency" when the
    waves wait on memory more than 40 % of their cycles while HBM moves less
    than 20 % of its peak, "valu" when the VALU issues on more than 60 % of
    the cycles, else "issue" (neither saturated: divergence / dependency
    stalls)."""
    t = pmc_traffic(workload, kname, sha)
    roof["isa_sha"] = sha
    roof["traffic"] = t["bytes_per_launch"] if t else None
    roof["traffic_source"] = t["file"] if t else None
    for k in ("valu_issue_frac", "lanes_active_frac", "wave_wait_frac", "mem_wait_frac"):
        roof[k] = t.get(k) if t else None
    wb = t.get("write_bytes") if t else None
    roof["write_bytes"] = wb
    roof["chunk_sum_bytes"] = chunk_sum_bytes
    roof["scratch_write_frac"] = (round(max(0.0, wb - chunk_sum_bytes) / wb, 4)
                                  if wb and chunk_sum_bytes is not None else None)
    vi, la, mw = roof["valu_issue_frac"], roof["lanes_active_frac"], roof["mem_wait_frac"]
    roof["valu_lane_frac"] = round(vi * la, 4) if vi is not None and la is not None else None
    hbm = (roof["traffic"] / (kernel_ms * 1e-3) / 1e9) if roof["traffic"] and kernel_ms else None
    roof["hbm_measured_gbs"] = round(hbm, 1) if hbm is not None else None
    roof["hbm_measured_frac"] = round(hbm / HBM_PEAK_GBS, 4) if hbm is not None else None
    if mw is not None and hbm is not None and mw > 0.4 and hbm / HBM_PEAK_GBS < 0.2:
        roof["bound_pmc"] = "latency"
    elif vi is not None:
        roof["bound_pmc"] = "valu" if vi > 0.6 else "issue"
    else:
        roof["bound_pmc"] = None
    return roof


def host_cpus():
    """CPUs this process may use on the host, and what lscpu says about them:
    the affinity mask, capped by a cgroup CPU quota when one is set (the GPU
    box gives each GPU a share of a larger machine)."""
    aff = len(os.sched_getaffinity(0))
    quota = None
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            quota = int(q) / int(per)
    except (OSError, ValueError):
        pass
    info = {"affinity_cpus": aff, "cgroup_cpu_quota": quota, "os_cpu_count": os.cpu_count()}
    try:
        import subprocess
        out = subprocess.run(["lscpu"], capture_output=True, text=True, timeout=10).stdout
        keys = {"Model name": "model", "Socket(s)": "sockets", "Core(s) per socket": "cores_per_socket",
                "Thread(s) per core": "threads_per_core", "CPU(s)": "cpus"}
        for line in out.splitlines():
            k, _, v = line.partition(":")
            if k.strip() in keys:
                info[keys[k.strip()]] = v.strip()
    except (OSError, ValueError, subprocess.SubprocessError):
        pass
    threads = aff if quota is None else max(1, min(aff, int(quota)))
    return threads, info


def cpu_baseline(scene, row_step):
    """The oracle (C restatement of the reference path, oracle/) timed on this
    host on a bounded, FIXED sample of the same workload: the stratified image
    rows step/2, 3 step/2, ... (every `row_step`-th row, the full width, all
    500 spp) of the 1200x800x500spp render, faithful reference-BVH traversal
    (bvh.rs incl. its per-visit node-AABB recomputation), one task per pixel
    over every CPU this process may use.  No pilot: every run times the same
    samples (sky and sphere rows differ several-fold in cost).  Test
    infrastructure used as the CPU baseline only -- never on the GPU path."""
    from oracle import oracle as O
    threads, info = host_cpus()
    cam = O.camera_build(**dict(O.simple_camera_kw(), image_width=W, image_height=H,
                                samples_per_pixel=SPP, max_depth=DEPTH))
    sc = O.Scene(**scene.__dict__)
    rows = (row_step // 2, H, row_step)
    res = {}
    for name, accel in (("bvh_ref", O.ACCEL_BVH_REF), ("bvh_cached", O.ACCEL_BVH_CACHED)):
        t0 = time.perf_counter()
        img, st = O.render(cam, sc, 99, accel=accel, threads=threads, rows=rows)
        dt = time.perf_counter() - t0
        res[name] = (st.samples / dt / 1e6, st.samples, dt)
        if name == "bvh_ref":
            ref_img = img
    v, n, dt = res["bvh_ref"]
    out = {"value": round(v, 4), "unit": "Msamples/s", "cores": threads, "kind": "port",
           "sample": f"the fixed rows {rows[0]}, {rows[0] + row_step}, ... (every {row_step}th, stratified) of the "
                     f"{W}x{H}x{SPP}spp depth-{DEPTH} render ({n} samples, {dt:.1f} s), oracle f64, reference BVH "
                     f"restated incl. per-visit node-AABB recomputation (bvh.rs:147-152), {threads} threads",
           "host": info}
    out["value_bvh_cached"] = round(res["bvh_cached"][0], 4)
    # each leg's samples and seconds, and the threads the host allowed
    out["legs"] = {name: {"msamples_s": round(v_, 4), "samples": int(n_), "s": round(dt_, 2)}
                   for name, (v_, n_, dt_) in res.items()}
    out["threads_note"] = (f"{threads} threads = this process's CPU share (affinity {info.get('affinity_cpus')}, "
                           f"cgroup quota {info.get('cgroup_cpu_quota')}) of a {info.get('os_cpu_count')}-CPU host")
    out["parity"] = parity_on_sample(scene, rows, 99, ref_img)
    return out


def parity_on_sample(scene, oracle_rows, seed, ref_full):
    """BASELINE.json's second metric, per-pixel MAE vs the reference CPU
    renderer, on the same sampled rows of the headline workload: the GPU
    renders the full 1200x800x500spp image in f64 (parity mode) and in f32
    (the benchmarked mode) with the oracle's seed; the oracle's rows (already
    rendered above) are the reference.  MAE of sum/spp over NaN-free pixels."""
    rows = list(range(*oracle_rows))
    ref = ref_full[rows]
    builder = rtw.scenes.simple_soa(SCENE_SEED)[1]
    gcam = builder.with_image_width(W).with_image_height(H).with_samples_per_pixel(SPP).with_max_depth(DEPTH).build()
    out = {"rows": len(rows), "pixels": len(rows) * W, "spp": SPP, "seed": seed}
    for name, prec in (("f64", rtw.RTW_F64), ("f32", rtw.RTW_F32)):
        with rtw.Renderer(device=torch.cuda.current_device(), precision=prec) as r:
            # the library's defaults, as timed: one sample per work item (chunk 1,
            # the chunk sums fit in the default partial_max), so the per-pixel
            # fold is the reference's sample-by-sample fold and f64 compares bit for bit
            r.set_scene(scene)
            t0 = time.perf_counter()
            img = r.render(gcam, seed)[rows]
            t = time.perf_counter() - t0
            chunk = int(r.stats.chunk)
        ok = ~(np.isnan(img).any(-1) | np.isnan(ref).any(-1))
        out[name] = {"mae": float(np.abs(img[ok] - ref[ok]).mean() / SPP),
                     "max_abs": float(np.abs(img[ok] - ref[ok]).max() / SPP),
                     "bit_identical": float((img == ref).all(-1)[ok].mean()),
                     "nan_mask_equal": bool(np.array_equal(np.isnan(img).any(-1), np.isnan(ref).any(-1))),
                     "nan_pixels": int(np.isnan(img).any(-1).sum()), "nan_pixels_ref": int(np.isnan(ref).any(-1).sum()),
                     "image_mean_rel_bias": float(img[ok].mean() / ref[ok].mean() - 1.0),
                     "render_s": round(t, 3), "chunk": chunk}
    out["tolerance"] = ("f64: per-pixel MAE < 1e-5 and identical NaN masks (north_star); f32: the "
                        "statistical tolerance of DESIGN.md §2 (tests/test_gpu_f32_tolerance.py)")
    return out


FLOPS_BASIS = ("executed, from the kernel's counters (rtw_stats, DESIGN.md §5): node_visits x bvh_width x 20 + "
               "sphere_tests x 17 + segments x planes x 6 + light_tests x 17 + grid_cells x 8 + lambertian x 40 "
               "(light_tests = Lambertian bounces x lights for the linear light loop; the light grid / BVH "
               "kernels count the lights they test)")


def exe_flops_of(st, n_pl):
    """Executed flops of one launch from the kernel's counters."""
    return st.node_visits * int(st.bvh_width) * FLOP_BOX + st.sphere_tests * FLOP_SPHERE + \
        st.segments * FLOP_PLANE * n_pl + st.light_tests * FLOP_LIGHT + st.grid_cells * FLOP_CELL + \
        st.lambertian * FLOP_LAMBERT_BASE


def counters_of(st):
    """The rtw_stats counters the flops / bytes formulas read (per launch)."""
    return {k: int(getattr(st, k)) for k in ("samples", "segments", "lambertian", "node_visits", "sphere_tests",
                                            "light_tests", "grid_cells", "bvh_width")}


def mode_line(scene, cam, precision, tuning, steps, warmup, dev):
    """A secondary single-GPU line of the same C2 workload: `steps` timed full
    renders after `warmup` untimed ones (device-resident output; the same
    counts as the headline) in another arithmetic mode,
    with its executed-flops roofline.  Modes: the f64 parity mode (bit-identical
    to the oracle; FP64 VALU peak) and f32 without f64 hit points (hit64 = 0:
    the plain-f32 speed mode, outside the stated f32 tolerance)."""
    prec = rtw.RTW_F32 if precision == "f32" else rtw.RTW_F64
    tdtype = torch.float32 if prec == rtw.RTW_F32 else torch.float64
    n_pl = len(scene.plane_mat)
    with rtw.Renderer(device=dev.index, precision=prec) as r:
        for k, v in tuning.items():
            r.set_tuning(k, v)
        r.set_scene(scene)
        buf = torch.empty((rtw.tiles_for_rank(W, H, 0, 1) * 64 * 3,), dtype=tdtype, device=dev)
        stream = rtw.torch_stream(dev.index)

        def step(seed):
            r.render_device(cam, seed, buf.data_ptr(), buf.numel() * buf.element_size(), stream=stream)
        elapsed = run_steps(step, steps, warmup, None, lambda: torch.cuda.synchronize(dev))
        render_ms, _ = r.get_timings(steps)
        st = r.get_stats()
        kname, sha = kernel_identity(r, precision)
    avg_ms = float(np.mean(render_ms))
    flops = exe_flops_of(st, n_pl)
    peak = PEAK_FP32_TFLOPS if prec == rtw.RTW_F32 else PEAK_FP64_TFLOPS
    rate = flops / (avg_ms * 1e-3) / 1e12
    line = {"value": round(W * H * SPP * steps / elapsed / 1e6, 3), "unit": "Msamples/s",
            "ms_per_step": round(elapsed / steps * 1e3, 3), "steps": steps, "warmup": warmup, "dtype": precision,
            "tuning": tuning, "kernel": kname, "chunk": int(st.chunk),
            "kernel_ms_avg": round(avg_ms, 3),
            "roofline": {"bound": "valu", "achieved": round(rate, 3), "peak": peak, "unit": "TFLOP/s",
                         "frac": round(rate / peak, 4), "flops_per_launch": int(flops),
                         "counters": counters_of(st)},
            "segments_per_sample": round(st.segments / max(st.samples, 1), 4)}
    esz = 4 if prec == rtw.RTW_F32 else 8
    attach_pmc(line["roofline"], f"book1_simple_{W}x{H}_{SPP}spp_depth{DEPTH}", kname, sha,
               chunk_sum_bytes=W * H * -(-SPP // int(st.chunk)) * 3 * esz, kernel_ms=avg_ms)
    return line


def cold_render(scene, cam, prec, dev):
    """One render of the headline workload by a fresh context, timed alone
    (host clock, device synced on both sides): what a one-shot
    Camera::render pays on top of the steady state: the work buffers, and the
    tile index order instead of longest tiles first (this first render counts
    the tile costs that order the next render's tasks; no separate pilot).
    The scene upload is excluded, as in the metric."""
    tdtype = torch.float32 if prec == rtw.RTW_F32 else torch.float64
    with rtw.Renderer(device=dev.index, precision=prec) as r:
        r.set_scene(scene)
        buf = torch.empty((rtw.tiles_for_rank(W, H, 0, 1) * 64 * 3,), dtype=tdtype, device=dev)
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        r.render_device(cam, 7, buf.data_ptr(), buf.numel() * buf.element_size(),
                        stream=rtw.torch_stream(dev.index))
        torch.cuda.synchronize(dev)
        dt = time.perf_counter() - t0
        render_ms, _ = r.get_timings(1)
    return {"ms": round(dt * 1e3, 3), "value": round(W * H * SPP / dt / 1e6, 3), "unit": "Msamples/s",
            "render_kernel_ms": round(float(render_ms[0]), 3) if render_ms else None,
            "includes": "work-buffer allocation + render in tile index order (counting the tile costs) + fold"}


def run_steps(step, steps, warmup, dist, sync, device=None):
    """W untimed warm-up steps, then EXACTLY `steps` timed steps bracketed by a
    barrier + device sync on both sides; the max over ranks of the elapsed
    time (seconds)."""
    for w in range(warmup):
        step(1000 + w)
    sync()
    if dist is not None:
        dist.barrier()
    sync()
    t0 = time.perf_counter()
    for k in range(steps):
        step(k)
    sync()
    if dist is not None:
        dist.barrier()
    sync()
    elapsed = time.perf_counter() - t0
    if dist is not None:
        t = torch.tensor([elapsed], dtype=torch.float64, device=device)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    return elapsed


def make_step(render, assemble, dist, rank, world_size, buf, gathered, image):
    """One step: this rank renders its tiles into `buf` (packed); with N > 1
    ranks they are gathered to rank 0 (ONE collective: RCCL over xGMI on the
    GPU box, gloo in the CPU test) into the rows of `gathered` [N, numel(buf)],
    which rank 0 un-interleaves into `image`."""
    def step(seed):
        render(seed, buf)
        if dist is not None:
            dist.gather(buf, list(gathered.unbind(0)) if rank == 0 else None, dst=0)
            if rank == 0:
                assemble(gathered, image)
        else:
            assemble(buf.view(1, -1), image)
    return step


def balance_split(local_costs, dist, device, deal, set_split):
    """The cost-dealt rank split of the one-process-per-GPU launch (DESIGN.md
    §7): `local_costs` = this rank's counted tile costs (uint32 [n_tiles],
    its own tiles filled, zeros elsewhere: rtw_tile_costs after one counting
    render), summed over the ranks by ONE all-reduce (the tiles are disjoint,
    so the sum is every tile's cost) -- a planning exchange, once per scene and
    camera, outside the timed steps -- then dealt on every rank by the same
    deterministic rtw_split_deal, so every rank holds the same split.  Returns
    (split, costs)."""
    t = torch.from_numpy(np.asarray(local_costs, np.int64)).to(device)
    dist.all_reduce(t)
    cost = t.cpu().numpy().astype(np.uint32)
    split = deal(cost)
    set_split(split, cost)
    return split, cost


CONFIGS = {   # BASELINE configs[2] and configs[4], one GPU each
    "C3": dict(n=50, w=1920, h=1080, spp=1024, steps=2, warmup=1),
    "C5": dict(n=500, w=1920, h=1080, spp=256, steps=1, warmup=1),
}


def config_line(name, precision, dev):
    """BASELINE configs[2] / configs[4] on one GPU: the scenes::simple generator
    over a 100 x 100 (C3, 10k spheres) or 1000 x 1000 (C5, 1M spheres) grid,
    1920x1080, 1024 / 256 spp, depth 50; `steps` timed full renders after
    `warmup` (the same run_steps as the headline).  C3's roofline is the VALU
    (executed flops, as the headline); C5's is the memory system: the bytes the
    traversal requests (node visits x node bytes + sphere tests x sphere bytes)
    per launch over the kernel time, against 8 TB/s (SURVEY.md §8d "C5 is the
    HBM/MALL point"); `traffic` is the PMC HBM bytes of an ISA-matched profile."""
    cfg = CONFIGS[name]
    prec = rtw.RTW_F32 if precision == "f32" else rtw.RTW_F64
    tdtype = torch.float32 if prec == rtw.RTW_F32 else torch.float64
    scene, b = rtw.scenes.simple_soa(SCENE_SEED, cfg["n"])
    cam = b.with_image_width(cfg["w"]).with_image_height(cfg["h"]).with_samples_per_pixel(cfg["spp"]) \
           .with_max_depth(DEPTH).build()
    n_pl, n_li = len(scene.plane_mat), len(scene.lights)
    with rtw.Renderer(device=dev.index, precision=prec) as r:
        t0 = time.perf_counter()
        r.set_scene(scene)
        t_stage = time.perf_counter() - t0
        buf = torch.empty((rtw.tiles_for_rank(cfg["w"], cfg["h"], 0, 1) * 64 * 3,), dtype=tdtype, device=dev)
        stream = rtw.torch_stream(dev.index)

        def step(seed):
            r.render_device(cam, seed, buf.data_ptr(), buf.numel() * buf.element_size(), stream=stream)
        elapsed = run_steps(step, cfg["steps"], cfg["warmup"], None, lambda: torch.cuda.synchronize(dev))
        render_ms, _ = r.get_timings(cfg["steps"])
        st = r.get_stats()
        kname, sha = kernel_identity(r, precision)
    avg_ms = float(np.mean(render_ms))
    samples = cfg["w"] * cfg["h"] * cfg["spp"]
    workload = f"{name}_simple_grid{2 * cfg['n']}_{cfg['w']}x{cfg['h']}_{cfg['spp']}spp_depth{DEPTH}"
    line = {"value": round(samples * cfg["steps"] / elapsed / 1e6, 3), "unit": "Msamples/s",
            "ms_per_step": round(elapsed / cfg["steps"] * 1e3, 3), "steps": cfg["steps"],
            "warmup": cfg["warmup"], "dtype": precision, "n_gpus": 1,
            "config": {"workload": workload, "spheres": len(scene.sphere_mat), "lights": n_li,
                       "width": cfg["w"], "height": cfg["h"], "spp": cfg["spp"], "max_depth": DEPTH,
                       "chunk": int(st.chunk)},
            "kernel": kname, "kernel_ms_avg": round(avg_ms, 3), "scene_stage_s": round(t_stage, 3),
            "segments_per_sample": round(st.segments / max(st.samples, 1), 4),
            "node_visits_per_segment": round(st.node_visits / max(st.segments, 1), 3),
            "sphere_tests_per_segment": round(st.sphere_tests / max(st.segments, 1), 3)}
    esz = 4 if prec == rtw.RTW_F32 else 8
    csum = cfg["w"] * cfg["h"] * -(-cfg["spp"] // int(st.chunk)) * 3 * esz
    line["light_tests_per_lambertian"] = round(st.light_tests / max(st.lambertian, 1), 3)
    line["grid_cells_per_lambertian"] = round(st.grid_cells / max(st.lambertian, 1), 3)
    if name == "C5":
        # f32 nodes (both child boxes + links) in both precisions: the f64 kernels cull on the f32 tree;
        # leaf spheres {c, r^2} f32 (+ the f64 sphere of a candidate in the parity mode); the light
        # grid's walks: a cell's offset pair (8 B) and each tested light {c, r} (16 B f32, 32 B f64)
        node_b, sph_b = 64, (16 if prec == rtw.RTW_F32 else 16 + 32)
        cell_b, light_b = 8, (16 if prec == rtw.RTW_F32 else 32)
        req = st.node_visits * node_b + st.sphere_tests * sph_b + st.grid_cells * cell_b + st.light_tests * light_b
        rate = req / (avg_ms * 1e-3) / 1e9
        # the requests are gathered rows served by the L2 / Infinity Cache (the working set fits the
        # 256 MB MALL): priced against the MALL's random-row gather rate, the L2's beside it; the
        # PMC-measured HBM rate and bound are attached by attach_pmc
        line["roofline"] = {"bound": "latency", "achieved": round(rate, 2), "peak": MALL_GATHER_GBS, "unit": "GB/s",
                            "frac": round(rate / MALL_GATHER_GBS, 4), "l2_frac": round(rate / L2_GATHER_GBS, 4),
                            "bytes_per_launch": int(req),
                            "basis": f"requests from the counters: node_visits x {node_b} B + sphere_tests x {sph_b} B "
                                     f"+ grid_cells x {cell_b} B + light_tests x {light_b} B, served by L2 / MALL "
                                     "(peak: the Infinity Cache's random-row gather rate, 8.6 TB/s; l2_frac against "
                                     "the L2's 17 TB/s); bound: latency (waves waiting on memory, HBM far from its "
                                     "peak: bound_pmc)",
                            "counters": counters_of(st)}
        attach_pmc(line["roofline"], workload, kname, sha, chunk_sum_bytes=csum, kernel_ms=avg_ms)
        if line["roofline"]["bound_pmc"] not in (None, "latency"):
            line["roofline"]["bound"] = line["roofline"]["bound_pmc"]
    else:
        flops = exe_flops_of(st, n_pl)
        peak = PEAK_FP32_TFLOPS if prec == rtw.RTW_F32 else PEAK_FP64_TFLOPS
        rate = flops / (avg_ms * 1e-3) / 1e12
        line["roofline"] = {"bound": "valu", "achieved": round(rate, 3), "peak": peak, "unit": "TFLOP/s",
                            "frac": round(rate / peak, 4), "flops_per_launch": int(flops),
                            "flops_basis": FLOPS_BASIS, "counters": counters_of(st)}
        attach_pmc(line["roofline"], workload, kname, sha, chunk_sum_bytes=csum, kernel_ms=avg_ms)
    return line


def resolve_launch(gpus, env, visible):
    """How this run spreads over GPUs: ("torchrun", N) -- one process per GPU,
    the driver's N > 1 launch (WORLD_SIZE set; --gpus must equal it),
    ("inproc", N) -- N > 1 GPUs from this one process through the C-ABI's
    multi-device context (needs N visible GPUs), or ("single", 1).  Raises
    SystemExit (non-zero) instead of silently timing fewer GPUs than asked."""
    ws = env.get("WORLD_SIZE")
    if ws is not None and int(ws) > 1:
        if gpus != int(ws):
            raise SystemExit(f"bench.py: --gpus {gpus} but WORLD_SIZE={ws} (torchrun): they must agree")
        return "torchrun", int(ws)
    if gpus < 1:
        raise SystemExit(f"bench.py: --gpus {gpus}: at least one GPU")
    if gpus > 1:
        if visible < gpus:
            raise SystemExit(f"bench.py: --gpus {gpus} but only {visible} GPU(s) visible")
        return "inproc", gpus
    return "single", 1


def main():
    a = parse()
    launch, world_size = resolve_launch(a.gpus, os.environ, torch.cuda.device_count())
    rank = int(os.environ.get("RANK", "0")) if launch == "torchrun" else 0
    local_rank = int(os.environ.get("LOCAL_RANK", "0")) if launch == "torchrun" else 0
    dist = None
    if launch == "torchrun":
        import torch.distributed as dist
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        torch.cuda.set_device(local_rank)
        dist.init_process_group("nccl", device_id=torch.device(f"cuda:{local_rank}"))
    else:
        torch.cuda.set_device(0)
    dev = torch.device(f"cuda:{local_rank}")
    prec = rtw.RTW_F32 if a.precision == "f32" else rtw.RTW_F64
    tdtype = torch.float32 if prec == rtw.RTW_F32 else torch.float64

    scene, builder = rtw.scenes.simple_soa(SCENE_SEED)
    cam = builder.with_image_width(W).with_image_height(H).with_samples_per_pixel(SPP) \
                 .with_max_depth(DEPTH).build()
    r = rtw.Renderer(device=dev.index, precision=prec,
                     devices=list(range(world_size)) if launch == "inproc" else None)
    r.set_accel({"auto": rtw.RTW_ACCEL_AUTO, "brute": rtw.RTW_ACCEL_BRUTE, "bvh": rtw.RTW_ACCEL_BVH}[a.accel])
    for kv in filter(None, a.tuning.split(",")):
        k, v = kv.split("=")
        r.set_tuning(k, int(v))
    r.set_scene(scene)
    r.set_tuning("balance", a.balance)
    plan = None
    assert rtw.tile_size() == sharding.TILE
    image = torch.empty((H, W, 3), dtype=tdtype, device=dev) if rank == 0 else None
    stream = rtw.torch_stream(dev.index)
    if launch == "inproc":
        # every GPU renders its tiles, one RCCL gather to GPU 0, assembled there:
        # all inside rtw_render_image_device (the drop-in's multi-device path)
        def step(seed):
            r.render_image_device(cam, seed, image.data_ptr(), image.numel() * image.element_size(),
                                  stream=stream)

        def sync():
            for k in range(world_size):
                torch.cuda.synchronize(k)
    else:
        # equal-size packed tile buffers (rank 0 holds the most tiles), as the gather needs
        max_tiles = rtw.tiles_for_rank(W, H, 0, world_size)
        buf = torch.zeros((max_tiles * 64 * 3,), dtype=tdtype, device=dev)
        gathered = torch.empty((world_size, buf.numel()), dtype=tdtype, device=dev) if (dist and rank == 0) else None

        def render(seed, out):
            r.render_device(cam, seed, out.data_ptr(), out.numel() * out.element_size(),
                            rank=rank, nranks=world_size, stream=stream)

        def assemble(ranks, img):
            r.assemble_tiles(ranks.data_ptr(), ranks.stride(0) * ranks.element_size(), ranks.shape[0], W, H,
                             img.data_ptr(), stream=stream)

        step = make_step(render, assemble, dist, rank, world_size, buf, gathered, image)

        def sync():
            torch.cuda.synchronize(dev)
        if dist is not None and a.balance:
            # the tiles dealt to the ranks by their costs: one counting render (the
            # round robin, tile index order), the costs all-reduced, the same deal on
            # every rank (the in-process path does this inside rtw_render_image_device)
            t0 = time.perf_counter()
            render(999, buf)
            sync()
            balance_split(r.tile_costs(cam, rank, world_size), dist, dev,
                          lambda c: rtw.split_deal(c, W, H, world_size),
                          lambda s, c: r.set_split(W, H, world_size, s, c))
            plan = {"renders": 1, "s": round(time.perf_counter() - t0, 3),
                    "what": "one counting render + one all-reduce of the tile costs + rtw_split_deal, before "
                            "the warm-up"}
    elapsed = run_steps(step, a.steps, a.warmup, dist, sync, device=dev)

    # live per-launch kernel times of the timed steps (HIP events on the launch
    # stream) and the counters, of rank 0 (the in-process path: its first device)
    r0 = r.rank_view(0) if launch == "inproc" else r
    render_ms, total_ms = r0.get_timings(a.steps)
    st = r0.get_stats()
    per_rank_ms = None
    if launch == "inproc":
        per_rank_ms = [round(float(np.mean(r.rank_view(k).get_timings(a.steps)[0])), 3)
                       for k in range(world_size)]
    samples_total = W * H * SPP * a.steps
    value = samples_total / elapsed / 1e6
    ms_per_step = elapsed / a.steps * 1e3

    if rank != 0:
        if dist is not None:
            dist.destroy_process_group()
        return
    # roofline of the dominant kernel (render_kernel): flops of rank 0's last
    # launch / its average launch duration (HIP events around each launch)
    n_sph, n_pl, n_li = len(scene.sphere_mat), len(scene.plane_mat), len(scene.lights)
    alg_flops = st.segments * (ALG_SPHERE * n_sph + ALG_PLANE * n_pl) + \
        st.lambertian * (ALG_SPHERE * n_li + ALG_LAMBERT_BASE)
    exe_flops = exe_flops_of(st, n_pl)
    accel = ACCEL_NAMES.get(int(st.accel), str(st.accel))
    avg_ms = float(np.mean(render_ms)) if render_ms else float("nan")
    alg_rate = alg_flops / (avg_ms * 1e-3) / 1e12
    exe_rate = exe_flops / (avg_ms * 1e-3) / 1e12
    peak = PEAK_FP32_TFLOPS if prec == rtw.RTW_F32 else PEAK_FP64_TFLOPS
    kname, sha = kernel_identity(r0, a.precision)
    out = {
        "metric": "Msamples/s (pixels x spp) on Book-1 final scene",
        "value": round(value, 3),
        "unit": "Msamples/s",
        "n_gpus": world_size,
        "steps": a.steps,
        "warmup": a.warmup,
        "ms_per_step": round(ms_per_step, 3),
        "higher_is_better": True,
        "scaling": "strong",
        "vs_baseline": None,
        "dtype": a.precision,
        "data": "synthetic: scenes::simple restated with seed 0x5EED0001 (484 spheres, "
                f"{n_li} lights), per-(pixel,sample) xoshiro256++ streams",
        "config": {"workload": f"book1_simple_{W}x{H}_{SPP}spp_depth{DEPTH}", "width": W,
                   "height": H, "spp": SPP, "max_depth": DEPTH, "spheres": n_sph,
                   "lights": n_li,
                   "parallelism": (f"tile8x8_cost_dealt{world_size}" if world_size > 1 and a.balance
                                   else f"tile8x8_interleave{world_size}"),
                   "launch": {"torchrun": "one process per GPU (torch.distributed, RCCL gather)",
                              "inproc": "one process, rtw_create_devices (one rank per GPU, RCCL gather)",
                              "single": "one GPU"}[launch],
                   "accel": accel if accel != "bvh" else f"bvh{int(st.bvh_width)}",
                   "chunk": int(st.chunk),
                   "arithmetic": ("f64, the reference's operation order (bit-identical to the oracle)"
                                  if a.precision == "f64" else
                                  "f32, self-intersection decided in f64 (hit64)" if "hit64=0" not in a.tuning
                                  else "f32")},
        "roofline": {"bound": "valu", "achieved": round(exe_rate, 3), "peak": peak,
                     "unit": "TFLOP/s", "frac": round(exe_rate / peak, 4),
                     "kernel": kname,
                     "kernel_ms_avg": round(avg_ms, 3),
                     "flops_per_launch": int(exe_flops),
                     "flops_basis": FLOPS_BASIS,
                     "counters": counters_of(st),
                     "algorithmic_equiv_tflops": round(alg_rate, 3),
                     "algorithmic_equiv_flops_per_launch": int(alg_flops),
                     "algorithmic_equiv_basis": "SURVEY.md 8d brute-force world query (23 flops x every sphere per "
                                                "segment + light loop); the BVH skips most of it, so this rate may exceed the peak",
                     "segments_per_sample": round(st.segments / max(st.samples, 1), 4),
                     "bvh_width": int(st.bvh_width),
                     "node_visits_per_segment": round(st.node_visits / max(st.segments, 1), 3),
                     "sphere_tests_per_segment": round(st.sphere_tests / max(st.segments, 1), 3),
                     "lambertian_per_sample": round(st.lambertian / max(st.samples, 1), 4)},
    }
    if per_rank_ms is not None:
        out["roofline"]["kernel_ms_per_rank"] = per_rank_ms
    if plan is not None:
        out["config"]["split_plan"] = plan
    attach_pmc(out["roofline"], out["config"]["workload"], kname, sha,
               chunk_sum_bytes=W * H * -(-SPP // int(st.chunk)) * 3 * (4 if prec == rtw.RTW_F32 else 8) // world_size,
               kernel_ms=avg_ms)
    if world_size == 1 and not a.no_modes:
        # the same workload in the other arithmetic modes (single GPU, after the timed region)
        out["modes"] = {}
        if a.precision == "f32":
            out["modes"]["f64_parity"] = mode_line(scene, cam, "f64", {}, a.steps, a.warmup, dev)
        else:
            out["modes"]["f32_hit64"] = mode_line(scene, cam, "f32", {}, a.steps, a.warmup, dev)
        out["modes"]["f32_plain"] = mode_line(scene, cam, "f32", {"hit64": 0}, a.steps, a.warmup, dev)
        out["cold_render"] = cold_render(scene, cam, prec, dev)
    if world_size == 1 and a.configs != "none":
        out["configs"] = {}
        for name in filter(None, a.configs.split(",")):
            for p in (a.precision, "f32" if a.precision == "f64" else "f64"):
                out["configs"][f"{name}_{p}"] = config_line(name, p, dev)
    if world_size == 1 and not a.no_cpu_baseline:
        out["cpu_baseline"] = cpu_baseline(scene, a.cpu_row_step)
    print(json.dumps(out), flush=True)
    r.close()
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
