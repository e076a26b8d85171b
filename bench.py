#!/usr/bin/env python3
"""Benchmark of the hot path: Msamples/s of the reference's ray_colour loop on
the Book-1 final scene (scenes::simple), BASELINE.json configs[1]:
1200x800, 500 spp, max_depth 50, f32 arithmetic, one MI355X per rank.

A step = one full render of the image (every pixel x every sample) from the
scene already resident in HBM; for N > 1 ranks the 8-row tile rows are
interleaved over the ranks and gathered to rank 0 over RCCL inside the step.

    python bench.py [--gpus N] [--steps K] [--warmup W]
    torchrun --nproc-per-node N bench.py --gpus N ...

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
# Roofline flops.  ALGORITHMIC (the roofline's `achieved`):
# per sample F = S*(23*N_s + 6*N_pl) + L*(23*N_L + 40) -- the reference's
# brute-force world query (every sphere's 23-flop discriminant per segment)
# plus the light loop, with S, L the measured segments and Lambertian
# bounces per sample.  EXECUTED (reported beside it): the arithmetic the
# BVH kernel actually performs, priced from its own counters.
ALG_SPHERE = 23              # flops to the discriminant
ALG_PLANE = 6
ALG_LAMBERT_BASE = 40
FLOP_SPHERE = 17             # oc (3) + half_b (5) + c = oc.oc - r^2 (6) + disc (3)
FLOP_BOX = 20                # one child slab test: 6 x (lo*inv - o*inv) + 6 min/max + 2 clamps
FLOP_PLANE = 6               # d.n (5) + compare
FLOP_LAMBERT_BASE = 40       # mixture sample + ONB + cosine pdf, per Lambertian bounce
FLOP_LIGHT = 17              # one light's Sphere::hit discriminant in HittablePdf::value
ACCEL_NAMES = {1: "brute_lds", 2: "bvh"}
KERNEL_NAMES = {0: "brute_l2", 1: "brute_lds", 2: "bvh2_loop", 3: "bvh2_ww", 4: "bvh4_octant",
                5: "bvh2_ww_lds"}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--precision", choices=["f32", "f64"], default="f32")
    ap.add_argument("--cpu-seconds", type=float, default=12.0,
                    help="target CPU time of the cpu_baseline sample")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--accel", choices=["auto", "brute", "bvh"], default="auto")
    ap.add_argument("--tuning", default="", help="rtw_set_tuning overrides, e.g. bvh_kind=1,auto_chunk=4")
    return ap.parse_args()


def pmc_traffic(workload, precision, world):
    """HBM bytes per render-kernel launch from the committed rocprofv3 PMC
    summary of this workload and kernel (tools/pmc_summary.py --traffic:
    FETCH_SIZE x2 + WRITE_SIZE, MI355X_MICROARCH.md "HBM"), or None."""
    import glob
    dtype = "float" if precision == "f32" else "double"
    import re
    best = None

    def version(f):   # profiles/r01_v11_traffic.json -> (1, 11): the newest profile wins
        m = re.search(r"r(\d+)_v(\d+)_traffic", os.path.basename(f))
        return (int(m.group(1)), int(m.group(2))) if m else (0, 0)

    for f in sorted(glob.glob(os.path.join(ROOT, "profiles", "*_traffic.json")), key=version):
        with open(f) as fh:
            d = json.load(fh)
        if d.get("workload") == workload and any(
                k.startswith(f"void rtw::dev::render_kernel<{dtype}, {world},") for k in d.get("kernel", [])):
            best = d
    return best


def cpu_baseline(scene, target_s):
    """The oracle (C restatement of the reference path, oracle/) timed on this
    host on a bounded sample of the same workload: every k-th image row of the
    1200x800x500spp render, faithful reference-BVH traversal (bvh.rs incl. its
    per-visit node-AABB recomputation).  Test infrastructure used as the CPU
    baseline only -- never on the GPU path."""
    from oracle import oracle as O
    threads = min(16, os.cpu_count() or 1)
    cam = O.camera_build(**dict(O.simple_camera_kw(), image_width=W, image_height=H,
                                samples_per_pixel=SPP, max_depth=DEPTH))
    sc = O.Scene(**scene.__dict__)
    res = {}
    for name, accel in (("bvh_ref", O.ACCEL_BVH_REF), ("bvh_cached", O.ACCEL_BVH_CACHED)):
        # pilot: one row, 1/10 of the width, to size the sample
        t0 = time.perf_counter()
        _, st = O.render(cam, sc, 99, accel=accel, threads=1, rows=(H // 2, H // 2 + 1, 1),
                         cols=(0, W // 10))
        per_sample = (time.perf_counter() - t0) / max(st.samples, 1)
        rows = int(max(1, min(H, target_s * threads / (per_sample * W * SPP))))
        step = max(1, H // rows)
        t0 = time.perf_counter()
        img, st = O.render(cam, sc, 99, accel=accel, threads=threads, rows=(0, H, step))
        dt = time.perf_counter() - t0
        res[name] = (st.samples / dt / 1e6, st.samples, step, dt)
        if name == "bvh_ref":
            ref_img = img
        if target_s < 5:
            break
    v, n, step, dt = res["bvh_ref"]
    out = {"value": round(v, 4), "unit": "Msamples/s", "cores": threads, "kind": "port",
           "sample": f"every {step}th row of the {W}x{H}x{SPP}spp depth-{DEPTH} render "
                     f"({n} samples, {dt:.1f} s), oracle f64, reference BVH restated incl. "
                     f"per-visit node-AABB recomputation (bvh.rs:147-152), {threads} threads"}
    if "bvh_cached" in res:
        out["value_bvh_cached"] = round(res["bvh_cached"][0], 4)
    out["parity"] = parity_on_sample(scene, (0, H, step), 99, ref_img)
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
            # one sample per work item (chunk 1), so the per-pixel fold is the
            # reference's sample-by-sample fold: f64 can be compared bit for bit
            r.set_tuning("partial_max", 16 << 30)
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
                     "render_s": round(t, 3), "chunk": chunk}
    out["tolerance"] = "f64: MAE < 1e-5 (north_star); f32: statistical (DESIGN.md §2)"
    return out


def main():
    a = parse()
    world_size = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    if world_size > 1:
        import torch.distributed as dist
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        torch.cuda.set_device(local_rank)
        dist.init_process_group("nccl", device_id=torch.device(f"cuda:{local_rank}"))
    else:
        torch.cuda.set_device(0)
    dev = torch.device(f"cuda:{local_rank if world_size > 1 else 0}")
    prec = rtw.RTW_F32 if a.precision == "f32" else rtw.RTW_F64
    tdtype = torch.float32 if prec == rtw.RTW_F32 else torch.float64

    scene, builder = rtw.scenes.simple_soa(SCENE_SEED)
    cam = builder.with_image_width(W).with_image_height(H).with_samples_per_pixel(SPP) \
                 .with_max_depth(DEPTH).build()
    r = rtw.Renderer(device=dev.index, precision=prec)
    r.set_accel({"auto": rtw.RTW_ACCEL_AUTO, "brute": rtw.RTW_ACCEL_BRUTE, "bvh": rtw.RTW_ACCEL_BVH}[a.accel])
    for kv in filter(None, a.tuning.split(",")):
        k, v = kv.split("=")
        r.set_tuning(k, int(v))
    r.set_scene(scene)
    assert rtw.tile_rows() == sharding.TILE_ROWS
    my_rows = rtw.rows_for_rank(H, rank, world_size)
    max_rows = max(rtw.rows_for_rank(H, k, world_size) for k in range(world_size))
    buf = torch.zeros((max_rows, W, 3), dtype=tdtype, device=dev)
    gathered = [torch.empty_like(buf) for _ in range(world_size)] if (dist and rank == 0) else None
    image = torch.empty((H, W, 3), dtype=tdtype, device=dev) if rank == 0 else None
    stream = torch.cuda.current_stream(dev)

    def step(seed):
        r.render_device(cam, seed, buf.data_ptr(), buf.numel() * buf.element_size(),
                        rank=rank, nranks=world_size, stream=stream.cuda_stream)
        if dist is not None:
            dist.gather(buf, gathered, dst=0)
            if rank == 0:
                sharding.assemble(image, gathered, H)
        elif image is not None:
            image.copy_(buf[:H])

    for w in range(a.warmup):
        step(1000 + w)
    torch.cuda.synchronize(dev)
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for k in range(a.steps):
        step(k)
    torch.cuda.synchronize(dev)
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize(dev)
    elapsed = time.perf_counter() - t0
    if dist is not None:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    # live per-launch kernel times of the timed steps (HIP events on `stream`)
    render_ms, total_ms = r.get_timings(a.steps)
    st = r.get_stats()
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
    exe_flops = st.node_visits * int(st.bvh_width) * FLOP_BOX + st.sphere_tests * FLOP_SPHERE + \
        st.segments * FLOP_PLANE * n_pl + st.lambertian * (FLOP_LIGHT * n_li + FLOP_LAMBERT_BASE)
    accel = ACCEL_NAMES.get(int(st.accel), str(st.accel))
    avg_ms = float(np.mean(render_ms)) if render_ms else float("nan")
    achieved = alg_flops / (avg_ms * 1e-3) / 1e12
    exe_achieved = exe_flops / (avg_ms * 1e-3) / 1e12
    peak = PEAK_FP32_TFLOPS if prec == rtw.RTW_F32 else PEAK_FP64_TFLOPS
    traffic = pmc_traffic(f"book1_simple_{W}x{H}_{SPP}spp_depth{DEPTH}", a.precision, int(st.kernel))
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
                   "lights": n_li, "parallelism": f"rowtile{world_size}",
                   "accel": accel if accel != "bvh" else f"bvh{int(st.bvh_width)}",
                   "chunk": int(st.chunk)},
        "roofline": {"bound": "valu", "achieved": round(achieved, 3), "peak": peak,
                     "unit": "TFLOP/s", "frac": round(achieved / peak, 4),
                     "traffic": traffic["bytes_per_launch"] if traffic else None,
                     "traffic_source": traffic["source"] if traffic else None,
                     "kernel": f"render_kernel<{a.precision}, {KERNEL_NAMES.get(int(st.kernel), st.kernel)}>",
                     "kernel_ms_avg": round(avg_ms, 3),
                     "flops_per_launch": int(alg_flops),
                     "flops_basis": "SURVEY.md 8d brute-force world query (23 flops x every sphere per "
                                    "segment + light loop); frac > 1 = the BVH does less arithmetic",
                     "executed": {"flops_per_launch": int(exe_flops), "achieved": round(exe_achieved, 3),
                                  "frac": round(exe_achieved / peak, 4)},
                     "segments_per_sample": round(st.segments / max(st.samples, 1), 4),
                     "bvh_width": int(st.bvh_width),
                     "node_visits_per_segment": round(st.node_visits / max(st.segments, 1), 3),
                     "sphere_tests_per_segment": round(st.sphere_tests / max(st.segments, 1), 3),
                     "lambertian_per_sample": round(st.lambertian / max(st.samples, 1), 4)},
    }
    if world_size == 1 and not a.no_cpu_baseline:
        out["cpu_baseline"] = cpu_baseline(scene, a.cpu_seconds)
    print(json.dumps(out), flush=True)
    r.close()
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
