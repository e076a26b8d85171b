#!/usr/bin/env python3
"""Per-rank render time of an image split over N ranks (C2 headline by
default; --size 3840x2160 --spp 4096 for C4 shares), measured on ONE
GPU (each rank's share rendered in turn with rtw_render_device(rank, nranks)):
the compute part of the strong-scaling curve the driver's N-GPU bench measures
(it adds the barrier and the one RCCL gather).  Prints one JSON line per N.

Per rank: the first render of a split ("cold": the round robin in tile index
order while it counts the tile costs -- or, with tuning lpt_inline=0, a 2-spp
pilot render first) and the best of --reps steady renders (longest tiles
first).  With --split cost (the default, what a multi-device context does by
itself) the steady renders follow the split dealt from ALL ranks' counted
costs (rtw_split_deal; each rank keeps its round-robin tile count); with
--split rr they stay on the round robin.  Per N the projected frame time adds, for N > 1, an estimate
of the one gather of the packed tiles to rank 0 (each rank's buffer over its
own xGMI link in parallel: 25 us + bytes / 50 GB/s, a conservative share of a
link's ~153 GB/s) and the measured device assemble of N buffers on rank 0.

    python tools/rank_split_time.py [--ns 1,2,4,8] [--reps 3]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

import ray_tracing_weekend_amd as rtw  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ns", default="1,2,4,8")
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--tuning", default="", help="k=v,... (rtw_set_tuning)")
    ap.add_argument("--size", default="1200x800", help="WxH (C4: 3840x2160)")
    ap.add_argument("--spp", type=int, default=500)
    ap.add_argument("--ranks", default="", help="only these ranks of each N (e.g. 0 for one C4 share)")
    ap.add_argument("--split", default="cost", choices=["cost", "rr"],
                    help="cost: the steady renders follow the tiles dealt by the cold renders' counted costs "
                         "(rtw_split_deal, the multi-device default); rr: the round robin T mod N")
    ap.add_argument("--precision", default="f64", choices=["f32", "f64"],
                    help="f64: the headline parity mode (default); f32: the hit64 speed mode")
    a = ap.parse_args()
    W, H = (int(x) for x in a.size.split("x"))
    SPP = a.spp
    scene, b = rtw.scenes.simple_soa()
    cam = b.with_image_width(W).with_image_height(H).with_samples_per_pixel(SPP).with_max_depth(50).build()
    prec = rtw.RTW_F64 if a.precision == "f64" else rtw.RTW_F32
    tdt = torch.float64 if prec == rtw.RTW_F64 else torch.float32
    r = rtw.Renderer(precision=prec)
    for kv in filter(None, a.tuning.split(",")):
        k, v = kv.split("=")
        r.set_tuning(k, int(v))
    r.set_scene(scene)
    buf = torch.empty((rtw.tiles_for_rank(W, H, 0, 1) * 64 * 3,), dtype=tdt, device="cuda:0")
    if W * H * SPP <= 2_000_000_000:
        r.render_device(cam, 1, buf.data_ptr(), buf.numel() * buf.element_size())     # warm-up
    torch.cuda.synchronize()
    base = base_cold = base_frame = None
    for n in (int(x) for x in a.ns.split(",")):
        per_rank, kern, rend, cold, cold_rend = [], [], [], [], []
        only = [int(x) for x in a.ranks.split(",")] if a.ranks else range(n)
        costs = np.zeros(rtw.n_tiles(W, H), np.uint32)
        r.set_split(W, H, n, None)     # the cold renders: the round robin, counting the tile costs
        for rank in only:
            r.set_scene(scene)   # drops the cached task order: the next render counts the tile costs
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            r.render_device(cam, 7, buf.data_ptr(), buf.numel() * buf.element_size(), rank=rank, nranks=n)   # cold render
            torch.cuda.synchronize()
            cold.append((time.perf_counter() - t0) * 1e3)
            cold_rend.append(r.get_timings(1)[0][0])   # the cold render's own kernel
            if a.split == "cost" and n > 1:
                r.tile_costs(cam, rank, n, out=costs)
        split = None
        if a.split == "cost" and n > 1 and not a.ranks:
            split = rtw.split_deal(costs, W, H, n)
            r.set_split(W, H, n, split, costs)
        for rank in only:
            best = float("inf")
            for _ in range(a.reps):
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                r.render_device(cam, 7, buf.data_ptr(), buf.numel() * buf.element_size(), rank=rank, nranks=n)
                torch.cuda.synchronize()
                best = min(best, time.perf_counter() - t0)
            tm = r.get_timings(a.reps)
            kern.append(min(tm[1]))
            rend.append(min(tm[0]))
            per_rank.append(best * 1e3)
        slowest = max(per_rank)
        base = base or slowest
        st = r.get_stats()
        # the gather + device assemble of the N packed buffers (rank 0)
        nbytes = rtw.tiles_for_rank(W, H, 0, n) * 64 * 3 * buf.element_size()
        gather_ms = 0.0 if n == 1 else (25e-6 + nbytes / 50e9) * 1e3
        ranks_buf = torch.zeros((n, rtw.tiles_for_rank(W, H, 0, n) * 64 * 3), dtype=tdt, device="cuda:0")
        img = torch.empty((H, W, 3), dtype=tdt, device="cuda:0")
        r.assemble_tiles(ranks_buf.data_ptr(), ranks_buf.stride(0) * ranks_buf.element_size(), n, W, H, img.data_ptr())
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(5):
            r.assemble_tiles(ranks_buf.data_ptr(), ranks_buf.stride(0) * ranks_buf.element_size(), n, W, H, img.data_ptr())
        torch.cuda.synchronize()
        assemble_ms = (time.perf_counter() - t0) / 5 * 1e3
        frame = slowest + gather_ms + assemble_ms
        frame_cold = max(cold) + gather_ms + assemble_ms
        base_frame = base_frame if n != 1 else frame
        base_cold = base_cold or frame_cold
        cost_share = None
        if split is not None:
            cost_share = [round(float(costs[split == k].astype(np.float64).sum() / costs.astype(np.float64).sum()) * n, 4)
                          for k in range(n)]
        print(json.dumps({"size": a.size, "spp": SPP, "tuning": a.tuning, "nranks": n, "ranks": list(only),
                          "split": a.split if split is not None else "rr", "dealt_cost_share_x_n": cost_share,
                          "chunk": int(st.chunk), "max_rank_ms": round(slowest, 2), "min_rank_ms": round(min(per_rank), 2),
                          "max_rank_cold_ms": round(max(cold), 2),
                          "max_rank_cold_render_kernel_ms": round(max(cold_rend), 2), "gather_est_ms": round(gather_ms, 3),
                          "gather_bytes_per_rank": nbytes, "assemble_ms": round(assemble_ms, 3),
                          "frame_ms": round(frame, 2), "frame_cold_ms": round(frame_cold, 2),
                          "speedup_frame_vs_1": round(base_frame / frame, 2) if base_frame and not a.ranks else None,
                          "speedup_cold_vs_1": round(base_cold / frame_cold, 2),
                          "speedup_vs_1": round(base / slowest, 2), "max_rank_launch_ms": round(max(kern), 2),
                          "max_rank_render_kernel_ms": round(max(rend), 2),
                          "msamples_s_if_parallel": round(W * H * SPP / (slowest * 1e-3) / 1e6, 1),
                          "per_rank_ms": [round(x, 2) for x in per_rank]}), flush=True)
    r.close()


if __name__ == "__main__":
    main()
