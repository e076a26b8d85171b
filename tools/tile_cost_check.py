#!/usr/bin/env python3
"""How well a counting render's tile costs predict the tiles' real cost
(experiment tool): one 8-rank C2 share (rank 0) counted with
`lpt_pilot_spp` = 2 (the default) and 64 samples per pixel, with the work
counts (cost_time 0: node visits + sphere tests + 12 per segment) and with
wave-time shares (cost_time 1).  Prints per pair the correlation of the tile
costs, the spread of the 2-spp / 64-spp ratio and the most misestimated tiles.

    python tools/tile_cost_check.py [--nranks 8] [--rank 0]
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

import ray_tracing_weekend_amd as rtw  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--nranks", type=int, default=8)
    ap.add_argument("--rank", type=int, default=0)
    a = ap.parse_args()
    W, H, SPP = 1200, 800, 500
    scene, b = rtw.scenes.simple_soa()
    cam = b.with_image_width(W).with_image_height(H).with_samples_per_pixel(SPP).with_max_depth(50).build()
    r = rtw.Renderer(precision=rtw.RTW_F64)
    buf = torch.empty((rtw.tiles_for_rank(W, H, 0, 1) * 64 * 3,), dtype=torch.float64, device="cuda:0")
    costs = {}
    for ct in (0, 1):
        for ps in (2, 64):
            r.set_tuning("cost_time", ct)
            r.set_tuning("lpt_pilot_spp", ps)
            r.set_scene(scene)                      # drops the cached counts
            r.render_device(cam, 7, buf.data_ptr(), buf.numel() * 8, rank=a.rank, nranks=a.nranks)
            full = r.tile_costs(cam, a.rank, a.nranks)
            mine = np.array(sorted(set(np.nonzero(full)[0].tolist())))
            costs[(ct, ps)] = full.astype(np.float64)
    tiles = np.nonzero(costs[(0, 64)])[0]
    out = {}
    for ct in (0, 1):
        c2, c64 = costs[(ct, 2)][tiles] * 32, costs[(ct, 64)][tiles]
        ratio = c2 / np.maximum(c64, 1)
        worst = np.argsort(np.abs(np.log(np.maximum(ratio, 1e-9))))[-8:]
        out[f"cost_time={ct}"] = {
            "corr_2_vs_64": round(float(np.corrcoef(c2, c64)[0, 1]), 4),
            "ratio_p1_p50_p99": [round(float(np.percentile(ratio, p)), 3) for p in (1, 50, 99)],
            "worst_tiles": [int(tiles[k]) for k in worst],
            "worst_ratio": [round(float(ratio[k]), 3) for k in worst],
            "worst_cost64_vs_median": [round(float(c64[k] / np.median(c64)), 2) for k in worst]}
    w64, t64 = costs[(0, 64)][tiles], costs[(1, 64)][tiles]
    tr = (t64 / t64.sum()) / (w64 / w64.sum())
    out["time_vs_work_64spp"] = {"corr": round(float(np.corrcoef(w64, t64)[0, 1]), 4),
                                 "share_ratio_p1_p50_p99": [round(float(np.percentile(tr, p)), 3) for p in (1, 50, 99)],
                                 "max": round(float(tr.max()), 3), "argmax_tile": int(tiles[np.argmax(tr)])}
    print(json.dumps(out), flush=True)
    r.close()


if __name__ == "__main__":
    main()
