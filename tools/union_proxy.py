#!/usr/bin/env python3
"""Price a world-space grouping of the union gather's lanes before building it.

The union gather (k_ppm_gather_union) gives each wave an 8x8 image tile and walks, per (z, y) cell
row, the union [min x_lo, max x_hi] of its lanes' windows; its time is the union photons it walks.
Each lane adds only its own accepted photons in ascending (z, y, sub-row, index) order, so any
grouping of the hit points into waves gives bit-identical sums.  This script runs one PPM
iteration on the GPU, reads the hit points and the grid, and counts at cell granularity (the
kernel refines to sub-rows and quarter cells) the photons walked per wave for
  tiles   the shipped 8x8 image tiles,
  morton  the gathering hit points sorted by the Morton code of their position (cell / 4 units),
          64 consecutive to a wave,
against the lanes' own candidates.  usage: union_proxy.py SCENE WxHxP
"""
import os
import sys

import numpy as np
import pandas as pd
import torch  # noqa: F401  (torch's HIP runtime before liborx's first HIP call)

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from oppositerenderer_amd import _abi, renderer, scenes  # noqa: E402


def morton3(x, y, z):
    def part(v):
        v = v.astype(np.uint64) & np.uint64(0x1FFFFF)
        v = (v | (v << np.uint64(32))) & np.uint64(0x1F00000000FFFF)
        v = (v | (v << np.uint64(16))) & np.uint64(0x1F0000FF0000FF)
        v = (v | (v << np.uint64(8))) & np.uint64(0x100F00F00F00F00F)
        v = (v | (v << np.uint64(4))) & np.uint64(0x10C30C30C30C30C3)
        v = (v | (v << np.uint64(2))) & np.uint64(0x1249249249249249)
        return v
    return part(x) | (part(y) << np.uint64(1)) | (part(z) << np.uint64(2))


def walked(group, lo, hi, gx, gy, off):
    """photons walked: per (group, row) the union x range; lo/hi: [n, 3] cell windows"""
    tot_union, tot_lane = 0, 0
    ny = hi[:, 1] - lo[:, 1] + 1
    nz = hi[:, 2] - lo[:, 2] + 1
    rows_g, rows_r, rows_l, rows_h = [], [], [], []
    for dz in range(int(nz.max())):
        for dy in range(int(ny.max())):
            m = (dz < nz) & (dy < ny)
            row = (lo[m, 2] + dz).astype(np.int64) * gy + (lo[m, 1] + dy)
            rows_g.append(group[m])
            rows_r.append(row)
            rows_l.append(lo[m, 0])
            rows_h.append(hi[m, 0])
    g = np.concatenate(rows_g)
    r = np.concatenate(rows_r)
    lo_x = np.concatenate(rows_l).astype(np.int64)
    hi_x = np.concatenate(rows_h).astype(np.int64)
    tot_lane = int((off[r * gx + hi_x + 1].astype(np.int64) - off[r * gx + lo_x]).sum())
    df = pd.DataFrame({"g": g, "r": r, "l": lo_x, "h": hi_x}).groupby(["g", "r"]).agg(l=("l", "min"), h=("h", "max"))
    rr = df.index.get_level_values(1).to_numpy()
    tot_union = int((off[rr * gx + df["h"].to_numpy() + 1].astype(np.int64) - off[rr * gx + df["l"].to_numpy()]).sum())
    return tot_union, tot_lane


def main():
    scene = scenes.scene_by_name(sys.argv[1] if len(sys.argv) > 1 else "SyntheticHall")
    W, H, P = (int(v) for v in (sys.argv[2] if len(sys.argv) > 2 else "1920x1080x2048").split("x"))
    r = renderer.OptixRenderer(_abi.default_config(seed=1645301512, photon_launch_width=P, photon_launch_height=P))
    r.initialize(0)
    r.initScene(scene)
    det = renderer.RenderRequestDetails(scene.default_camera.set_aspect_ratio(W / H), scene.name,
                                        _abi.PROGRESSIVE_PHOTON_MAPPING, W, H)
    rad = scene.initial_ppm_radius()
    for it in range(3):
        r.renderNextIteration(it, it, rad, True, det)
        hp = r.read_buffer(_abi.BUF_HITPOINTS).reshape(H, W, 13)
        off = r.read_buffer(_abi.BUF_GRID_OFFSETS, np.uint32)
        st = r.stats()
        gx, gy, gz = (int(v) for v in st.grid_size)
        cell = np.float32(st.cell_size)
        org = np.array(list(st.world_origin), np.float32)
        flags = hp[:, :, 12].view(np.uint32)
        act = (flags & np.uint32(_abi.PRD_HIT_NON_SPECULAR)) != 0
        ys, xs = np.nonzero(act)
        pos = hp[ys, xs, 0:3].astype(np.float32)
        npos = pos - org
        inv = np.float32(1.0) / cell
        rf = np.float32(rad)
        lo = np.maximum(0, np.trunc((npos - rf) * inv)).astype(np.int64)
        hi = np.minimum(np.array([gx - 1, gy - 1, gz - 1]), np.trunc((npos + rf) * inv)).astype(np.int64)
        ok = (lo <= hi).all(axis=1)
        xs, ys, pos, lo, hi = xs[ok], ys[ok], pos[ok], lo[ok], hi[ok]
        tile = (ys // 8) * ((W + 7) // 8) + xs // 8
        q = np.clip(np.trunc((pos - org) * inv * 4), 0, 2 ** 21 - 1).astype(np.int64)
        order = np.argsort(morton3(q[:, 0], q[:, 1], q[:, 2]), kind="stable")
        mgroup = np.empty(len(order), np.int64)
        mgroup[order] = np.arange(len(order)) // 64
        ut, lt = walked(tile, lo, hi, gx, gy, off)
        um, _ = walked(mgroup, lo, hi, gx, gy, off)
        nt, nm = len(np.unique(tile)), int(mgroup.max()) + 1
        print(f"it{it} {scene.name} {W}x{H} P{P} r={rad:.4g} cell={cell:.4g} gathering px {len(xs)}: lane candidates "
              f"{lt / len(xs):.1f}/px | tiles {nt} waves, union {ut / len(xs):.1f}/px (factor {64 * ut / lt:.3f}) | "
              f"morton {nm} waves, union {um / len(xs):.1f}/px (factor {64 * um / lt:.3f}) | morton/tiles {um / ut:.3f}",
              flush=True)
        rad = renderer.next_ppm_radius(rad, it)


if __name__ == "__main__":
    main()
