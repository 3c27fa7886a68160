"""Algorithmic HBM bytes per pass launch (DESIGN.md "Roofline"), the units the
bench's `roofline.achieved` is computed from.

"Algorithmic" = the bytes the pass must move at minimum with this data
layout: every input read once, every output written once.  BVH node and
triangle fetches and cache re-reads (a gather visits a grid photon once per
overlapping pixel) are not algorithmic; they show up in the PMC traffic.
SURVEY.md 8(d) prices the gather's visited photons (V x 36 B) as HBM bytes;
on MI355X those re-reads are served by L2/MALL (PMC FETCH_SIZE evidences it),
so the roofline here counts each resident photon once and reports V x 36 B
separately as `visited_photon_GBps`.
"""
from __future__ import annotations

from . import _abi

R_RNG = 24            # XORWOW state: v0..v4, d (six dword planes); read + written per use
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md)

KERNELS_OF_PASS = {
    "ppm_eye": ["k_ppm_eye"],
    "ppm_photon": ["k_ppm_photon"],
    # the bucket-sort grid build
    "grid_hash": ["k_grid_setup", "k_bs_count"],
    "grid_scan": ["k_bs_scan_reduce", "k_bs_scan_partials", "k_bs_scan_apply"],
    "grid_scatter": ["k_bs_place", "k_bs_cells", "k_grid_coarse_offsets", "k_grid_permute"],
    # the wave-union kernel (default below 4 segments) or the per-lane kernel; one of them per launch
    "ppm_gather": ["k_ppm_gather_union", "k_ppm_gather"],
    "ppm_direct_output": ["k_ppm_direct_output"],
    "pt": ["k_pt"],
    "vcm_light": ["k_vcm_light"],
    "vcm_camera": ["k_vcm_camera"],
    "vcm_shadow": ["k_vcm_light_shadow", "k_vcm_shadow", "k_vcm_accum"],
}


# the other photon maps (orx_config.photon_map): the grid passes' event slots time their build and gather
KERNELS_OF_PASS_MAP = {
    1: {"grid_hash": ["k_hash_build"], "ppm_gather": ["k_ppm_gather_hash"]},
    2: {"grid_hash": ["k_kd_*", "k_rs_*"], "ppm_gather": ["k_ppm_gather_kd_wave"]},
}


def kernels_of(pass_name: str, photon_map: int = 0) -> list:
    return KERNELS_OF_PASS_MAP.get(photon_map, {}).get(pass_name, KERNELS_OF_PASS.get(pass_name, [pass_name]))


def paths_per_iteration(method: int, W: int, H: int, photons: int) -> int:
    """PT W*H; PPM W*H eye + emitted photon paths; VCM 2*W*H."""
    if method == _abi.PROGRESSIVE_PHOTON_MAPPING:
        return W * H + photons
    if method == _abi.VCM_BIDIRECTIONAL_PATH_TRACING:
        return 2 * W * H
    return W * H


def pass_bytes(method: int, W: int, H: int, photons: int, valid: float = 0.0, cells: int = 0,
               light_vertices: float = 0.0, deposits_max: int = 4, grid_max: int = 1000000,
               photon_map: int = 0, vcm_entries: float = 0.0, vcm_light_entries: float = 0.0) -> dict:
    """Bytes per launch of each pass.

    valid: grid-resident photons (deposits with power > 0); cells: grid cells G;
    light_vertices: stored VCM light vertices per iteration; deposits_max: D
    slots per emitted photon; grid_max: PHOTON_GRID_MAX_SIZE (bucket table size); vcm_entries: the
    camera pass's deferred connection shadow rays per iteration (0: traced in place); vcm_light_entries:
    the light pass's camera connections deferred to the same resolve."""
    N = W * H
    slots = photons * deposits_max
    table = ((cells + 1023) // 1024) * ((slots + 16383) // 16384)
    R2 = 2 * R_RNG
    if method == _abi.PROGRESSIVE_PHOTON_MAPPING and photon_map == 2:
        # kd-tree: the build reads each valid photon's position once and writes its 48 B node;
        # the gather reads every hitpoint and writes the indirect (node reads are visit-dependent)
        return {
            "ppm_eye": N * (R2 + 40),
            "ppm_photon": photons * (R2 + 1) + valid * (36 + 12),
            "grid_hash": photons * 1 + valid * (12 + 48),
            "ppm_gather": N * (40 + 12) + valid * 48,
            "ppm_direct_output": N * (40 + R2 + 12 + 12 + 24),
        }
    if method == _abi.PROGRESSIVE_PHOTON_MAPPING:
        return {
            # RNG RMW + one 40 B hitpoint (pos|flags 16, normal-or-radiance|atten.x 16, atten.yz 8)
            "ppm_eye": N * (R2 + 40),
            # RNG RMW + 1 B deposit mask per emitted photon + 36 B per stored deposit
            # + its 12 B compact position copy (the grid build's key input)
            "ppm_photon": photons * (R2 + 1) + valid * (36 + 12),
            # mask per emitted photon, position 12 B per deposit, key 4 B per slot
            "grid_hash": photons * 1 + valid * 12 + slots * 4,
            # bucket x chunk table read + written (counts -> offsets)
            "grid_scan": table * 8,
            # keys read, (key, slot) pairs written + read twice, permutation written + read,
            # offsets written, photon 36 B read + written
            "grid_scatter": slots * 4 + valid * (8 + 16 + 4 + 4 + 36 + 36) + (cells + 1) * 4,
            # hitpoint 40 B + indirect 12 B per pixel, each grid photon once, offset table once
            "ppm_gather": N * (40 + 12) + valid * 36 + (cells + 1) * 4,
            # hitpoint, RNG RMW, indirect read, direct written, output read + written
            "ppm_direct_output": N * (40 + R2 + 12 + 12 + 24),
        }
    if method == _abi.VCM_BIDIRECTIONAL_PATH_TRACING and vcm_entries:
        return {
            # RNG RMW, vertex count, 64 B per stored light vertex, a 48-B entry per deferred camera connection
            "vcm_light": N * (R2 + 4) + light_vertices * 64 + vcm_light_entries * 48,
            # RNG RMW, vertex count, every stored vertex read once, a 49-B entry per connection, the
            # pixel's list head and emitter term
            "vcm_camera": N * (R2 + 4 + 4 + 16) + light_vertices * 64 + vcm_entries * 49,
            # entries read by the shadow rays (ray, occlusion byte written) and by the colour sums (link,
            # byte, contribution); list head, emitter term, splat read, camera colour, output RMW per pixel
            # and the light pass's connections read (48 B) with their splat (12 B read + written)
            "vcm_shadow": vcm_entries * (32 + 1 + 16 + 1 + 16) + N * (4 + 16 + 12 + 12 + 24)
                          + vcm_light_entries * (48 + 24),
        }
    if method == _abi.VCM_BIDIRECTIONAL_PATH_TRACING:
        return {
            # RNG RMW, vertex count, 64 B per stored light vertex
            "vcm_light": N * (R2 + 4) + light_vertices * 64,
            # RNG RMW, vertex count, splat read, camera colour, output RMW, every stored vertex read once
            "vcm_camera": N * (R2 + 4 + 12 + 12 + 24) + light_vertices * 64,
        }
    return {"pt": N * (R2 + 24)}


def roofline(pass_name: str, bytes_per_launch: float, ms_per_launch: float, traffic=None, photon_map: int = 0,
             kernels=None) -> dict:
    """kernels: the pass's kernels the profile of this workload saw dispatched (default: all of the pass)"""
    achieved = bytes_per_launch / (ms_per_launch * 1e-3) / 1e9 if ms_per_launch > 0 else 0.0
    return {"kernel": "+".join(kernels or kernels_of(pass_name, photon_map)), "pass": pass_name,
            "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBS, 5), "traffic": traffic,
            "bytes_per_launch": int(bytes_per_launch), "avg_launch_ms": round(ms_per_launch, 4)}
