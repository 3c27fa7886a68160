/*
 * orx_kernels.h — launch interface between the host orchestration
 * (orx_capi.cpp) and the gfx950 kernels (orx_kernels.hip).
 */
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "orx_device.h"

namespace orx {

/* Device-resident uniform grid parameters, produced by k_grid_setup from the
 * photon AABB without a host round trip (the reference copies the thrust
 * reduction result to the host, OptixRenderer_SpatialHash.cu:219-236). */
struct GridParams {
    float ox, oy, oz;   /* photonsWorldOrigo (padded AABB min) */
    float cell;         /* photonsGridCellSize */
    uint32_t gx, gy, gz;
    uint32_t G;         /* number of cells */
    uint32_t valid;     /* photons in cells (offsets[G]) */
    uint32_t error;     /* 1: G > PHOTON_GRID_MAX_SIZE */
    uint32_t any_valid;
    uint32_t pad;
    uint64_t photons_visited;   /* this iteration */
    uint64_t cells_visited;
    uint64_t photons_visited_total; /* since orx_reset_timing */
    uint64_t cells_visited_total;
    uint64_t valid_total;
    uint64_t union_photons_total; /* reserved (always 0) */
    uint64_t st_lane_batches, st_wave_batches, st_lane_rows, st_wave_rows; /* ORX_TRAV_STATS builds: gather SIMT */
    uint64_t st_accepted;   /* ORX_TRAV_STATS builds: gather photons within r and facing the normal */
    float clo[3], chi[3];   /* the AABB of the photons in the grid (slab mode's gather cull; empty: +inf/-inf) */
};
/* grid bounds from the caller (slab mode: the AABB of ALL ranks' photons, ordered-int bits as the
 * bbox replicas hold them), so every rank's grid has the single-device grid's origin and cells */
struct GridBox {
    uint32_t on;
    uint32_t b[6]; /* f2ord(lo xyz), f2ord(hi xyz) */
};

/* Per-frame pixel state. Pixel (x,y) of rank r is stored at local row
 * j = (y - r)/world (row-interleaved ownership). */
struct PixelBufs {
    uint32_t W, H;      /* full image */
    uint32_t rank, world;
    uint32_t rows;      /* local rows = number of y with y % world == rank */
    uint32_t RW;        /* RNG buffer width (slot = y*RW + x, global y) */
    RngPlanes rng;      /* local RNG rows: slot index = j*RW + x */
    /* hitpoints: one segment of seg_rows rows laid out as planes
     * [A: seg_rows*W float4][B: seg_rows*W float4][C: seg_rows*W float2]
     * (the multi-GPU export format, 40 B per pixel) */
    float4* hpA;        /* pos.xyz, flags bits */
    float4* hpB;        /* normal.xyz (non-specular hit) | radiance.xyz, atten.x */
    float2* hpC;        /* atten.y, atten.z */
    uint32_t seg_rows;  /* rows per hitpoint segment (= ceil(H/world)) */
    float* indirect;    /* [rows*W*3] */
    float* direct;      /* [rows*W*3] */
    float* output;      /* [rows*W*3] running SUM */
    uint32_t* dbg;      /* [rows*W*2] cells/photons visited, or NULL */
};

constexpr uint32_t BBOX_REPLICAS = 64;
/* grid-ordered photon planes (PhotonBufs::sorted): position, the int8 direction
 * prefilter word of the gather's facing test, exact direction, power */
enum : uint32_t { SP_X = 0, SP_Y, SP_Z, SP_DIRQ, SP_DX, SP_DY, SP_DZ, SP_PX, SP_PY, SP_PZ, SP_PLANES };
#ifndef ORX_SUBX
#define ORX_SUBX 4
#endif
constexpr uint32_t SUBX = ORX_SUBX; /* sub-cells per grid cell along x (bucket-sort grid, gather chord trimming) */
#ifndef ORX_SUBR
#define ORX_SUBR 2
#endif
constexpr uint32_t SUBR = ORX_SUBR; /* sub-rows per grid cell along y and along z (bucket-sort grid, nsub = SUBR^2) */

struct PhotonBufs {
    uint32_t PW, PH;    /* photon launch (full) */
    uint32_t prows;     /* local photon rows */
    uint32_t D;         /* max deposits per emitted photon */
    uint32_t S;         /* local slots = prows*PW*D */
    uint32_t gmax;      /* PHOTON_GRID_MAX_SIZE: capacity of the cell arrays */
    uint32_t gcells;    /* cell count the cell size is chosen for (getSmallestPossibleCellSize): gmax, or
                         * gmax / N for a row shard of world N, whose 1/N of the photons would otherwise
                         * sit in single-device cells (cell edge x N^(1/3), the same photons per cell) */
    float4* slots;      /* [S][4] 64-B deposit records: pos.xyz|power.x, dir.xyz|power.y, power.z, unused
                         * (one record per cache-line half: the grid permute reads it in one go) */
    uint8_t* vmask;     /* [S/D] bit k: deposit k stored with fmaxf(power) > 0 */
    float* sorted;      /* grid-ordered photons, SP_PLANES float planes (SoA): x y z | dirq | dir x y z | power x y z */
    uint32_t splane;    /* plane stride in floats (multiple of 4, >= S + 4) */
    uint32_t* perm;     /* [S] grid position -> photon slot (counting-sort scatter target) */
    uint32_t* keys;     /* [S] sub-cell keys (k_bs_count) */
    uint32_t* offsets;  /* [gmax+2] */
    uint32_t* bbox;     /* [6][BBOX_REPLICAS] ordered-float min xyz, max xyz */
    GridParams* grid;
    float4* pos4;       /* [S] deposit positions (compact copy of the records' first float4) */
    uint32_t bshift;    /* bucket sort: cells per bucket = 1 << bshift, at most BS_MAXB buckets */
    uint32_t bs_nchunk; /* slot chunks (ceil(S / BS_CHUNK)) */
    uint32_t* bs_table; /* [buckets][chunks] counts, then exclusive offsets */
    uint32_t* bs_partials; /* scan partials + grand total */
    uint2* bs_pairs;    /* [S] (sub-cell key, slot) in bucket order; sub-cell key = cell * SUBX + x slice */
    uint32_t* subofs;   /* [SUBX nsub G + 1] first photon of each sub-cell */
    uint32_t nsub;      /* sub-rows per cell row: 1 (photons in cell order) or SUBR^2 (see k_bs_count) */
    /* stochastic-hash photon map (orx_config.photon_map = 1) */
    uint32_t hash;      /* 1: deposits go to the hash table, D = slot capacity per photon */
    uint32_t Dlim;      /* deposits that end a photon path: D (uniform grid), none (hash: store_photon.h never counts) */
    uint32_t hnum;      /* photonsSize = NUM_PHOTONS = PW * PH * max deposits (OptixRenderer.cpp:50) */
    uint32_t* hcount;   /* [hnum] photonsHashTableCount */
    uint32_t* hwin;     /* [hnum] slot + 1 of the photon the cell keeps (0: empty) */
    /* the photon pass's traversal-stack entries below the LDS part: [block][tdeep][64] for tlanes
     * lanes (StackH: a block's offsets stay small whatever the launch size) */
    uint32_t* tstk;
    uint32_t tlanes, tdeep;
};

/* kd-tree photon map (orx_config.photon_map = 2, orx_kdtree.hip): the implicit
 * balanced tree of OptixRenderer_CPUKdTree.cpp built on the device */
struct KdBufs {
    uint32_t S;          /* photon slots (bound on the valid photons) */
    uint32_t tree_size;  /* m_photonKdTreeSize = pow2roundup(S + 1) - 1 (OptixRenderer.cpp:207) */
    uint32_t levels;     /* log2(tree_size + 1): depth bound of any tree of <= S photons */
    uint32_t ntiles;     /* radix-sort tiles of RS_TILE elements */
    float4* tree;        /* [tree_size]: pos.xyz | axis bits */
    float4* tree_bc;     /* [tree_size][2]: power.xyz | dir.x, dir.y dir.z */
    uint32_t* ids[2][3]; /* [S] radix-sort slot lists (ids[1][0]: valid slots in slot order) */
    float4* lst[2][3];   /* [S] per axis, position order: photon position | slot bits; ping-pong per level */
    uint2* nkey;         /* [tree_size] split nodes: the median's (ordered key on the split axis, slot) */
    uint32_t* keys[2];   /* [S] radix-sort keys */
    uint32_t* nodepos;   /* [S] tree node of each position at the current level (0xffffffff: placed) */
    uint2* seg;          /* [tree_size] segment [start, end) of each node (0xffffffff: not in the tree) */
    float* box;          /* [tree_size][6] bbmin, bbmax handed down by buildKDTree */
    uint32_t* ninfo;     /* [tree_size] split nodes: median << 2 | axis; else 0xffffffff */
    uint32_t* nodeP;     /* [tree_size][3] per list: in-block exclusive (left | median << 16) prefix at the segment start */
    uint32_t* ppart;     /* [6][S/1024] block counts, then their scan */
    uint32_t* table;     /* [256][ntiles] radix digit counts, then their scan */
    uint32_t* tpart;     /* scan partials */
    uint32_t* vpart;     /* [S/1024] valid-slot block counts */
    uint32_t* count;     /* [4]: [0] valid photons n */
};
void launch_kd_build(hipStream_t s, const PhotonBufs& pb, const KdBufs& kd);

/* Stochastic-hash grid of one iteration: initializeStochasticHashPhotonMap
 * (OptixRenderer_SpatialHash.cu:286-302), computed on the host */
struct HashParams {
    float ox, oy, oz;   /* photonsWorldOrigo = scene AABB min - (r + 0.0001) */
    float cell;         /* photonsGridCellSize = r */
    uint32_t gx, gy, gz;
    uint32_t mask;      /* photonsSize - 1 (getHashValue, PhotonGrid.h:30-33) */
};

struct Consts {
    uint32_t max_photon_depth;
    uint32_t max_radiance_depth;
    float ppm_radius;
    float ppm_radius2;
    float emitted_f;    /* emittedPhotonsPerIterationFloat (global count) */
    uint32_t local_iteration;
    uint32_t media;     /* participating medium on: no shadow samples in the direct pass */
};

/* participating medium: the box + volumetric table (VolMap, orx_device.h), the eye pass's
 * per-pixel volumetricRadiance and the photon pass's per-photon last volumetric event */
struct MediaBufs {
    VolMap vm;
    float* volR;   /* [rows*W*3] */
    float4* ev_a;  /* [photons]: last event position, event count bits */
    float4* ev_b;  /* [photons]: its power */
};
/* the volumetric photon table of one photon pass and its grid (orx_media.hip) */
struct VolBuild {
    const float4* ev_a;
    const float4* ev_b;
    uint32_t nphot, D, NV;          /* photons, max deposits (pm_index stride), table slots */
    uint32_t* vcnt;                 /* [NV] numDeposits */
    uint32_t* vwin;                 /* [NV] winning photon + 1 */
    float4* vA;                     /* [NV] position */
    float4* vB;                     /* [NV] power */
    uint32_t* keys;                 /* [NV] cell, G (outside the grid) or G + 1 (empty) */
    uint32_t* vals;                 /* [NV] slot */
    uint32_t* keys_sorted;
    uint32_t* vals_sorted;
    void* sort_tmp;
    size_t sort_tmp_bytes;
    uint32_t* start;                /* [G + 2] */
    float4* rec;                    /* [NV][2] */
};
size_t vol_sort_tmp_bytes(uint32_t NV);
/* clear + resolve + grid + sort + records; vm: the grid parameters (host) */
void launch_vol_build(hipStream_t s, const VolBuild& vb, const VolMap& vm);
/* indirect += volR / emitted (IndirectRadianceEstimation.cu:215-218) */
void launch_vol_indirect(hipStream_t s, const PixelBufs& px, const float* volR, float emitted_f);

/* on-device BVH build (orx_bvh.hip): V float3 [n_vertices], I uint3 [nt] on the
 * device; writes out4 (capacity cap4 nodes) and leaf_order [nt] */
hipError_t device_build_bvh4(hipStream_t s, const float* V, const uint32_t* I, uint32_t nt, int bins, uint32_t leaf_max,
                             float leaf_sah, int treelet_passes, int treelet_leaves, bool sah_collapse, DevBvh4* out4,
                             uint32_t cap4,
                             uint32_t* leaf_order, uint32_t* nodes4, uint32_t* stack_bound, uint32_t* max_depth,
                             bool* ok);
void launch_rng_init(hipStream_t s, RngPlanes rng, uint32_t RW, uint32_t rows, uint32_t rank, uint32_t world,
                     uint32_t seed);
void launch_ppm_eye(hipStream_t s, const DevScene& S, const DevCamera& cam, const PixelBufs& px, const Consts& c,
                    const MediaBufs* mb = nullptr);
/* global (deep) traversal-stack entries per lane of k_ppm_photon / k_vcm_shadow for a tree whose
 * stack bound is `entries` (StackH::deep of their LDS depths) */
uint32_t photon_stack_deep(uint32_t entries);
uint32_t vcm_shadow_stack_deep(uint32_t entries);
bool launch_ppm_photon(hipStream_t s, const DevScene& S, const PixelBufs& px, const PhotonBufs& pb, const Consts& c,
                       const MediaBufs* mb = nullptr);
void launch_grid_setup(hipStream_t s, const PhotonBufs& pb, const GridBox& gb = GridBox{});
/* atomic-free grid build: keys + bucket histogram / scan of the table /
 * bucket placement + per-bucket cells (offsets, permutation) + permute */
void launch_grid_bucket_count(hipStream_t s, const PhotonBufs& pb);
void launch_grid_bucket_scan(hipStream_t s, const PhotonBufs& pb);
void launch_grid_bucket_place(hipStream_t s, const PhotonBufs& pb);
/* slab mode (sharded PPM with a spatial photon partition): nb bins per axis over the scene AABB */
struct SlabBins {
    float lo[3];
    float inv[3]; /* nb / extent */
    uint32_t nb;
};
/* the bin of coordinate v on axis a; one function for histogram, pack and ownership, so the
 * host plan's counts and the ranks' ownership agree exactly */
__device__ __forceinline__ uint32_t slab_bin(const SlabBins& sb, float v, uint32_t a) {
    const int32_t b = orx_f2i_sat(orx_floorf((v - sb.lo[a]) * sb.inv[a]));
    return b < 0 ? 0u : (b >= (int32_t)sb.nb ? sb.nb - 1u : (uint32_t)b);
}
/* gathers `rows` pixel rows whose hitpoints are in hp{A,B,C} against the
 * local photon grid; writes indirect (and debug counters) */
/* Hitpoints to gather: `segments` segments of seg_rows x W pixels, each in the
 * plane layout of PixelBufs (segment k starts at base + k*seg_bytes). */
struct GatherIn {
    const uint8_t* base;
    size_t seg_bytes;
    uint32_t segments, seg_rows, W;
    float* indirect;    /* [segments*seg_rows*W*3] */
    uint32_t* dbg;      /* [segments*seg_rows*W*2] or NULL */
    uint32_t cull;      /* 1: a hit point whose sphere misses the AABB of the grid's photons gathers
                         * nothing (its window would only clamp onto cells without them); 2 (slab
                         * mode): only the hit points this rank owns gather (bin of own_axis in
                         * [own_lo, own_hi] over own_bins), the others get 0 */
    uint32_t own_axis, own_lo, own_hi;
    SlabBins own_sb;
    /* slab mode: the 16x16-pixel tiles that gather here, ascending (tile_list[0..*tile_count)),
     * dealt to the XCDs in contiguous bands; NULL: every tile */
    const uint32_t* tile_list = nullptr;
    const uint32_t* tile_count = nullptr;
    uint32_t order = 0; /* tile order: 0 image bands per XCD, S > 0 super-tiles of S x S tiles (gather_tile) */
    uint32_t raw = 0;   /* 1: the sharded gather's exported hit points (orx_export_hitpoints): planes A pos|flags
                         * float4 and N normal float3, 28 B per pixel, no attenuation; the estimate is left
                         * unattenuated and the owner applies its hit point's attenuation (orx_ppm_finish).
                         * 0: the renderer's own planes (40 B per pixel: A, B normal|atten.x, C atten.yz) */
    uint32_t visits;    /* 1: count the reference's per-pixel visits (IndirectRadianceEstimation.cu:113/124)
                         * into dbg and the stats; 0 for the sharded gather, which has no per-pixel
                         * debug buffers and whose rank-local counts are not the reference's
                         * (measured: per-rank hall gather at N=8 0.89 -> 0.44 ms without them) */
};
/* The gather kernels tile IMAGE rows y.  With several row-interleaved segments (the
 * sharded gather: segment s = rank s holds image rows y = s + lj*segments) the hit points
 * and the indirect output are segment-major, row j = s*seg_rows + lj: tiling j directly
 * would give a wave 8 image rows that are `segments` apart (a union that grows with the
 * rank count); tiling y keeps a wave's pixels neighbours in the image. */
__device__ __forceinline__ uint32_t gather_row(const GatherIn& gi, uint32_t y) {
    if (gi.segments <= 1) return y;
    const uint32_t s = y % gi.segments, lj = y / gi.segments;
    return s * gi.seg_rows + lj;
}
/* The gather's hit point j (row of the segment-major layout), pixel x: position|flags (A),
 * normal|attenuation.x (B) and attenuation.yz (C).  gi.raw: the 28-B export layout, attenuation 1
 * (the owner applies it, orx_ppm_finish) */
/* pixels per plane of the 28-B export layout: padded to a multiple of 4, so every segment's
 * planes stay 16-B aligned (plane A is read as float4) */
__host__ __device__ __forceinline__ size_t hp_export_plane(size_t npx) { return (npx + 3) & ~(size_t)3; }
__device__ __forceinline__ void hp_load(const GatherIn& gi, uint32_t j, uint32_t x, float4& A, float4& B, float2& Cc) {
    const uint32_t seg = j / gi.seg_rows, lj = j - seg * gi.seg_rows;
    const size_t plane = gi.raw ? hp_export_plane((size_t)gi.seg_rows * gi.W) : (size_t)gi.seg_rows * gi.W;
    const uint8_t* b = gi.base + seg * gi.seg_bytes;
    const size_t li = (size_t)lj * gi.W + x;
    A = ((const float4*)b)[li];
    if (gi.raw) {
        const float* n = (const float*)(b + plane * 16) + 3 * li;
        B = make_float4(n[0], n[1], n[2], 1.0f);
        Cc = make_float2(1.0f, 1.0f);
    } else {
        B = ((const float4*)(b + plane * 16))[li];
        Cc = ((const float2*)(b + plane * 32))[li];
    }
}
__device__ __forceinline__ float4 hp_load_a(const GatherIn& gi, uint32_t j, uint32_t x) {
    const uint32_t seg = j / gi.seg_rows, lj = j - seg * gi.seg_rows;
    return ((const float4*)(gi.base + seg * gi.seg_bytes))[(size_t)lj * gi.W + x];
}

/* 8x8-pixel wave tiles; the wave-union kernel, or the per-lane kernel for gathers of >= 8 segments */
void launch_ppm_gather(hipStream_t s, const GatherIn& gi, const PhotonBufs& pb, const Consts& c);
/* slab mode: flags[tile] / the ascending list of the tiles with a hit point that gathers here
 * (the others' indirect is zeroed here); ntiles of the gather's 16x16 tiling */
void launch_export_hp(hipStream_t s, const PixelBufs& px, uint32_t n, float* dst);
void launch_indirect_atten(hipStream_t s, const PixelBufs& px, uint32_t n, const float* in);
void launch_gather_tiles(hipStream_t s, const GatherIn& gi, const PhotonBufs& pb, const Consts& c, uint8_t* flags,
                         uint32_t* list, uint32_t* count);
constexpr uint32_t SLAB_VOX = 32; /* coarse voxels per axis of the slab histogram (include/orx.h) */
void launch_slab_hist(hipStream_t s, const PhotonBufs& pb, const PixelBufs& px, const SlabBins& sb,
                      const SlabBins& vb, uint32_t* hist);
void launch_slab_pack(hipStream_t s, const PhotonBufs& pb, const SlabBins& sb, uint32_t axis, uint32_t halo,
                      const uint8_t* bin_dest, uint32_t world, uint32_t* cursor, uint32_t cap, float* send);
void launch_slab_import(hipStream_t s, const PhotonBufs& pb, const float* recv, uint32_t n);
/* the own photon pass's AABB (folded bbox replicas, ordered-int bits) -> out[6] */
void launch_slab_bbox(hipStream_t s, const PhotonBufs& pb, uint32_t* out);
void launch_hash_build(hipStream_t s, const PhotonBufs& pb, const HashParams& hp);
void launch_ppm_gather_hash(hipStream_t s, const GatherIn& gi, const PhotonBufs& pb, const HashParams& hp,
                            const Consts& c);
void launch_ppm_gather_kd(hipStream_t s, const GatherIn& gi, const PhotonBufs& pb, const KdBufs& kd, const Consts& c);
/* mode 0: direct + output; 1: direct only; 2: output only */
void launch_ppm_direct_output(hipStream_t s, const DevScene& S, const PixelBufs& px, const Consts& c, int mode = 0);
void launch_pt(hipStream_t s, const DevScene& S, const DevCamera& cam, const PixelBufs& px, const Consts& c);

/* ---- VCM (orx_vcm.hip) ---- */
constexpr uint32_t VCM_MAX_VERTS = 9; /* VCM_MAX_PATH_LENGTH - 1 (OptixRenderer.cpp:343-344) */
/* camera pass shadow-ray queue per wave, in float4: [64 lanes x (1 + 9) tests][2] + [64] points */
constexpr uint32_t VCM_SHQ_PER_WAVE = 2 * 64 * (VCM_MAX_VERTS + 1) + 64;
constexpr uint32_t VCM_END = 0xffffffffu;     /* end of a pixel's deferred-entry list */
/* light subpath p = x + y*W pairs with pixel p; RNG slot y*RW + x serves both */
struct VcmBufs {
    uint32_t RW;
    RngPlanes rng;
    uint32_t* vcount;   /* [W*H] stored vertices per light subpath */
    float4* vA;         /* [9][W*H] pos.xyz | material id bits */
    float4* vB;         /* [9][W*H] throughput.xyz | dVCM */
    float4* vC;         /* [9][W*H] normal.xyz | dVC */
    float4* vD;         /* [9][W*H] localDirFix.xyz | dVM */
    float4* vE;         /* [9][lcount] texel colour of Texture vertices (NULL without Texture materials) */
    float4* shq;        /* [max(camera-, light-pass waves)][VCM_SHQ_PER_WAVE] deferred shadow-ray queues */
    float* splat;       /* [world][max_rows][W][3] connectCameraT1 accumulation of this iteration (owner-block layout) */
    const float* splat_in; /* [rows][W][3] summed splats of the own rows (camera pass) */
    float* cam;         /* [W*H*3] camera subpath colour of this iteration */
    float* output;      /* [W*H*3] running sum */
    uint32_t* work;     /* [2] camera-pass, light-pass work-item counters (zeroed by the launches) */
    /* the camera pass's connection shadow rays, deferred to k_vcm_shadow (launch_vcm_camera): one entry
     * per connection in creation order, each pixel's entries linked in the order the reference adds them */
    float4* dq0;        /* [dcap] connection point xyz | distance */
    float4* dq1;        /* [dcap] direction xyz | next entry of the pixel (uint bits, VCM_END) */
    float4* dq2;        /* [dcap] unoccluded contribution xyz | unused */
    uint8_t* docc;      /* [dcap] 1: occluded (k_vcm_shadow) */
    uint32_t* dhead;    /* [lcount] the pixel's first entry, or VCM_END */
    float4* demis;      /* [lcount] the emitter contribution ending the subpath xyz | 1 if there is one */
    uint32_t* dctl;     /* [4] entries written, overflow flag (more entries than dcap: the resolve reruns in place) */
    uint32_t dcap;
    /* the RNG words each camera subpath starts from, stored by the walk (k_vcm_camera<., 1>) as it loads
     * them: the in-place rerun after an overflow starts its subpaths from here */
    RngPlanes rsave;
    uint32_t* shstk;    /* k_vcm_shadow's traversal-stack entries below its LDS part: [block][shdeep][64] */
    uint32_t shstk_lanes, shdeep;
    struct VcmConsts* consts; /* device copy of the pass constants (written by the launches) */
    /* this iteration's constants as the resolve's rerun reads them: the next iteration's launches
     * rewrite `consts` while the resolve runs beside them (one copy per entry-list set) */
    struct VcmConsts* consts_keep;
    float4* shq_rerun;  /* the rerun's shadow-ray queues (it runs beside the light pass and walk using shq) */
    uint32_t splat_n;   /* floats in `splat` (the light-image bound of k_vcm_light_shadow's splats) */
    /* the light pass's camera connections (connectCameraT1), deferred to k_vcm_light_shadow with the
     * camera pass's resolve (the overlapped single-device schedule; NULL: traced in the light pass).
     * A wave whose queue does not fit traces it in place, as without the list. */
    float4* lcq = nullptr;  /* [lcap][3] queue entries (LightShadowRays' layout) */
    uint32_t* lctl = nullptr; /* [2] entries written, entries dropped to in-place tracing */
    uint32_t lcap = 0;
};
struct VcmConsts {
    f3 eye, lookdir, u, v;          /* Camera (Camera.cpp:333-345) */
    f3 unitU, unitV, lookdirN;
    float lookdirLen, ipsx, ipsy;   /* imagePlaneSize = 2*(ulen, vlen) */
    float psfx, psfy;               /* pixelSizeFactor (OptixRenderer.cpp:846) */
    float misVc, misVm;             /* 1/etaVCM, 0 (vcmUseVM = false) */
    uint32_t W, H, count;           /* count = lightSubpathCount = W*H (global) */
    uint32_t rank, world, rows, max_rows, lcount; /* own rows y = rank + j*world; lcount = rows*W */
    uint32_t maxPathLen;
};
void launch_vcm_light(hipStream_t s, const DevScene& S, const VcmBufs& vb, const VcmConsts& c, bool estimate);
void launch_vcm_camera(hipStream_t s, const DevScene& S, const VcmBufs& vb, const VcmConsts& c);
/* its parts, in this order: the walk (RNG, light vertices, constants, entry lists), the resolve (deferred
 * shadow rays, colours, and the in-place rerun should the entry list have overflowed) */
void launch_vcm_camera_walk(hipStream_t s, const DevScene& S, const VcmBufs& vb, const VcmConsts& c);
void launch_vcm_camera_resolve(hipStream_t s, const DevScene& S, const VcmBufs& vb, const VcmConsts& c);
uint32_t vcm_camera_waves(uint32_t tiles); /* persistent camera-pass waves for `tiles` 8x8 tiles */
uint32_t vcm_light_waves(uint32_t items);  /* persistent light-pass waves for `items` 64-subpath items */

}  // namespace orx
