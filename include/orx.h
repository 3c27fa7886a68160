/*
 * orx.h — C ABI of the MI355X-native render core (liborx.so).
 *
 * This is the drop-in boundary for ico-eagleye/OppositeRenderer's
 * `OptixRenderer` (RenderEngine/renderer/OptixRenderer.h:21-43) and the
 * parts of `IScene` (RenderEngine/scene/IScene.h:16-29) that the renderer
 * consumes.  Plain pointers and sizes only; no C++ or torch types cross it.
 * Errors never throw: every call returns an orx_status and the message of
 * the last failure is kept per renderer (orx_last_error), replacing the
 * reference's std::exception(const char*) (OptixRenderer.cpp:816-820).
 *
 * Reference entry point -> orx call
 *   OptixRenderer::OptixRenderer() + initialize(ComputeDevice)
 *       (OptixRenderer.cpp:81-104, :113-400)              -> orx_create
 *   OptixRenderer::initScene(IScene&) (:436-485)          -> orx_init_scene
 *   OptixRenderer::renderNextIteration(...) (:507-821)    -> orx_render_next_iteration
 *   OptixRenderer::getOutputBuffer(void*) (:860-865)      -> orx_get_output
 *   getWidth/getHeight/getScreenBufferSizeBytes (:850-870)-> orx_width/orx_height/orx_output_bytes
 *   OptixRenderer::EMITTED_PHOTONS_PER_ITERATION (.h:43)  -> orx_emitted_photons_per_iteration
 *   ~OptixRenderer() (:106-111)                           -> orx_destroy
 */
#ifndef ORX_H
#define ORX_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define ORX_ABI_VERSION 1u

typedef struct orx_renderer orx_renderer;

typedef enum {
    ORX_OK = 0,
    ORX_ERR_INVALID_ARGUMENT = 1,
    ORX_ERR_STATE = 2,          /* e.g. initScene before initialize, render before initScene */
    ORX_ERR_DEVICE = 3,         /* HIP runtime failure */
    ORX_ERR_NO_LIGHTS = 4,      /* "No lights exists in this scene." (OptixRenderer.cpp:444-447) */
    ORX_ERR_GRID_TOO_LARGE = 5, /* "Too many cells in SpatialHash.cu" (OptixRenderer_SpatialHash.cu:243-247) */
    ORX_ERR_OUT_OF_MEMORY = 6,
    ORX_ERR_UNSUPPORTED = 7
} orx_status;

/* RenderMethod::E order (RenderEngine/renderer/RenderMethod.h:13-19). */
typedef enum {
    ORX_METHOD_PATH_TRACING = 0,
    ORX_METHOD_VCM_BIDIRECTIONAL_PATH_TRACING = 1,
    ORX_METHOD_PROGRESSIVE_PHOTON_MAPPING = 2
} orx_method;

/* Camera inputs (Camera.h:72-79).  The engine derives lookdir / camera_u /
 * camera_v exactly as Camera::setup (Camera.cpp:333-345). */
typedef struct {
    float eye[3];
    float lookat[3];
    float up[3];
    float hfov;     /* degrees */
    float vfov;     /* degrees */
    float aperture; /* > 0 enables thin-lens depth of field (helpers/camera.h:11-27) */
} orx_camera;

/* RenderServerRenderRequestDetails (clientserver/RenderServerRenderRequestDetails.h:15-33). */
typedef struct {
    orx_camera camera;
    int32_t method;  /* orx_method */
    uint32_t width;
    uint32_t height;
    double ppm_alpha;
} orx_request;

/* Material classes of RenderEngine/material (one per .cpp). */
typedef enum {
    ORX_MAT_DIFFUSE = 0,         /* Diffuse(Kd)                           Diffuse.cpp:17-20  */
    ORX_MAT_DIFFUSE_EMITTER = 1, /* DiffuseEmitter(power, Kd)+inverseArea DiffuseEmitter.cpp:17-25 */
    ORX_MAT_MIRROR = 2,          /* Mirror(Kr)                            Mirror.cpp:17-20   */
    ORX_MAT_GLASS = 3,           /* Glass(ior, Kr, Kt)                    Glass.cpp:17-22    */
    ORX_MAT_GLOSSY = 4,          /* Glossy(Kd, Ks, exponent)              Glossy.cpp:16-33   */
    ORX_MAT_TEXTURE = 5          /* Texture(diffuse map [, normal map])   Texture.cpp:18-29  */
} orx_material_type;

typedef struct {
    int32_t type;        /* orx_material_type */
    float Kd[3];         /* diffuse albedo (Diffuse, Glossy, DiffuseEmitter) */
    float Ks[3];         /* Glossy specular */
    float Kr[3];         /* Mirror / Glass reflectance */
    float Kt[3];         /* Glass transmittance */
    float ior;           /* Glass index of refraction */
    float exponent;      /* Glossy Phong exponent */
    float power[3];      /* DiffuseEmitter power (scaled by Kd inside the engine, as the ctor does) */
    float inverse_area;  /* DiffuseEmitter 1/area of the emitting quad */
    int32_t texture;     /* Texture: index into orx_scene.textures */
} orx_material;

/* Texture images (util/Image.cpp): RGBA8 rows, row 0 first, sampled as
 * rtTextureSampler<uchar4, 2, cudaReadModeNormalizedFloat> with bilinear
 * filtering, wrap addressing and normalised coordinates (Texture.cpp:109-122). */
typedef struct {
    uint32_t width, height;
    const uint8_t* rgba;          /* width * height * 4: diffuseSampler */
    uint32_t normal_width, normal_height;
    const uint8_t* normal_rgba;   /* normalMapSampler, or NULL (hasNormals = 0) */
} orx_texture;

/* Light::LightType (renderer/Light.h:14-54). */
typedef enum { ORX_LIGHT_AREA = 0, ORX_LIGHT_POINT = 1, ORX_LIGHT_SPOT = 2 } orx_light_type;

typedef struct {
    int32_t type;        /* orx_light_type */
    float power[3];
    float position[3];   /* area: anchor */
    float v1[3];         /* area: edge 1 */
    float v2[3];         /* area: edge 2 */
    float direction[3];  /* spot */
    float angle;         /* spot, degrees */
} orx_light;

/* Flattened scene (replaces IScene::getSceneRootGroup's OptiX node graph).
 * Deep-copied by orx_init_scene.  Primitive order defines the tie-break of
 * equal-distance hits (lowest global primitive id wins): quads first, then
 * spheres, then triangles. */
typedef struct {
    uint32_t n_quads;
    const float* quads;              /* n_quads * 9: anchor, offset1, offset2 (Cornell.cpp:33-64) */
    const uint32_t* quad_material;   /* n_quads */
    uint32_t n_spheres;
    const float* spheres;            /* n_spheres * 4: center xyz, radius (Sphere.cu) */
    const uint32_t* sphere_material; /* n_spheres */
    uint32_t n_vertices;
    const float* vertices;           /* n_vertices * 3 */
    const float* normals;            /* n_vertices * 3 or NULL (TriangleMesh.cu:56-59) */
    uint32_t n_triangles;
    const uint32_t* triangles;       /* n_triangles * 3 vertex indices */
    const uint32_t* triangle_material;
    uint32_t n_materials;
    const orx_material* materials;
    uint32_t n_lights;
    const orx_light* lights;         /* IScene::getSceneLights */
    float aabb_min[3];               /* IScene::getSceneAABB */
    float aabb_max[3];
    /* TriangleMesh.cu attribute buffers (Scene.cpp:395-440) */
    const float* texcoords;          /* n_vertices * 2 or NULL (textureCoordinate = 0) */
    const float* tangents;           /* n_vertices * 3 or NULL; with bitangents: hasTangentsAndBitangents */
    const float* bitangents;         /* n_vertices * 3 or NULL */
    uint32_t n_textures;
    const orx_texture* textures;
    /* participating media (AABInstance + ParticipatingMedium(sigma_s, sigma_a), Scene.cpp:337-350):
     * at most one axis-aligned box; used when orx_config.enable_media is set */
    uint32_t n_media;
    const float* media;              /* n_media * 8: box min xyz, box max xyz, sigma_s, sigma_a */
} orx_scene;

/* Compile-time constants of config.h / OptixRenderer.cpp:38-61 as runtime config. */
typedef struct {
    uint32_t photon_launch_width;     /* PHOTON_LAUNCH_WIDTH  = 1024 */
    uint32_t photon_launch_height;    /* PHOTON_LAUNCH_HEIGHT = 1024 */
    uint32_t max_photon_deposits;     /* MAX_PHOTONS_DEPOSITS_PER_EMITTED = 4 */
    uint32_t photon_grid_max_size;    /* PHOTON_GRID_MAX_SIZE = 100*100*100 */
    uint32_t max_photon_trace_depth;  /* MAX_PHOTON_TRACE_DEPTH = 7 */
    uint32_t max_radiance_trace_depth;/* MAX_RADIANCE_TRACE_DEPTH = 9 */
    uint32_t vcm_max_path_length;     /* VCM_MAX_PATH_LENGTH = 10 */
    uint32_t seed;                    /* 0: 574133*clock()+47844152748*time() like SpatialHash.cu:322; else DEBUG_RANDOM_SEED */
    uint32_t debug_counters;          /* 1: keep per-pixel cells/photons visited (OptixRenderer.cpp:872-953) */
    uint32_t gather_variant;          /* photon-grid layout for the gather: 2 photons ordered by cell-row
                                         quarter sub-rows (y and z halves) and x quarters; 1 photons in cell
                                         order with x quarters only; 0 (default) the faster of the two for the
                                         renderer: sub-rows on a single device, cell order for a shard of
                                         world >= 2 (orx_set_shard: it holds 1/N of the photons, so the
                                         per-sub-row work outweighs the photons it trims).  The image does not
                                         depend on it.  Any other value: ORX_ERR_INVALID_ARGUMENT */
    uint32_t photon_map;              /* ACCELERATION_STRUCTURE (config.h): 0 uniform grid (the shipped
                                         configuration), 1 stochastic hash (OptixRenderer_SpatialHash.cu:286-302,
                                         store_photon.h, IndirectRadianceEstimation.cu:131-162; needs
                                         PW*PH*max deposits a power of two, one rank, trace depth <= 9),
                                         2 kd-tree (ACCELERATION_STRUCTURE_KD_TREE_CPU:
                                         OptixRenderer_CPUKdTree.cpp, IndirectRadianceEstimation.cu:164-209;
                                         built on the device here) */
    uint32_t enable_media;            /* ENABLE_PARTICIPATING_MEDIA (config.h:29): the scene's medium box
                                         (orx_scene.media) scatters photons and eye rays gather its volumetric
                                         photons (ParticipatingMedium.cu, VolumetricPhotonSphere*.cu); the PPM
                                         direct pass takes no shadow samples (DirectRadianceEstimation.cu:54).
                                         All of this applies only when the scene has a medium box: with
                                         enable_media set and orx_scene.n_media == 0 the renderer runs exactly
                                         as with enable_media = 0 (the direct pass keeps its 4 shadow samples,
                                         unlike a reference build with the macro on).  PPM on one device only
                                         (other methods / world > 1: ORX_ERR_UNSUPPORTED) */
    uint32_t volumetric_photons;      /* NUM_VOLUMETRIC_PHOTONS = 200000 (config.h:35): volumetric photon table */
    uint32_t reserved[3];
} orx_config;

void orx_default_config(orx_config* cfg);

orx_status orx_create(int hip_device, const orx_config* cfg, orx_renderer** out);
orx_status orx_init_scene(orx_renderer* r, const orx_scene* scene);
orx_status orx_render_next_iteration(orx_renderer* r, uint64_t iteration_number,
                                     uint64_t local_iteration_number, float ppm_radius,
                                     int create_output, const orx_request* details);
/* W*H*3 floats into caller-owned host memory; SUM over local iterations. */
orx_status orx_get_output(orx_renderer* r, float* dst, size_t dst_bytes);
/* Same, device-to-device into caller-owned device memory on the renderer's
 * device (used by the multi-GPU harness to hand the buffer to RCCL). */
orx_status orx_get_output_device(orx_renderer* r, void* dst_device, size_t dst_bytes);
uint32_t orx_width(const orx_renderer* r);
uint32_t orx_height(const orx_renderer* r);
size_t orx_output_bytes(const orx_renderer* r);
uint32_t orx_emitted_photons_per_iteration(const orx_renderer* r);
const char* orx_last_error(const orx_renderer* r);
void orx_destroy(orx_renderer* r);

/* ---- inspection (parity tests, profiling; not part of the reference API) ---- */
/* test hook: pretend the photon pass's deep-stack buffer covers only `lanes` lanes (bookkeeping only;
 * the next resize or initScene sizes it again), so that the next PPM photon pass must return
 * ORX_ERR_STATE instead of launching past the buffer (OptixRenderer.cpp:816-820 throws) */
orx_status orx_debug_limit_photon_stack(orx_renderer* r, uint32_t lanes);
/* test hook: rerun the last VCM iteration's resolve (deferred shadow rays, colours) with stale list
 * state -- entry count past the capacity, odd pixels' list heads past the entries, light-connection
 * entries whose pixel offsets lie past the light image -- which the resolve's device-side bounds must
 * absorb; synchronous, colours in ORX_BUF_VCM_CAMERA (the output is accumulated once more) */
orx_status orx_debug_vcm_stale_resolve(orx_renderer* r);
typedef enum {
    ORX_BUF_RNG = 0,        /* uint32 [slots][6]: xorwow v0..v4, d */
    ORX_BUF_HITPOINTS = 1,  /* float  [W*H][13]: pos3 normal3 atten3 radiance3 flags(bits) */
    ORX_BUF_PHOTONS = 2,    /* float  [S][9] grid-sorted photons: power3 position3 direction3 (valid prefix);
                               stochastic hash: [photonsSize][9] the photon each table entry holds (0 if empty) */
    ORX_BUF_GRID_OFFSETS = 3,/* uint32 [G+1]; stochastic hash: [photonsSize] photonsHashTableCount */
    ORX_BUF_INDIRECT = 4,   /* float  [W*H][3] */
    ORX_BUF_DIRECT = 5,     /* float  [W*H][3] */
    ORX_BUF_OUTPUT = 6,     /* float  [W*H][3] */
    ORX_BUF_PHOTON_SLOTS = 7,/* float [S][9] unsorted photon slots: power3 position3 direction3 (0 when cleared) */
    ORX_BUF_DEBUG_VISITED = 8,/* uint32 [W*H][2]: cells visited, photons visited */
    /* VCM (vcm/VCMLightPass.cu, VCMCameraPass.cu); light subpath p = x + y*W pairs with pixel p */
    ORX_BUF_VCM_VERTEX_COUNT = 9, /* uint32 [W*H]: stored light vertices per subpath (lightSubpathVertexCountBuffer) */
    ORX_BUF_VCM_VERTICES = 10,    /* float [9][W*H][16]: per vertex slot k, subpath p: pos3 mat(bits) throughput3 dVCM
                                     normal3 dVC dirFix3 dVM; entries k >= count[p] are stale */
    ORX_BUF_VCM_SPLAT = 11,       /* float [W*H][3]: this iteration's light-tracing splats (connectCameraT1) */
    ORX_BUF_VCM_CAMERA = 12,      /* float [W*H][3]: this iteration's camera subpath colour (cameraPrd.color) */
    /* kd-tree photon map (photon_map = 2): the implicit tree m_photonKdTree of pow2roundup(S + 1) - 1 nodes,
       node i's children at 2i+1, 2i+2; per node power3 position3 direction3 axis(uint32 bits: PPM_X 1, PPM_Y 2,
       PPM_Z 4, PPM_LEAF 8, PPM_NULL 16, config.h:12-16).  Only nodes reachable from the root are defined (the
       reference never clears the buffer; a NULL node defines axis and power only). */
    ORX_BUF_KD_TREE = 13,
    /* participating medium (orx_config.enable_media) */
    ORX_BUF_VOLUMETRIC = 14,        /* float [W*H][3]: the last eye pass's Hitpoint::volumetricRadiance */
    ORX_BUF_VOLUMETRIC_PHOTONS = 15 /* float [volumetric_photons][7]: the last photon pass's volumetric photon
                                       table, power3 position3 numDeposits(uint32 bits); 0 when empty */
} orx_buffer_id;
/* Copies buffer `id` to host; returns the byte size through *out_bytes
 * (call with dst=NULL to query). */
orx_status orx_read_buffer(orx_renderer* r, int32_t id, void* dst, size_t dst_bytes, size_t* out_bytes);

/* Passes timed with HIP events on the renderer's stream. */
typedef enum {
    ORX_PASS_PPM_EYE = 0,      /* PPM_RAYTRACE_PASS */
    ORX_PASS_PPM_PHOTON = 1,   /* PPM_PHOTON_PASS (+ fused photon AABB) */
    ORX_PASS_GRID_HASH = 2,    /* grid setup + calculateHashCellsKernel + histogram */
    ORX_PASS_GRID_SCAN = 3,    /* exclusive scan -> hashmapOffsetTable */
    ORX_PASS_GRID_SCATTER = 4, /* sort_by_key as counting-sort scatter */
    ORX_PASS_PPM_GATHER = 5,   /* PPM_INDIRECT_RADIANCE_ESTIMATION_PASS */
    ORX_PASS_PPM_DIRECT = 6,   /* PPM_DIRECT_RADIANCE_ESTIMATION_PASS + PPM_OUTPUT_PASS */
    ORX_PASS_PT = 7,           /* PT_RAYTRACE_PASS */
    ORX_PASS_VCM_LIGHT = 8,    /* VCM_LIGHT_PASS */
    ORX_PASS_VCM_CAMERA = 9,   /* VCM_CAMERA_PASS: the camera subpaths and their connections */
    ORX_PASS_VCM_SHADOW = 10,  /* VCM_CAMERA_PASS, second half: the connections' deferred shadow rays and colours */
    ORX_PASS_COUNT = 11
} orx_pass;

typedef struct {
    uint32_t grid_size[3];
    float cell_size;
    float world_origin[3];
    uint32_t valid_photons;      /* photons in the grid (offset[G]) of the last iteration */
    uint32_t num_cells;
    uint64_t photons_visited;    /* gather: photons visited, last iteration (debug counters) */
    uint64_t cells_visited;      /* gather: (y,z) cell rows visited, last iteration */
    uint64_t photons_visited_total; /* summed since orx_reset_timing */
    uint64_t cells_visited_total;
    uint64_t valid_photons_total;
    uint32_t vcm_shadow_rays;     /* VCM: connection shadow rays the last camera pass deferred (launch_vcm_camera) */
    uint32_t vcm_shadow_overflow; /* VCM: 1 if they exceeded the entry list and the pass reran in place */
    uint32_t timed_iterations;   /* iterations since orx_reset_timing */
    uint32_t bvh_stack_entries;  /* LDS traversal stack depth bound of the scene's BVH4 */
    float pass_ms[16];           /* device time per orx_pass summed since orx_reset_timing */
    uint32_t vcm_light_connections; /* VCM: the last light pass's camera connections deferred to the resolve */
    uint32_t vcm_light_inplace;     /* VCM: of its connections, those traced in the light pass (list full) */
} orx_stats;
orx_status orx_get_stats(orx_renderer* r, orx_stats* out);
/* starts a new timed region for orx_get_stats' *_total and pass_ms fields */
orx_status orx_reset_timing(orx_renderer* r);
/* 1 if the last iteration ran pipelined: PPM, its gather and output pass (ORX_PASS_PPM_GATHER and the
 * output half of ORX_PASS_PPM_DIRECT) on a second stream beside the next iteration's eye, photon and
 * grid passes; VCM, its deferred shadow rays and colours (ORX_PASS_VCM_SHADOW) beside the next
 * iteration's light pass and camera subpaths; so those pass_ms are overlapped wall time; 0 otherwise */
int orx_ppm_pipelined(const orx_renderer* r);
/* The single-device pipelined PPM schedule's grid build (uniform grid): 0 on the renderer's stream before
 * the next photon pass, 1 on a stream of its own beside it, -1 not chosen yet.  By default (ORX_GRID_ASYNC
 * unset) the renderer chooses after the first pipelined iterations following a resize: the first is timed
 * (its photon pass + grid build, and its gather, which the next photon pass then waits for), and the
 * asynchronous build is taken when photon + grid exceed 1.15x the gather; ORX_GRID_ASYNC=0 / 1 fixes it.
 * probe_ms (optional, 2 floats): the measured photon + grid and gather times (ms; 0 when not measured).
 * No reference counterpart (OptiX schedules its own launches); images are identical either way. */
int orx_ppm_grid_schedule(const orx_renderer* r, float* probe_ms);
/* Single-device PPM iteration pipelining and VCM shadow-ray overlap: 1 on, 0 off (serial passes), -1
 * the ORX_PIPELINE environment default (on).  Takes effect at the next iteration (an outstanding pipelined
 * iteration is finished first); images are identical either way. */
orx_status orx_set_iteration_pipelining(orx_renderer* r, int mode);

/* ---- Multi-GPU sharding ----
 * Rank `rank` of `world` owns every RNG-slot row y with y % world == rank:
 * its pixel rows and its photon-launch rows (photon thread (x,y) aliases RNG
 * slot (x,y), OptixRenderer_SpatialHash.cu:310-334), so RNG states never
 * leave their GPU.  cfg.photon_launch_height is the GLOBAL launch height.
 * One PPM iteration of a sharded renderer is driven by the caller:
 *   orx_ppm_local_passes      eye pass (own pixel rows), photon pass (own rows), photon grid (own photons)
 *   orx_export_hitpoints      own hitpoints -> caller buffer (orx_hitpoint_export_bytes)
 *   (caller all-gathers the export buffers of all ranks, rank-major)
 *   orx_ppm_gather_external   gather every rank's hitpoints against the own grid -> partial indirect
 *   (caller reduce-scatters (sum) the partial indirect buffers, rank-major blocks)
 *   orx_ppm_finish            direct pass + output accumulation on own rows
 * The sum over ranks of the partial gathers equals the single-GPU gather up
 * to fp32 summation order (the gather is linear in the photon set and its
 * normalisation uses the global emitted count).  orx_render_next_iteration
 * is the world == 1 composition of the same phases.  With world > 1,
 * orx_get_output returns only the rank's own rows (local row j = global
 * row rank + j*world). */
orx_status orx_set_shard(orx_renderer* r, uint32_t rank, uint32_t world);
/* hipStream_t the renderer launches on (as void*). */
void* orx_stream(orx_renderer* r);
/* use_external != 0: launch everything on the caller's hipStream_t `hip_stream`
 * (NULL = the legacy default stream), e.g. torch's current stream, so kernels
 * and the caller's collectives are ordered; use_external == 0: own stream. */
orx_status orx_set_stream(orx_renderer* r, void* hip_stream, int use_external);
/* rows owned by this rank for the current resolution, and ceil(H/world) */
uint32_t orx_local_rows(const orx_renderer* r);
uint32_t orx_max_local_rows(const orx_renderer* r);
/* P * 28 with P = max_local_rows * W rounded up to a multiple of 4: plane A (position | flags bits,
 * float4) then plane N (the normal of a non-specular hit, the radiance of another, float3), P
 * pixels each (the padding keeps every segment of an all-gathered buffer 16-B aligned).  The
 * attenuation stays with the owner: orx_ppm_gather_external returns the unattenuated estimate
 * (sum of weighted photon powers / (pi r^2 emitted)) and orx_ppm_finish multiplies the summed own
 * rows by their hit points' attenuation (IndirectRadianceEstimation.cu:220; fp32 order differs) */
size_t orx_hitpoint_export_bytes(const orx_renderer* r);
orx_status orx_ppm_local_passes(orx_renderer* r, uint64_t iteration_number, uint64_t local_iteration_number,
                                float ppm_radius, const orx_request* details);
/* the two halves of orx_ppm_local_passes, so that the hitpoint all-gather can
 * overlap the photon pass: eye pass only / photon pass + grid only */
orx_status orx_ppm_local_eye(orx_renderer* r, uint64_t iteration_number, uint64_t local_iteration_number,
                             float ppm_radius, const orx_request* details);
orx_status orx_ppm_local_photons(orx_renderer* r);
orx_status orx_export_hitpoints(orx_renderer* r, void* dst_device, size_t dst_bytes);
/* hitpoints_device: `segments` export buffers back to back; indirect_device:
 * segments * max_local_rows * W * 3 floats */
orx_status orx_ppm_gather_external(orx_renderer* r, const void* hitpoints_device, uint32_t segments,
                                   void* indirect_device, size_t indirect_bytes);
/* indirect_device: max_local_rows * W * 3 floats for the own rows: the summed unattenuated
 * estimates (times each own hit point's attenuation here) */
orx_status orx_ppm_finish(orx_renderer* r, const void* indirect_device, size_t indirect_bytes);
/* orx_ppm_finish on `stream` (a hipStream_t; NULL: as orx_ppm_finish).  Pipelined (orx_set_ppm_pipeline), the
 * finish of iteration i may be issued after iteration i+1's orx_ppm_local_eye -- behind i+1's hit-point
 * all-gather, so that the reduce-scatter of i does not hold that all-gather back on RCCL's in-order stream --
 * and then finishes i (its pixel buffers and constants are held for it); at most one such finish may be
 * outstanding when the next eye pass is issued (ORX_ERR_STATE otherwise) */
orx_status orx_ppm_finish_on(orx_renderer* r, const void* indirect_device, size_t indirect_bytes, void* stream);
/* Pipelined sharded PPM (uniform grid or kd-tree: the hash is single-device, and pipelines on
 * its own without this call; call before the first iteration, like orx_set_shard):
 * orx_ppm_gather_external and orx_ppm_finish of iteration i run on `side_stream` (a hipStream_t
 * of the caller's, who also issues the indirect reduce-scatter there), overlapping iteration
 * i+1's eye, photon and grid passes on the renderer's stream; the direct pass runs on an internal
 * stream right after the photon pass.  Two buffer sets alternate, events order the RNG chain and
 * buffer reuse; the caller makes `side_stream` wait for the hitpoint all-gather before the
 * gather.  enable = 0 restores the serial phases. */
orx_status orx_set_ppm_pipeline(orx_renderer* r, void* side_stream, int enable);

/* Spatial photon partition of the sharded gather ("slab mode", uniform grid only; call before the
 * first iteration, like orx_set_shard).  Rank g owns a slab of bins of one axis of the scene AABB:
 * it receives the photons of ALL ranks in its slab plus those within halo_bins bins of it, and
 * gathers exactly the non-specular hit points whose position lies in its slab, so every hit point
 * is gathered once, with its complete window, and the gather's per-pixel work divides by N (the
 * row partition above gathers all W*H hit points on every rank).  One PPM iteration:
 *   orx_ppm_local_eye + orx_ppm_local_photon_trace   (or orx_ppm_local_trace: both)  eye pass,
 *                            photon pass of the own rows; no grid yet
 *   orx_ppm_slab_histogram   per-bin counts [2][3][nbins] (uint32): the own valid deposits and the
 *                            own non-specular hit points, per axis, nbins bins over the scene AABB
 *                            (nbins a multiple of ORX_SLAB_VOXELS, at most 1024); then 6 words: the
 *                            AABB of the own deposits as order-preserving integers (f >= 0:
 *                            bits | 2^31, f < 0: ~bits; empty: lo 0xffffffff, hi 0); then
 *                            [2][V^3] counts of both over V = ORX_SLAB_VOXELS voxels per axis of
 *                            the scene AABB (x + V (y + V z)): orx_slab_histogram_words(nbins) words
 *   (caller all-gathers the histograms and plans on the host: one axis and a bin -> rank table, the
 *    same on every rank; photons from rank s to rank d = the sum of s's photon bins mapped to d)
 *   orx_ppm_slab_pack        the own valid deposits, rank-major into the caller's send buffer: a
 *                            photon in bin b goes to every rank from bin_dest[b - halo_bins] to
 *                            bin_dest[b + halo_bins] (clamped; bin_dest ascending), at dest_base[d] + k
 *                            for the k-th photon sent to d (9 floats each: position, direction,
 *                            power); host arrays bin_dest[nbins], dest_base[world].  halo_bins >=
 *                            floor(r / bin width) + 2 makes every photon within r of a hit point
 *                            reach the hit point's owner
 *   (caller all-to-alls the photon records)
 *   orx_ppm_slab_import      the received records become this rank's photon set; grid build over
 *                            photon_box (host, 6 words as above: the min/max over ranks of the
 *                            histograms' AABBs, so every rank's grid has the single-device grid's
 *                            origin and cell size; NULL: the AABB of the imported photons); the
 *                            rank owns the hit points whose bin on `axis` lies in [own_lo, own_hi]
 *                            (own_lo > own_hi: none)
 *   orx_export_hitpoints / orx_ppm_gather_external / orx_ppm_finish as above (the gather skips hit
 *   points whose sphere misses this rank's photon grid)
 * Each hit point's indirect comes whole from its owner (the others write 0), so the reduce-scatter
 * sum is the single-GPU gather of that pixel up to fp32 order inside its window.  Capacity: the
 * import takes up to the global photon launch's deposit slots (PW * PH * max deposits) per rank. */
#define ORX_SLAB_VOXELS 32u
/* 6 nbins + 6 + 2 ORX_SLAB_VOXELS^3 */
size_t orx_slab_histogram_words(uint32_t nbins);
orx_status orx_set_slab_partition(orx_renderer* r, int enable);
orx_status orx_ppm_local_trace(orx_renderer* r, uint64_t iteration_number, uint64_t local_iteration_number,
                               float ppm_radius, const orx_request* details);
orx_status orx_ppm_local_photon_trace(orx_renderer* r);
orx_status orx_ppm_slab_histogram(orx_renderer* r, uint32_t* hist_device /* orx_slab_histogram_words */,
                                  uint32_t nbins);
/* the halo for radius r: floor(r * nbins / extent of the scene AABB on axis) + 2 bins */
uint32_t orx_ppm_slab_halo(const orx_renderer* r, uint32_t nbins, uint32_t axis, float radius);
orx_status orx_ppm_slab_pack(orx_renderer* r, const uint8_t* bin_dest, uint32_t nbins, uint32_t axis,
                             uint32_t halo_bins, const uint32_t* dest_base, uint64_t send_records,
                             void* send_device);
orx_status orx_ppm_slab_import(orx_renderer* r, const void* recv_device, uint64_t n_records,
                               const uint32_t* photon_box, uint32_t axis, uint32_t nbins, uint32_t own_lo,
                               uint32_t own_hi);

/* One VCM iteration of a sharded renderer (OptixRenderer.cpp:675-795 split at
 * the light-tracing splats).  Light subpath i pairs with camera pixel i
 * (lightSubpathCount = W*H, VCMLightPass.cu:52), so each rank traces the light
 * subpaths and camera paths of its own rows; the only cross-rank effect is
 * connectCameraT1 (vcm.h:311-384), whose splats may land on any row:
 *   orx_vcm_local_light     light pass over own rows; splats into an owner-block
 *                           buffer [world][max_local_rows][W][3]
 *   orx_export_vcm_splats   that buffer -> caller (orx_vcm_splat_bytes)
 *   (caller reduce-scatters (sum) the buffers, rank-major blocks)
 *   orx_vcm_finish          camera pass over own rows with the summed own-row splats
 * The summed splats equal the single-GPU ones up to fp32 atomic order (the
 * single-GPU pass accumulates them with atomics too). */
size_t orx_vcm_splat_bytes(const orx_renderer* r); /* world * max_local_rows * W * 12 */
orx_status orx_vcm_local_light(orx_renderer* r, uint64_t iteration_number, uint64_t local_iteration_number,
                               float ppm_radius, const orx_request* details);
orx_status orx_export_vcm_splats(orx_renderer* r, void* dst_device, size_t dst_bytes);
/* splat_own_rows_device: local_rows * W * 3 floats (the own block of the sum) */
orx_status orx_vcm_finish(orx_renderer* r, const void* splat_own_rows_device, size_t bytes);

#ifdef __cplusplus
}
#endif

#endif /* ORX_H */
