/*
 * orx_oracle.h — CPU restatement of OppositeRenderer's render core.
 *
 * TEST INFRASTRUCTURE ONLY.  This library is the parity checker and the
 * CPU baseline of bench.py; nothing in the product (liborx.so, the
 * oppositerenderer_amd package) may link, load or call it.  Only tests/,
 * __graft_entry__.smoke() and bench.py's cpu_baseline leg use it.
 *
 * Parity status: the reference (OptiX 3.6 / CUDA 5.5 / Windows) cannot be
 * built or run in this environment and ships no tests, fixtures or golden
 * vectors, so this restatement is pinned only by
 * known-answer tests of its building blocks (cuRAND XORWOW constants,
 * analytic intersection and sampling identities, grid invariants) and by
 * golden images it generated itself (tests/golden/).  Against the reference
 * binary itself parity is UNPINNED.
 *
 * The API mirrors include/orx.h so that tests drive the oracle and the HIP
 * renderer through the same calls.
 */
#ifndef ORX_ORACLE_H
#define ORX_ORACLE_H

#include "orx.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct orc_renderer orc_renderer;

orx_status orc_create(const orx_config* cfg, orc_renderer** out);
orx_status orc_init_scene(orc_renderer* r, const orx_scene* scene);
orx_status orc_render_next_iteration(orc_renderer* r, uint64_t iteration_number,
                                     uint64_t local_iteration_number, float ppm_radius,
                                     int create_output, const orx_request* details);
orx_status orc_get_output(orc_renderer* r, float* dst, size_t dst_bytes);
orx_status orc_read_buffer(orc_renderer* r, int32_t id, void* dst, size_t dst_bytes, size_t* out_bytes);
orx_status orc_get_stats(orc_renderer* r, orx_stats* out);
const char* orc_last_error(const orc_renderer* r);
void orc_destroy(orc_renderer* r);
void orc_set_threads(int n);
void orc_default_config(orx_config* cfg);

/* sharded phase API (see include/orx.h "Multi-GPU sharding") */
orx_status orc_set_shard(orc_renderer* r, uint32_t rank, uint32_t world);
uint32_t orc_local_rows(const orc_renderer* r);
uint32_t orc_max_local_rows(const orc_renderer* r);
size_t orc_hitpoint_export_bytes(const orc_renderer* r);
orx_status orc_ppm_local_passes(orc_renderer* r, uint64_t iter, uint64_t local, float ppm_radius, const orx_request* det);
orx_status orc_export_hitpoints(orc_renderer* r, void* dst, size_t bytes);
orx_status orc_ppm_gather_external(orc_renderer* r, const void* hp, uint32_t segments, void* indirect, size_t bytes);
orx_status orc_ppm_finish(orc_renderer* r, const void* indirect, size_t bytes);
/* sharded VCM: light pass over own rows; splats in owner-block layout
 * [world][max_rows][W][3]; the caller sums them across ranks and hands each
 * rank its own block for the camera pass */
size_t orc_vcm_splat_bytes(const orc_renderer* r);
orx_status orc_vcm_local_light(orc_renderer* r, uint64_t iter, uint64_t local, float ppm_radius, const orx_request* det);
orx_status orc_export_vcm_splats(orc_renderer* r, void* dst, size_t bytes);
orx_status orc_vcm_finish(orc_renderer* r, const void* splat_own_rows, size_t bytes);

/* building blocks exposed for known-answer tests */
void orc_xorwow_init(uint64_t seed, uint32_t state[6]);
uint32_t orc_xorwow_next(uint32_t state[6]);
float orc_uniform(uint32_t state[6]); /* getRandomUniformFloat (helpers/random.h:65-69) */
/* closest hit against the current scene: returns prim id or -1, writes t */
int32_t orc_trace_closest(orc_renderer* r, const float o[3], const float d[3], float tmin, float tmax, float* t_out);
int32_t orc_trace_any(orc_renderer* r, const float o[3], const float d[3], float tmin, float tmax);
void orc_sample_unit_hemisphere_cos(const float n[3], float u1, float u2, float out[3]);
void orc_sample_unit_hemisphere(const float n[3], float u1, float u2, float out[3]);
void orc_camera_setup(const orx_camera* cam, float lookdir[3], float u[3], float v[3]);
/* tex2D of a w x h RGBA8 image (orx_detmath.h orx_tex2d_linear) */
void orc_tex2d(const uint8_t* rgba, uint32_t w, uint32_t h, float u, float v, float out[4]);

#ifdef __cplusplus
}
#endif
#endif
