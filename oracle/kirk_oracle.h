/*
 * kirk_oracle.h -- TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement of the hot path of lucashilbig/BA_Pathtracing_Fur ("KIRK"):
 * the CPU PathTracer + BVH + Cylinder/Triangle + Shaders + BSDFs + Lights
 * (file:line citations in kirk_oracle.c).  It is the parity checker for the
 * HIP product path and the `cpu_baseline` leg of bench.py; only tests/,
 * __graft_entry__.smoke() and bench.py's cpu_baseline may load it.  The
 * product never links, loads or calls it.
 *
 * PARITY UNPINNED by the reference itself: KIRK ships no test cases and no
 * golden vectors (src/unittests has a gtest driver with zero TEST()s), it
 * cannot be compiled here (GLM/GLEW/GLFW/assimp absent, MSVC-only _j0,
 * std::_Pi, `for each`), and its RNGs are std::random_device-seeded and
 * shared across threads.  This restatement replaces every random draw by a
 * documented counter RNG (see DESIGN.md "RNG") and every libm call by the
 * documented kmath functions, so results are reproducible bit-for-bit; its
 * fixtures under tests/golden/ are minted from it and pinned by analytic
 * known-answer tests (tests/test_oracle_kat.py).
 *
 * The input layout is the boundary's (include/kirk_hip.h): the oracle reads
 * the same khp_scene / khp_render_params structs the product does.
 */
#ifndef KIRK_ORACLE_H
#define KIRK_ORACLE_H

#include <stdint.h>
#include "../include/kirk_hip.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct ko_ctx ko_ctx;

int ko_create(ko_ctx** out, const khp_scene* scene);   /* flatten + BVH build */
void ko_destroy(ko_ctx* c);

/* PathTracer::render over `spp` samples; out_rgb running mean (W*H*3).
 * n_threads: row-parallel worker threads (ThreadManager::for_loop_double). */
int ko_render(ko_ctx* c, const khp_render_params* p, int n_threads, float* out_rgb);
/* Render only rows [y0,y1) (bounded CPU-baseline sample); _step: every ystep-th row. */
int ko_render_rows(ko_ctx* c, const khp_render_params* p, int n_threads, uint32_t y0, uint32_t y1,
                   float* out_rgb);
int ko_render_rows_step(ko_ctx* c, const khp_render_params* p, int n_threads, uint32_t y0, uint32_t y1,
                        uint32_t ystep, float* out_rgb);

int ko_trace_closest(ko_ctx* c, uint32_t n, const float* orig, const float* dir, float* t_out,
                     int32_t* obj_out, float* uv_out, uint64_t* node_visits, uint64_t* prim_tests);
int ko_trace_closest_log(ko_ctx* c, uint32_t n, const float* orig, const float* dir, float* t_out, int32_t* log,
                         uint64_t cap, uint64_t* offsets);
int ko_trace_any(ko_ctx* c, uint32_t n, const float* orig, const float* dir, const float* tmax,
                 uint8_t* hit_out);

/* Structural views for parity of the flatten + build stages. */
uint32_t ko_n_objects(ko_ctx* c);
/* ABI 7 light-path variant (include/kirk_hip.h khp_bdpt_params); ko_light_paths:
 * the subpaths of sample index k, [light_paths][n_lights][vertices] x
 * (valid, pos.xyz, din.xyz, hit_color.xyz). */
int ko_set_bdpt(ko_ctx* c, const khp_bdpt_params* p);
int ko_light_paths(ko_ctx* c, uint32_t seed, uint32_t k, float* out10);
/* per object: bmin.xyz, bmax.xyz, centroid.xyz (9 floats) */
void ko_object_bounds(ko_ctx* c, float* out9);
/* per cone: base.xyz r0 | u.xyz slope | v.xyz min_d | w.xyz max_d | base_d height (18 floats) */
void ko_cone_records(ko_ctx* c, float* out18);
/* per triangle: A B C ab ac na nb nc (24 floats) + lA */
void ko_tri_records(ko_ctx* c, float* out24, int32_t* lA);
/* BVH in DFS preorder (node, left subtree, right subtree):
 * per node: bmin.xyz bmax.xyz (6 floats), leaf_first, leaf_count (count 0 = interior).
 * object_ids: the leaf-ordered object id array. returns node count. */
uint32_t ko_bvh_nodes(ko_ctx* c, float* out6, int32_t* first, int32_t* count, int32_t* object_ids);
uint32_t ko_bvh_depth(ko_ctx* c);

/* ABI-6 test hooks: Environment::getColor (dir: 3 floats -> rgb) and
 * Texture::getColor of texture t of the scene (-> rgba). */
void ko_env_color(ko_ctx* c, const float* dir, float* rgb);
void ko_tex_color(ko_ctx* c, uint32_t t, float x, float y, float* rgba);

/* Direct access to single functions for known-answer tests. */
float ko_sinf(float x);
float ko_cosf(float x);
float ko_atan2f(float y, float x);
float ko_acosf(float x);
float ko_asinf(float x);
float ko_expf(float x);
float ko_sinhf(float x);
double ko_j0(double x);
uint32_t ko_rand_u32(uint32_t seed, uint32_t pixel, uint32_t sample, uint32_t dim);

/* One BSDF::sample call (Bsdf.cpp:179-184) on a synthetic hit.
 * hit_obj: object id whose U/V/W frame (cones) is used; mat: material.
 * in: ray_in (negative incident direction), n: normal.
 * sample_io[2] in/out (hair BSDFs overwrite sample.x = theta_i).
 * rng_hair[2]: the two hair draws (alpha, beta) in [0,1).
 * Returns flags; writes out_dir[3], pdf, f[3]. */
int ko_bsdf_sample(ko_ctx* c, int hit_obj, const khp_material* mat, const float in[3], const float n[3],
                   float sample_io[2], const float rng_hair[2], int flags_in,
                   float out_dir[3], float* pdf, float f[3]);

/* Output stage (kirk_tonemap.c): Texture::setPixel byte conversion and
 * Tonemapper::map, sequential in KIRK's order. */
void ko_tonemap_defaults(khp_tonemap* t);
/* The output stage's log / exp / pow replacements (same algorithm as kmath.h k_*_d). */
double ko_log_d(double x);
double ko_exp_d(double x);
double ko_pow_d(double x, double y);
void ko_to_rgba8(uint32_t n_pixels, const float* rgb, uint8_t* out_rgba);
int ko_tonemap(uint32_t W, uint32_t H, const float* rgb, const khp_tonemap* tm, float* out_rgb, float* max_lum,
               float* world_lum);

#ifdef __cplusplus
}
#endif
#endif
