/*
 * kirk_hip.h -- C-ABI of the MI355X-native fur path-tracing core.
 *
 * This is the drop-in boundary for the hot path of lucashilbig/BA_Pathtracing_Fur
 * ("KIRK"): camera ray -> BVH closest hit over hair cone frusta and triangles ->
 * shader/BSDF -> next-event shadow ray -> accumulate.  Every entry point below
 * replaces one KIRK C++ interface; the replaced interface is cited (file:line,
 * relative to the KIRK source tree src/libraries/KIRK/).
 *
 * Conventions
 *  - plain C: no exceptions cross the ABI, no C++ or torch types in signatures;
 *  - every call returns a khp_status; khp_last_error() returns a thread-local
 *    message for the last failing call of this thread;
 *  - all inputs are host pointers and are copied; outputs are caller-owned;
 *  - one khp_ctx is single-threaded, like KIRK's non-re-entrant
 *    CPU_Raytracer::render (KIRK/Utils/Threading.h:117);
 *  - internally: one HIP device + one stream per context, optional RCCL comm.
 *
 * Coordinates/units are KIRK's: world space, right-handed, y up; images are
 * stored row-major with row 0 at the BOTTOM of the frame (Camera::getRayFromPixel
 * starts at m_bottom_left, KIRK/Common/Camera.cpp:59-66).
 */
#ifndef KIRK_HIP_H
#define KIRK_HIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define KHP_ABI_VERSION 13

typedef struct khp_ctx khp_ctx;

typedef enum {
    KHP_OK = 0,
    KHP_EINVAL = 1,       /* bad argument (KIRK: std::invalid_argument)          */
    KHP_ENOMEM = 2,       /* host or device allocation failed                   */
    KHP_EDEVICE = 3,      /* HIP / RCCL error, or no device                     */
    KHP_ENOTREADY = 4,    /* call order violated (e.g. render before build)     */
    KHP_EUNSUPPORTED = 5  /* feature outside the hot path (textures, env maps)  */
} khp_status;

/* ---------------------------------------------------------------------------
 * BSDF and shader kinds.  KIRK registers BSDFs by name in a singleton factory
 * (Bsdf.h:133-241, BsdfFactory.cpp:28-55) and binds std::function callbacks;
 * callbacks cannot run on a GPU, so the GPU side is a closed enum keyed by the
 * same names (khp_bsdf_kind_from_name).
 * ------------------------------------------------------------------------- */
typedef enum {
    KHP_BSDF_LAMBERTIAN_REFLECTION = 0,   /* "LambertianReflectionBSDF"   Bsdf.cpp:186-202 */
    KHP_BSDF_SPECULAR_REFLECTION = 1,     /* "SpecularReflectionBSDF"     Bsdf.cpp:210-219 */
    KHP_BSDF_SPECULAR_TRANSMISSION = 2,   /* "SpecularTransmissionBSDF"   Bsdf.cpp:258-290 */
    KHP_BSDF_GLOSSY = 3,                  /* "GlossyBSDF"                 Bsdf.cpp:227-250 */
    KHP_BSDF_GLASS = 4,                   /* "GlassBSDF"                  Bsdf.cpp:326-359 */
    KHP_BSDF_MILK_GLASS = 5,              /* "MilkGlassBSDF"              Bsdf.cpp:367-418 */
    KHP_BSDF_LAMBERTIAN_TRANSMISSION = 6, /* "LambertianTransmissionBSDF" Bsdf.cpp:298-318 */
    KHP_BSDF_EMISSION = 7,                /* "EmissionBSDF"               Bsdf.cpp:427-437 */
    KHP_BSDF_TRANSPARENT = 8,             /* "TransparentBSDF"            Bsdf.cpp:445-456 */
    KHP_BSDF_MARSCHNER_HAIR = 9,          /* "MarschnerHairBSDF"          Bsdf.cpp:465-776 */
    KHP_BSDF_DEON_HAIR = 10,              /* "DEonHairBSDF"               Bsdf.cpp:784-1056 */
    KHP_BSDF_COUNT = 11
} khp_bsdf_kind;

typedef enum {
    KHP_SHADER_SIMPLE = 0,          /* "SimpleShader"        SimpleShader.h:31-152        */
    KHP_SHADER_MARSCHNER_HAIR = 1,  /* "MarschnerHairShader" MarschnerHairShader.h:31-138 */
    KHP_SHADER_COUNT = 2
} khp_shader_kind;

/* KIRK::Material (Material.h:53-152): the parameter values.  Textured
 * parameters (MatParamColor/MatParamFloat with a texture) are given by
 * khp_scene.material_textures below (ABI 6). */
typedef struct {
    int32_t bsdf;          /* khp_bsdf_kind   */
    int32_t shader;        /* khp_shader_kind */
    float diffuse[3];      /* m_diffuse   */
    float specular[3];     /* m_specular  */
    float volume[3];       /* m_volume    */
    float emission[3];     /* m_emission  */
    float ior;             /* m_ior (KIRK default 1.52, Material.h:83)    */
    float roughness;       /* m_roughness (KIRK default 1.0)             */
} khp_material;

typedef enum {
    KHP_LIGHT_POINT = 0,   /* PointLight Light.cpp:127-199 */
    KHP_LIGHT_QUAD = 1,    /* QuadLight  Light.cpp:216-296 */
    KHP_LIGHT_SPOT = 2,    /* SpotLight  Light.cpp:327-440 */
    KHP_LIGHT_SUN = 3      /* SunLight   Light.cpp:463-511 */
} khp_light_kind;

/* Constructor arguments of the KIRK light classes (Light.h), identity node
 * transform.  The library derives the same state KIRK derives in the ctor
 * and in Light::transform (normalised direction, quad vertices). */
typedef struct {
    int32_t kind;          /* khp_light_kind */
    float color[3];
    float position[3];
    float direction[3];    /* ctor argument; normalised by the library      */
    float size[2];         /* QuadLight m_size                               */
    float radius;          /* point/spot/sun m_radius                        */
    float att_const, att_lin, att_quad;
    float inner_angle, outer_angle;   /* SpotLight, degrees                  */
} khp_light;

/* KIRK::Environment (Environment.h): background colour + ambient.  The
 * CUBE_MAP / SPHERE_MAP types are khp_scene.env_map (ABI 6). */
typedef struct {
    float color[3];
    float ambient[3];
} khp_environment;

/* ABI 6: KIRK::Texture as the CPU path tracer reads it (Texture.cpp:243-287):
 * 8-bit texels, 1..4 channels, row y at data + y * width * channels (KIRK's
 * m_texture_data), looked up nearest-texel with KIRK's wrap rule. */
#define KHP_TEX_WRAP_CLAMP 0   /* TEXTURE_WRAP_MODE_CLAMP (Texture.h:34) */
#define KHP_TEX_WRAP_TILE 1    /* TEXTURE_WRAP_MODE_TILE  (Texture.h:35), KIRK's default */
typedef struct {
    uint32_t width, height;
    uint32_t channels;         /* 1 (rrrr), 2 (rrrg), 3 (rgb1) or 4 (rgba)         */
    uint32_t wrap_mode;        /* m_texture_wrap_mode                              */
    const uint8_t* data;       /* width * height * channels bytes, copied          */
} khp_texture;

/* ABI 6: which material parameters are textured (index into khp_scene.textures,
 * -1: the khp_material value).  Material::getFromParam (Material.cpp:15-23):
 * colours take the texel's rgb, roughness takes the length of its rgba. */
typedef struct {
    int32_t diffuse, specular, volume, emission, roughness;
} khp_material_textures;

/* ABI 6: Environment::m_type (Environment.h:25-30, getColor Environment.cpp:91-133). */
#define KHP_ENV_COLOR 0
#define KHP_ENV_CUBE_MAP 1     /* tex: posx, posy, posz, negx, negy, negz (loadCubeMap order) */
#define KHP_ENV_SPHERE_MAP 2   /* tex[0] */
typedef struct {
    int32_t type;
    int32_t tex[6];            /* indices into khp_scene.textures                  */
} khp_env_map;

/* The state KIRK::Camera::applyParameters derives (Camera.cpp:6-37). */
typedef struct {
    float position[3];
    float bottom_left[3];
    float axis_x[3];
    float axis_y[3];
    float pixel_size;
} khp_camera;

/* Flattened scene = what KIRK::CPU::Scene::flattenNode produces
 * (CPU_Scene.cpp:73-197), before the Triangle/Cylinder constructors run.
 * Object order (it shapes the BVH): triangles [0,n_tris) then cones. */
typedef struct {
    uint32_t n_tris;
    const float* tri_v;           /* [n_tris][3][3] vertices a,b,c (Triangle ctor args) */
    const float* tri_n;           /* [n_tris][3][3] vertex normals na,nb,nc             */
    const uint32_t* tri_mat;      /* [n_tris] material index                            */
    uint32_t n_cones;
    const float* cone_base_r0;    /* [n_cones][4] basePoint.xyz, baseRadius  (Cylinder ctor) */
    const float* cone_apex_r1;    /* [n_cones][4] apexPoint.xyz, apexRadius                  */
    const uint32_t* cone_mat;     /* [n_cones] material index                                */
    uint32_t n_materials;
    const khp_material* materials;
    uint32_t n_lights;
    const khp_light* lights;
    khp_environment env;
    khp_camera camera;
    /* ABI 4: optional [n_tris][3][3] hair frame u, v, w per triangle
     * (Object::setU/V/W, set by CPU_Scene::fiberToTriangles, CPU_Scene.cpp:
     * 232-345, for fur drawn as triangle tubes; read by the hair BSDFs).
     * NULL: zero frames (KIRK leaves them uninitialised on plain triangles). */
    const float* tri_frame;
    /* ABI 6: node transforms of the cones.  flattenNode hands each fiber's
     * Cylinder the transform base_transform * child->m_transform
     * (CPU_Scene.cpp:119, 136-137); the ctor maps base/apex by it and the frame
     * by its inverse transpose (Cylinder.cpp:5-29).  cone_base_r0/apex_r1 are
     * then the PRE-transform points.  n_cone_models = 0: world-space cones
     * (identity, the ctor's arithmetic without the matrix products). */
    uint32_t n_cone_models;
    const float* cone_models;     /* [n_cone_models][16] glm::mat4, column-major             */
    const uint32_t* cone_model;   /* [n_cones] index into cone_models; NULL: model 0 for all */
    /* ABI 6: textures (a17 / a16 / a9 in SURVEY §8) */
    uint32_t n_textures;
    const khp_texture* textures;
    const khp_material_textures* material_textures;  /* [n_materials], or NULL: untextured */
    const float* tri_uv;          /* [n_tris][3][2] texcoords tca, tcb, tcc, or NULL: zeros   */
    khp_env_map env_map;          /* type KHP_ENV_COLOR: env.color (zero-initialised = COLOR) */
} khp_scene;

#define KHP_RENDER_OUT_DEVICE   (1u << 0)  /* out_rgb is a device pointer        */
#define KHP_RENDER_NO_READBACK  (1u << 1)  /* keep framebuffer in HBM only       */
#define KHP_RENDER_STATS        (1u << 2)  /* instrumented kernels for this call  */
#define KHP_RENDER_ASYNC        (1u << 3)  /* enqueue and return (ABI 5): frames in flight overlap;
                                              no readback, no STATS; khp_sync completes them */

/* One khp_render call = samples [first_sample, first_sample+spp) of
 * PathTracer::render (CPU_PathTracer.cpp:17-52) for every pixel this rank
 * owns; the framebuffer holds KIRK's running mean (drawTexture, :61-90). */
typedef struct {
    uint32_t width, height;
    uint32_t spp;            /* samples in this call                               */
    uint32_t depth;          /* max bounces, PathTracer m_depth (Demo uses 5)      */
    uint32_t seed;           /* frame seed of the counter RNG                      */
    uint32_t first_sample;   /* progressive resume: 0 starts a new frame           */
    uint32_t tile_size;      /* square tiles; 0 -> 64                              */
    uint32_t tile_rank;      /* this rank renders tiles with id % tile_nranks == tile_rank */
    uint32_t tile_nranks;    /* 0 or 1 -> all tiles                                */
    uint32_t flags;          /* KHP_RENDER_*                                       */
} khp_render_params;

typedef struct {
    uint64_t n_objects, n_nodes, n_leaves;
    uint32_t bvh_depth, max_leaf_size;
    uint64_t device_bytes;           /* scene + BVH + queues resident in HBM  */
    double build_ms;                 /* flatten + BVH build (host)            */
    double upload_ms;
    double render_ms;                /* last khp_render, device time          */
    double extend_ms, shade_ms, shadow_ms, other_ms;  /* per-kernel device time, last render */
    uint64_t extend_rays, shadow_rays, extend_launches;
    uint64_t node_visits, prim_tests, shadow_node_visits, shadow_prim_tests; /* KHP_CTX_STATS only */
    uint64_t stack_spills;           /* traversal-stack entries spilled from LDS (stats only) */
    /* per bounce (index = bounce, up to KHP_MAX_BOUNCE_STATS), instrumented renders only */
    uint64_t bounce_rays[16], bounce_nodes[16], bounce_prims[16];
    uint64_t bounce_shadow_rays[16], bounce_shadow_nodes[16], bounce_shadow_prims[16];
    double bounce_extend_ms[16], bounce_shadow_ms[16];
    /* traversal-loop efficiency (instrumented renders): wave iterations and the
     * lanes that had a record to fetch in them (busy / (64 * iters) = lane use) */
    uint64_t bounce_wave_iters[16], bounce_lanes_busy[16];
    uint64_t bounce_shadow_wave_iters[16], bounce_shadow_lanes_busy[16];
    /* diagnostic builds (KHP_PROFILE_STEPS=1) only: k_extend wave cycles spent in
     * resolve / record fetch / compute / loop+refill, summed over waves */
    uint64_t step_cycles[4];
    /* ABI 3: where khp_build_accel built the BVH and how long it took */
    uint32_t bvh_on_device;          /* 1: device build (default), 0: host   */
    uint32_t subframes;              /* always 1 (ABI 6: one path set per frame slot) */
    double flatten_ms;               /* khp_set_scene (flatten, incl. copies) */
    double bvh_ms;                   /* BVH build wall time incl. transfers   */
    double bvh_kernel_ms;            /* device build: GPU time of its kernels  */
    double layout_ms;                /* node pairing + leaf slots + slot records */
    double flatten_kernel_ms;        /* device flatten: GPU time of its kernels */
    double layout_kernel_ms;         /* device layout: GPU time of its kernels  */
    /* stack entries popped only to fail the prune test (instrumented renders) */
    uint64_t extend_pruned_pops, shadow_pruned_pops;
    /* ABI 5: frames this report covers -- 1 after a synchronous khp_render (1 +
     * render_ahead when the call rendered the next calls' passes in its fused
     * batch, whose timings and counters it then reports); after khp_sync, every
     * asynchronous frame completed since the previous report, with timings
     * (extend_ms, extend_launches, ...) and counters summed over them */
    uint64_t frames;
    /* ABI 5: wall time during which at least one k_extend launch of the report
     * was running (union of the launches' HIP-event intervals); equals extend_ms
     * when launches do not overlap (synchronous renders) */
    double extend_busy_ms;
    /* ABI 6: the shadow stage split -- shadow_ms above is k_shadow + the shadow
     * finish; shadow_finish_ms is the finish alone, shadow_launches counts the
     * any-hit (k_shadow) launches */
    double shadow_finish_ms;
    uint64_t shadow_launches;
    /* ABI 13: render-ahead (khp_ctx_params.render_ahead), last synchronous render:
     * its paths earlier calls had already finished (all of them when an earlier
     * wavefront call's fused batch held its pass), and those it resumed from park
     * records (0 when the call had nothing rendered ahead) */
    uint64_t ahead_finished, ahead_resumed;
} khp_stats;
#define KHP_MAX_BOUNCE_STATS 16

#define KHP_CTX_STATS  (1u << 0)   /* instrumented kernels: count node/prim visits */
#define KHP_CTX_HOST_BUILD (1u << 1) /* khp_build_accel builds the BVH on the host
                                       (default: on the device, the same tree)   */

/* ABI 6: scheduling parameters of a context.  They decide how the wavefront
 * is cut and overlapped on the device, never what it computes: every value
 * gives the same frames bit for bit.  khp_ctx_params_defaults() fills the
 * measured defaults; khp_set_params completes in-flight frames
 * first.  (KIRK has no counterpart: its PathTracer segments by the GUI's
 * maxBufferSize, CPU_PathTracer.cpp:211-241, which chunk_paths mirrors.) */
typedef struct {
    uint32_t fuse_frames;        /* asynchronous frames with equal parameters fused into one batch,
                                    1..32 (default 32)                                               */
    uint32_t frames_in_flight;   /* batches in flight at once, 1..3 (default 1)                     */
    uint64_t chunk_paths;        /* paths per wavefront chunk, >= 4096; 0 (default): the smaller of
                                    2^28 (2^27 before round 6) and what fits in half the free HBM    */
    uint32_t heavy_iters;        /* longest-first queues: a path whose last traversal took more
                                    iterations has its next rays claimed first (default 0xFFFFFFFF =
                                    off since round 6; 160 before).  No effect on the extension rays
                                    of bounces regrouped by ray_sort_from (their claim order is the
                                    cell order; shadow rays keep it); path_order 2 marks its heavy
                                    pixels with it                                                  */
    int32_t dump_bounce;         /* debug: keep the extension rays of this bounce of the next
                                    synchronous render for khp_debug_queue (-1: off, default)       */
    uint32_t trace_kernels;      /* khp_trace_closest / khp_trace_any run on 0: one-ray-per-thread
                                    kernels (default), 1: the instrumented persistent kernels (KIRK's
                                    visit counts), 2: the production persistent kernels             */
    uint32_t shade_order;        /* ABI 7: 0 (default): k_shade takes the hits in queue order; 1: hits are
                                    first grouped by shading class (no hit / BSDF kind), a counting
                                    sort per bounce -- KIRK's GLSL template only compacts its hits
                                    (pt_sortHits.compute:17-38); measured in DESIGN.md §4            */
    uint32_t serial_stages;      /* ABI 7: 1 = the shadow stage runs on the extend stream, so no two
                                    kernels of a frame overlap and each kernel's timing is its own
                                    (bench.py's isolated per-kernel rooflines); 0 (default) = two
                                    streams, shadow stage b beside extend b+1                         */
    uint32_t path_order;         /* ABI 9: how a fused chunk numbers its paths.  0: frame-major (frame f's
                                    pixels x samples form one block); 1 (default): pixel-major (all fused
                                    frames' samples of one pixel are adjacent paths, so a wave traces one
                                    pixel of 8 frames at 8 spp); 2: pixel-major, and the wavefront takes the
                                    pixels whose previous camera ray was long first (a per-batch permutation
                                    of the pixel list; results unchanged).  Measured in DESIGN.md §5a   */
    uint32_t wide_from;          /* ABI 10: the first bounce whose closest-hit traversal runs on two-level
                                    node records (one 128-B record per step: a node's child boxes and the
                                    near child's own, KIRK's order and counts kept); earlier bounces use the
                                    64-B records.  Default 2 (measured); >= depth: never.
                                    The shadow stage (any hit) of bounce b uses them when b >= max(wide_from,
                                    2).  Batch queries with trace_kernels use them iff wide_from == 0   */
    uint32_t path_kernel;        /* ABI 11: 0 (default) automatic, 1 never, 2 whenever supported: run a chunk's
                                    paths through all their bounces in ONE persistent launch (k_path: a lane
                                    traces, shades, traces the shadow ray and continues with the next bounce)
                                    instead of the per-bounce wavefront, whose every launch ends with its
                                    slowest ray.  Automatic: synchronous renders (KIRK's own one-call-per-pass
                                    use) of at most 14 x 2^20 paths (1080p up to 7 spp; past that the
                                    wavefront's steady rate wins).  Not with the light-path variant, hit
                                    sorting, instrumented renders or queue dumps (those always run the
                                    wavefront).  Measured in DESIGN.md §5b                              */
    uint32_t ray_sort_from;      /* ABI 12: the first bounce whose extension rays are regrouped before
                                    k_extend by the Morton cell (32^3 over the scene box) of their origin, so
                                    that the rays of a claim block start close together and share cache
                                    lines; the path state stays in place.  Which lane traces which ray
                                    changes no result.  0 (default): automatic -- bounce 2 when the tree's
                                    node records exceed 64 MB, else never (a cache-resident tree has no
                                    misses to save; measured); 1..: that bounce; >= depth:
                                    never.  Not with hit sorting (shade_order 1), the light-path variant or
                                    queue dumps; the path kernel never sorts                              */
    uint32_t lds_nodes;          /* ABI 12: 0 (default) or 7: the tree's top three levels of node records
                                    staged in each traversal wave's LDS beside its stack rings (the 64-B
                                    loops of k_extend and k_shadow), the rest fetched from HBM as before.
                                    Same walk, same counts, same frames.  Measured in DESIGN.md §4    */
    uint32_t render_ahead;       /* ABI 13: 0..3 (default 3).  A synchronous render that runs the path kernel
                                    in one chunk lets the lanes that would idle in its launch's drain (its
                                    longest paths finishing alone) start the paths of the next render_ahead
                                    calls of a progressive series -- the same pixels, spp, depth and seed,
                                    first_sample + spp, + 2 spp, ...: KIRK's PathTracer::render loop,
                                    CPU_PathTracer.cpp:17-52.  A call still returns as soon as its own
                                    paths end (at once when earlier calls finished them all); the paths of
                                    later calls in flight then are parked and resumed by later calls, which
                                    accumulate the colours already finished.  Any other call, and any change
                                    of scene, camera or parameters, drops that work.  A synchronous render
                                    that runs the wavefront (one chunk) and continues the series of the
                                    previous synchronous call renders its own pass and the next render_ahead
                                    calls' passes as one fused batch; those calls then only accumulate.
                                    Frames, textures and framebuffers are those of each call alone, bit for
                                    bit.  Measured in DESIGN.md §5c                                        */
    uint32_t path_from;          /* ABI 13: 0 (default) or b >= 1: a wavefront render hands the paths still
                                    alive at bounce b to ONE path-kernel launch (k_path), which carries them
                                    through the remaining bounces without a barrier per bounce -- the last
                                    bounces' launches are short and end with their slowest ray.  Not with the
                                    light-path variant, hit sorting, instrumented renders or queue dumps;
                                    >= depth: off.  No value changes a pixel.  Measured in DESIGN.md §5d   */
} khp_ctx_params;   /* 64 bytes */

/* ---- context --------------------------------------------------------------- */
/* device: HIP device ordinal (one process per GPU). */
khp_status khp_create(khp_ctx** out, int device, uint32_t flags);
void khp_destroy(khp_ctx* ctx);
const char* khp_last_error(void);
int khp_abi_version(void);
void khp_ctx_params_defaults(khp_ctx_params* out);
khp_status khp_set_params(khp_ctx* ctx, const khp_ctx_params* params);
khp_status khp_get_params(khp_ctx* ctx, khp_ctx_params* out);

/* Replaces CPU::Scene::setSceneGraph (CPU_Scene.cpp:25-43) + the Triangle and
 * Cylinder constructors (Triangle.cpp:3-129, Cylinder.cpp:5-67). Copies. */
khp_status khp_set_scene(khp_ctx* ctx, const khp_scene* scene);

/* Replaces BVH::addBaseDataStructure (CPU_BVH.cpp:16-44): binned SAH, 16 bins,
 * leaf threshold 1 (CPU_BVH.h:64); uploads scene + BVH to HBM. */
khp_status khp_build_accel(khp_ctx* ctx);

/* Replaces PathTracer::render (CPU_PathTracer.cpp:17-52).  out_rgb: W*H*3
 * floats (host unless KHP_RENDER_OUT_DEVICE, ignored with NO_READBACK).
 * Pixels of tiles not owned by this rank are left untouched. */
khp_status khp_render(khp_ctx* ctx, const khp_render_params* p, float* out_rgb);

/* ABI 7: the light-path (bidirectional) variant of KIRK's GLSL path tracer,
 * lbb_construction.compute:195-403 builds light subpaths
 * (generatePrimaryLightRays / traceLightRays / shadeLightRays) and
 * pt_shade.compute:146-201 connects every camera hit to the vertices of one
 * randomly chosen subpath (sampling.is_bidirectional) instead of KIRK's
 * next-event estimate.  Per sample index k of a render, `light_paths`
 * subpaths per light are traced, each with up to `vertices` vertices (the
 * first on the light).  The exact rules, with the points where the GLSL is
 * undefined and this restatement decides, are in DESIGN.md §10.  KIRK's GLSL
 * marks the feature "experimental"; its estimator is not KIRK's CPU one, so
 * frames differ from khp_render without it (not a parity mode). */
typedef struct {
    uint32_t enabled;       /* 0: KIRK's next-event estimate (default)                          */
    uint32_t light_paths;   /* samples_per_light: subpaths per light and sample index, 1..65536  */
    uint32_t vertices;      /* bounces_per_path: vertices per subpath incl. the light's, 1..16   */
    float bias;             /* debug.bias: connection-ray origin offset along the normal         */
    float bounce_bias;      /* debug.bounce_bias: light-ray origin offset and vertex pull-back   */
    float min_pdf;          /* debug.min_pdf: a light vertex with pdf <= min_pdf ends its subpath */
    uint32_t image_plane;   /* also connect each sample's light vertices to its point on the
                               sensor (shadeBDPTImagePlane, pt_shade.compute:17-97):
                               0 off; 1 (default) the GLSL's target as written, record j's ray
                               origin + bias * its direction, i.e. the PREVIOUS vertex nudged
                               along the segment (pt_shade.compute:38-44 with
                               lbb_construction.compute:229-235, 391-395); 2 the vertex itself
                               pulled back by bounce_bias, like the hit connections (ABI 8)   */
} khp_bdpt_params;
void khp_bdpt_params_defaults(khp_bdpt_params* out);   /* off; 256 paths, 4 vertices, 1e-4 x 3, image plane on */
khp_status khp_set_bdpt(khp_ctx* ctx, const khp_bdpt_params* params);
khp_status khp_get_bdpt(khp_ctx* ctx, khp_bdpt_params* out);

/* Completes every frame enqueued with KHP_RENDER_ASYNC (ABI 5).  A progressive
 * caller (KIRK's PathTracer::render loop) enqueues its passes and syncs before
 * reading the texture; passes accumulate in call order.  Any synchronous call
 * (render, read, gather, scene change) also completes in-flight frames first. */
khp_status khp_sync(khp_ctx* ctx);

/* khp_set_scene with the per-object arrays in device memory of ctx's GPU:
 *   device: tri_v, tri_n, tri_mat, tri_frame, tri_uv, cone_base_r0,
 *           cone_apex_r1, cone_mat, cone_model;
 *   host:   materials, lights, camera, env, cone_models (the matrix table,
 *           inverted on the host), textures and their texel data,
 *           material_textures -- a device pointer there is refused (EINVAL).
 * The objects are flattened on the device; the arrays are
 * read during the call only.  Not with KHP_CTX_HOST_BUILD. */
khp_status khp_set_scene_device(khp_ctx* ctx, const khp_scene* scene);

/* khp_gen_hairball followed by khp_fibers_to_cones, on the device: writes
 * n_strands * (verts - 1) cones (float4 base.xyz r0 / apex.xyz r1) into the
 * device arrays d_base_r0 / d_apex_r1; bit-identical to the host pair. */
khp_status khp_gen_hairball_device(khp_ctx* ctx, uint32_t n_strands, uint32_t verts, const float center[3],
                                   float ball_radius, float root_radius, uint32_t seed, float* d_base_r0,
                                   float* d_apex_r1);

/* khp_gen_hairball followed by khp_fibers_to_triangles, on the device, into
 * device arrays of n_strands*(verts-1)*2*res*res triangles (9 floats each). */
khp_status khp_gen_hairball_tris_device(khp_ctx* ctx, uint32_t n_strands, uint32_t verts, const float center[3],
                                        float ball_radius, float root_radius, uint32_t seed, uint32_t resolution,
                                        float* d_v, float* d_n, float* d_frame);

/* Device memory on ctx's GPU for the arrays above (plain hipMalloc / hipFree),
 * and a synchronous copy (to_device 1: host -> device, 0: device -> host). */
khp_status khp_device_alloc(khp_ctx* ctx, size_t bytes, void** out);
khp_status khp_device_free(khp_ctx* ctx, void* p);
khp_status khp_device_copy(khp_ctx* ctx, void* dst, const void* src, size_t bytes, int to_device);

/* Copy the device framebuffer (running mean, W*H*3) to host. */
khp_status khp_read_framebuffer(khp_ctx* ctx, float* out_rgb);

/* KIRK::Tonemapper parameters (Utils/Tonemapping.h:22-33; defaults in the
 * comments; khp_tonemap_defaults() fills them). */
typedef struct {
    float exposure;     /* m_exposure   0     (exposure factor 2^exposure) */
    float bias;         /* m_biasParam  0.85                               */
    float gamma;        /* m_gammaval   1                                  */
    float contrast;     /* m_contParam  0     (0: off)                     */
    float white, black; /* m_white 1, m_black 0                            */
    int32_t rec_gamma;  /* m_use_rec_gamma 0                               */
    int32_t center_weight;   /* m_center_weight 0: world luminance from a
                                Gaussian window (luminance_from_center)     */
    float kernel_multiplier; /* m_kernel_multiplier 0.125                   */
    int32_t center_x, center_y; /* m_center_x/y -1: W/2, H/2                */
} khp_tonemap;

/* Output stage on the device: PathTracer::drawTexture -> Texture::setPixel
 * (CPU_PathTracer.cpp:61-90, Texture.h:252-254), optionally after
 * PathTracer::applyToneMapping -> Tonemapper::map (CPU_PathTracer.cpp:92-104,
 * Tonemapping.cpp).  out_rgba: W*H*4 bytes, row y = KIRK texture row y (row 0
 * = bottom of the frame); byte = (uint8)max(min(c*255, 255), 0) truncated,
 * NaN -> 0; alpha 255.  tm = NULL: no tonemapping. */
khp_status khp_read_rgba8(khp_ctx* ctx, const khp_tonemap* tm, uint8_t* out_rgba);

/* ABI 8: the same 8-bit texture (tm = NULL form) without waiting, for a viewer
 * that shows every progressive pass (KIRK's GUI calls PathTracer::render once
 * per sample, CPU_PathTracer.cpp:17-52, then draws the texture).  The
 * conversion is enqueued in call order behind the asynchronous renders, like
 * a gather (inside a fused batch it runs between two frames' accumulates);
 * out_rgba (W*H*4 bytes of the frame it follows) is written by the time
 * khp_snapshot_wait(ticket) or khp_sync returns and must stay valid until
 * then.  Tonemapped textures need KIRK's sequential host sum and stay
 * synchronous (khp_read_rgba8). */
khp_status khp_read_rgba8_async(khp_ctx* ctx, uint8_t* out_rgba, uint64_t* ticket);
/* Delivers snapshot `ticket` and every older one.  wait = 1: enqueues what is
 * still pending and blocks; wait = 0: KHP_ENOTREADY if it has not completed. */
khp_status khp_snapshot_wait(khp_ctx* ctx, uint64_t ticket, int wait);

/* The Tonemapper member defaults (Tonemapping.h:23-33). */
void khp_tonemap_defaults(khp_tonemap* tm);

/* Batch forms of CPU_DataStructure::closestIntersection / isIntersection
 * (CPU_DataStructure.h:25-28, BVH impl CPU_BVH.cpp:51-93), on the GPU.
 * orig/dir: [n][3] host arrays; dir is normalised like KIRK::Ray (Ray.cpp:11-15).
 * closest: t_out = lambda (FLT_MAX if none), obj_out = object id or -1,
 *          uv_out (optional, [n][2]) = barycentric u,v (0 for cones).
 * any:     hit_out[i] = 1 if an object is hit with t in [0, tmax[i]]. */
khp_status khp_trace_closest(khp_ctx* ctx, uint32_t n, const float* orig, const float* dir,
                             float* t_out, int32_t* obj_out, float* uv_out);
khp_status khp_trace_any(khp_ctx* ctx, uint32_t n, const float* orig, const float* dir,
                         const float* tmax, uint8_t* hit_out);

khp_status khp_get_stats(khp_ctx* ctx, khp_stats* out);

/* ---- multi-GPU: tile sharding + RCCL framebuffer gather -------------------- */
/* RCCL unique id (128 bytes), created on rank 0 and broadcast by the caller. */
khp_status khp_comm_unique_id(uint8_t out_id[128]);
/* Joins the RCCL communicator of nranks ranks (one process per GPU).  ABI 11:
 * the communicator is non-blocking (ncclConfig_t.blocking = 0) and no call of
 * this context waits without a bound while it exists: RCCL calls are polled to
 * completion, and every device wait (khp_sync, synchronous renders, reads,
 * khp_destroy) polls ncclCommGetAsyncError.  An RCCL error, or an RCCL
 * operation that stays runnable (the work queued before it done) without
 * completing for the context's timeout (khp_comm_set_timeout, default 120 s:
 * e.g. a peer that never joins or a gather without its counterpart; a wait on
 * compute alone is never cut short, ABI 11 as amended in round 5), aborts the
 * communicator (ncclCommAbort) and returns KHP_EDEVICE with a message naming
 * this rank and its peers; gathers then return KHP_ENOTREADY until the next
 * khp_comm_init.  KIRK has no multi-device path; its only failure mode is the
 * loud exit of CPU_PathTracer.cpp:236-240. */
khp_status khp_comm_init(khp_ctx* ctx, int nranks, int rank, const uint8_t id[128]);
/* ABI 11: the bound (ms, > 0) of the waits above, for this context. */
khp_status khp_comm_set_timeout(khp_ctx* ctx, uint32_t timeout_ms);
/* Gather every rank's owned tiles (per p->tile_*) into rank root's device
 * framebuffer over RCCL; root may then khp_read_framebuffer. Collective. */
khp_status khp_gather_framebuffer(khp_ctx* ctx, const khp_render_params* p, int root);

/* ABI 8: an in-process group of contexts (rank = index in ctxs, all on one
 * device) for khp_gather_framebuffer without RCCL -- RCCL needs one GPU per
 * rank, this transport lets one process (e.g. a single-GPU test box) run every
 * rank's contexts and the product's gather plan, pack and unpack kernels.  A
 * sender's k-th gather packs into ring slot k % 64, stamped with k; the root's
 * k-th gather copies every sender's slot k, so each sender must have ENQUEUED
 * its k-th gather (khp_sync flushes fused frames) before the root's k-th gather
 * is enqueued (else the root's call returns KHP_ENOTREADY; a gather issued
 * with no asynchronous renders pending can then be repeated, but one queued
 * behind pending asynchronous renders runs when that fused batch is enqueued,
 * and its KHP_ENOTREADY then ends the batch where it stands: khp_sync the
 * senders before such a root gather), and a sender 64 gathers ahead of the root gets KHP_ENOTREADY instead of
 * overwriting a slot the root has not taken (ABI 11: stamps; before, both cases
 * copied stale pixels silently).  A member's pack into a slot waits for the
 * root's copy of its previous content.  Re-initialising a member removes it
 * from its old group. */
khp_status khp_comm_init_local(khp_ctx* const* ctxs, int nranks);

/* ABI 8: the pixel plan khp_gather_framebuffer moves, as seen from `rank`
 * (host only, no device needed).  KIRK has no multi-device path; its analogue
 * is the square-segment split of BufferSegmentation (Utils/BufferSegmentation.h:
 * 34-75).  Tile t (tile_size px, 0 -> 64, row-major) is rendered by rank
 * t % nranks.  counts (nullable, [nranks]): pixels rank r sends to root in
 * this rank's view -- the root lists every sender, a sender lists only itself,
 * the root's own entry is 0; pixels (nullable): their pixel indices y*W + x,
 * concatenated in rank order, each tile as 8x8 blocks; *n_pixels = the total.
 * A sender's counts[rank] equals the root's counts[rank] by construction. */
khp_status khp_gather_plan(uint32_t width, uint32_t height, uint32_t tile_size, int nranks, int rank, int root,
                           uint64_t* counts, uint32_t* pixels, uint64_t* n_pixels);

/* The BVH khp_build_accel built (device or host path), in the layout of
 * khp_host_build below: call with null arrays for *n_nodes / *depth. */
khp_status khp_read_bvh(khp_ctx* ctx, uint32_t* n_nodes, uint32_t* depth, float* node_boxes, int32_t* node_first,
                        int32_t* node_count, int32_t* object_ids);

/* The traversal records khp_build_accel left in HBM: n_records interior-node
 * records (64 B each: L.min.xyz L.max.x | L.max.yz R.min.xy | R.min.z R.max.xyz
 * | Lref Rref Lcnt Rcnt), n_slots primitive records (16 floats) and their aux
 * words (base_d, material, object, flags).  Null arrays: sizes only. */
khp_status khp_read_layout(khp_ctx* ctx, uint32_t* n_records, uint32_t* n_slots, void* node_records,
                           float* prim_records, uint32_t* prim_aux);

/* ---- host-only introspection (no device needed) ---------------------------- */
/* Runs exactly the flatten + BVH build of khp_set_scene/khp_build_accel on the
 * host.  Call with null arrays first to get *n_nodes / *depth.  Nodes are in
 * DFS preorder (node, left subtree, right subtree), like the recursion of
 * BVHNode::split (CPU_BVH.cpp:95-138).
 *   node_boxes [n_nodes][6] bmin.xyz bmax.xyz; node_first/node_count: leaf
 *   candidate range into object_ids (count 0 = interior, first = -1);
 *   object_ids [n_obj] leaf order; obj_bounds [n_obj][9] bmin bmax centroid;
 *   records [n_obj][16] the 64-byte intersection record of every object. */
khp_status khp_host_build(const khp_scene* scene, uint32_t* n_nodes, uint32_t* depth, float* node_boxes,
                          int32_t* node_first, int32_t* node_count, int32_t* object_ids, float* obj_bounds,
                          float* records);

/* ABI 12 (round 5): the host half of the tonemapped texture (khp_read_rgba8 with a
 * khp_tonemap): KIRK's `float sum; sum += log(...)` over the per-pixel log
 * luminances (Tonemapping.cpp:66-91, the terms in double, every step rounded
 * to float), continued from `start`, bit for bit but at one double add per
 * pixel (tonemap_host.cpp).  Exposed for tests and hosts that tonemap their own
 * framebuffer reads. */
khp_status khp_tonemap_log_sum(const double* terms, uint64_t n, float start, float* out);

/* Debug introspection: when the last synchronous khp_render ran with
 * khp_ctx_params.dump_bounce = b, the extension rays of bounce b (queue order) are
 * kept on the host.  Call with null arrays to get *n, then with [n][3] arrays. */
khp_status khp_debug_queue(khp_ctx* ctx, uint32_t* n, float* orig, float* dir);
/* The same render's shadow rays of bounce b as k_shadow traces them (after the
 * zero-colour skip): origin, direction ([n][3]) and t_max ([n]). */
khp_status khp_debug_shadow_queue(khp_ctx* ctx, uint32_t* n, float* orig, float* dir, float* tmax);
/* ABI 13, test hook for the bounded device waits of a rank: builds
 * one RCCL-operation bracket (events `pre` / `post`, as around an ncclSend /
 * ncclRecv) on the context stream around a gate kernel that spins until
 * `release_ms` after the call starts (or 10 s), then waits for the stream with
 * the bound `bound_ms` as khp_sync would on a rank.  scenario 0: the gate
 * before `pre` (the operation never became runnable: no timeout); 1: the gate
 * between `pre` and `post` (runnable, not completing: KHP_EDEVICE after the
 * bound); 2: `pre` only, no `post` (retired once `pre` completes, then no
 * timeout).  *waited_ms: the wait's wall time.  The context keeps no
 * communicator state afterwards.  No RCCL call is made. */
khp_status khp_debug_comm_wait(khp_ctx* ctx, int scenario, uint32_t bound_ms, uint32_t release_ms,
                               double* waited_ms);

/* ---- registries / host helpers --------------------------------------------- */
/* BsdfFactory::getBsdf / ShaderFactory::getShader by KIRK name; -1 if unknown
 * (KIRK throws std::invalid_argument, BsdfFactory.cpp:39-45). */
int khp_bsdf_kind_from_name(const char* name);
const char* khp_bsdf_name(int kind);
int khp_shader_kind_from_name(const char* name);

/* Camera::applyParameters (Camera.cpp:6-37) for a camera at `position`
 * looking along `look_at` (a direction, KIRK m_local_look_at) with `up`;
 * sensor size and focal length in metres (KIRK defaults 0.036x0.024, 0.0415). */
khp_status khp_camera_setup(const float position[3], const float look_at[3], const float up[3],
                            float sensor_w, float sensor_h, float focal_length,
                            uint32_t width, uint32_t height, khp_camera* out);

/* ABI 13: replaces the scene's camera without rebuilding anything (KIRK's GUI
 * moves the Camera between PathTracer::render calls and resets the pass
 * count, after which render() restarts its buffers, CPU_PathTracer.cpp:17-19).
 * Completes in-flight frames first; the next render uses the new camera.
 * Drops render-ahead work. */
khp_status khp_set_camera(khp_ctx* ctx, const khp_camera* camera);

/* Fur fibers -> cone frusta exactly as CPU_Scene::flattenNode does with
 * m_fiberAsCylinder (CPU_Scene.cpp:121-144): base pulled back by 0.8 % of the
 * segment, base radius shrunk 5 % (segment index <= 3) or 10 %.
 * positions [n_fibers][verts][3], radii [n_fibers][verts];
 * out arrays [n_fibers*(verts-1)][4]. */
khp_status khp_fibers_to_cones(uint32_t n_fibers, uint32_t verts_per_fiber,
                               const float* positions, const float* radii,
                               float* out_base_r0, float* out_apex_r1);

/* Fur fibers -> triangle tubes exactly as CPU_Scene::fiberToTriangles
 * (CPU_Scene.cpp:232-345, identity mesh transform), the flatten path KIRK
 * takes with m_fiberAsCylinder = false: per segment a (res+1)^2 vertex grid
 * and 2 res^2 triangles, each carrying the segment's frame.
 * out_v / out_n / out_frame: [n_fibers*(verts-1)*2*res*res][3][3]. */
khp_status khp_fibers_to_triangles(uint32_t n_fibers, uint32_t verts_per_fiber, const float* positions,
                                   const float* radii, uint32_t resolution, float* out_v, float* out_n,
                                   float* out_frame);

/* Seeded synthetic inputs (stand-ins for SceneGraph + Mesh::addFurToFaces,
 * Mesh.cpp:82-148).  Bit-reproducible on any host.
 * hairball: roots uniform on a sphere, strands of `verts` vertices following
 * the addFurToFaces recurrence in the root's tangent frame.
 * positions [n][verts][3], radii [n][verts]. */
khp_status khp_gen_hairball(uint32_t n_strands, uint32_t verts, const float center[3],
                            float ball_radius, float root_radius, uint32_t seed,
                            float* positions, float* radii);
/* icosphere with `subdiv` subdivisions: 20*4^subdiv triangles (tri_v/tri_n as khp_scene). */
khp_status khp_gen_icosphere(uint32_t subdiv, const float center[3], float radius,
                             float* tri_v, float* tri_n);
/* torus grid nu x nv quads -> 2*nu*nv triangles. */
khp_status khp_gen_torus(uint32_t nu, uint32_t nv, const float center[3], float major_r,
                         float minor_r, float* tri_v, float* tri_n);

#ifdef __cplusplus
}
#endif

#endif /* KIRK_HIP_H */
