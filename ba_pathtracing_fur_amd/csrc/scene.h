// scene.h -- host-side scene model of the core: the state KIRK's Triangle and
// Cylinder constructors derive (flatten), the binned-SAH BVH, and the device
// record layouts the kernels read.  Host only (g++), shared by render.hip.
#pragma once

#include <stdint.h>

#include <string>
#include <vector>

#include "../../include/kirk_hip.h"
#include "kmath.h"

namespace khp {

// ---- device record layouts (64 B per primitive, 64 B per interior node) ----
// cone   : (base.xyz, r0) (u.xyz, slope) (v.xyz, min_d) (w.xyz, max_d)
// triangle: (A.xyz, TRI_TAG) (ab.xyz, 0) (ac.xyz, 0) (0,0,0,0)
constexpr uint32_t TRI_TAG = 0x7fc0deadu;
// aux per slot: (base_d, material, object id, flags); flags bit 0 = cone,
// bits 8..31 = candidate count of the leaf that starts at this slot (0 otherwise).
struct Aux {
    float base_d;
    uint32_t mat;
    uint32_t obj;
    uint32_t flags;
};
// packed child/stack reference: interior node index, or LEAF_BIT | count << 24 | first slot
// (count 127 = escape: read the count from Aux::flags of the first slot).
constexpr uint32_t LEAF_BIT = 0x80000000u;
constexpr uint32_t LEAF_CNT_ESC = 127u;
constexpr uint32_t MAX_SLOTS = 1u << 24;
// interior node: (L.min.xyz, L.max.x) (L.max.yz, R.min.xy) (R.min.z, R.max.xyz) (Lref, Rref, Lcnt, Rcnt)
// ref = packed reference (LEAF_BIT ...); cnt = leaf candidate count or 0 for an interior child.
struct DevNode {
    float a[4], b[4], c[4];
    int32_t ref[2], cnt[2];
};
static_assert(sizeof(DevNode) == 64, "node must be one 64 B record");

// light state derived by the KIRK light ctors + Light::transform
struct DevLight {
    int32_t kind;
    float color[3];
    float position[3];
    float direction[3];
    float radius, c, l, q, inner, outer;
    float vert[4][3];
};

// ABI 6 textures: one entry per khp_texture, texels packed into one byte pool
struct DevTexture {
    uint32_t w, h, ch, wrap;
    uint64_t off;   // byte offset of texel (0, 0) in the pool
};
// per material: texture of diffuse, specular, volume, emission, roughness (-1: value)
struct DevMatTex {
    int32_t t[5];
};
enum : int { MT_DIFFUSE = 0, MT_SPECULAR = 1, MT_VOLUME = 2, MT_EMISSION = 3, MT_ROUGHNESS = 4 };

struct BuildNode {
    v3 mn, mx;
    int32_t left, right, first, count;
};

struct HostScene {
    uint32_t n_tris = 0, n_cones = 0, n_obj = 0;
    // per object (object id order)
    std::vector<float> rec;        // n_obj * 16
    std::vector<Aux> aux;          // n_obj
    std::vector<float> bounds;     // n_obj * 6
    std::vector<float> centroid;   // n_obj * 3
    std::vector<float> tri_nrm;    // n_tris * 9 (na, nb, nc after ctor reordering)
    std::vector<float> tri_frame;  // n_tris * 9 (hair frame u, v, w; fiberToTriangles) or zeros
    // ABI 6 textures (empty when the scene has none)
    std::vector<float> tri_uv;     // n_tris * 6 (tca, tcb, tcc after the ctor's reordering)
    std::vector<float> cone_h;     // n_cones (Cylinder::m_height, pre-transform)
    std::vector<DevTexture> tex;
    std::vector<uint8_t> texels;
    std::vector<DevMatTex> mtex;   // n_materials
    khp_env_map env_map{};
    bool textured = false;         // any textured material parameter or environment map
    // ABI 6 cone node transforms: per model M (16) then mat3(transpose(inverse(M))) (9)
    std::vector<float> models;
    std::vector<khp_material> mats;
    std::vector<DevLight> lights;
    khp_environment env{};
    khp_camera cam{};
    // BVH
    std::vector<BuildNode> nodes;  // DFS preorder
    std::vector<uint32_t> ids;     // leaf-ordered object ids (slot -> object)
    uint32_t depth = 0, max_leaf = 0;
    // device layout
    std::vector<DevNode> dnodes;   // interior nodes
    std::vector<float> slot_rec;   // n_obj * 16, slot order
    std::vector<Aux> slot_aux;     // slot order
    uint32_t n_slots = 0;          // >= n_obj: 2-candidate leaves start at even slots
    int32_t root_ref = 0, root_cnt = 0;   // root_ref packed
    float root_box[6] = {0, 0, 0, 0, 0, 0};
};

// Returns an error string (empty on success).
// objects=false: validate and keep materials/lights/env/camera only (the
// device flattens the objects).
std::string flatten_scene(const khp_scene* s, HostScene& hs, bool objects = true);
// Validates and copies the scene's textures / material texture indices /
// environment map into hs (both flatten paths); empty string on success.
std::string scene_textures(const khp_scene* s, HostScene& hs);
// Per-model M and inverse-transpose table (both flatten paths).
std::string scene_models(const khp_scene* s, HostScene& hs);
void build_bvh(HostScene& hs, int n_threads);
void make_device_layout(HostScene& hs);
void light_init(DevLight& L, const khp_light& in);

// The pixels (y*W + x) of the T x T tiles with id % nranks == rank, tile by
// tile, each tile as 8x8 blocks of 64 pixels (the wavefront's path order).
void owned_pixels(uint32_t W, uint32_t H, uint32_t T, uint32_t rank, uint32_t nranks, std::vector<uint32_t>& out);
// The framebuffer gather as seen from `rank` (khp_gather_plan in kirk_hip.h):
// counts[r] = pixels rank r sends to root in this rank's view, `flat` = their
// lists concatenated in rank order.  Empty string on success.
std::string gather_plan(uint32_t W, uint32_t H, uint32_t T, int nranks, int rank, int root,
                        std::vector<uint64_t>& counts, std::vector<uint32_t>& flat);

// Per-thread message behind khp_last_error(); every failing entry point sets it.
khp_status fail(khp_status s, const std::string& msg);
// tonemap_host.cpp: KIRK's sequential float running sum s <- (float)((double)s + l[k])
// over n terms, continued from s (RGB_to_Yxy's log-luminance sum), bit for bit.
float log_sum_feed(float s, const double* l, size_t n);
const char* last_error();

}  // namespace khp
