// device_build.h -- device-side acceleration-structure build (bvh_build.hip),
// shared by render.hip.  hipcc only.
#pragma once

#include <hip/hip_runtime.h>

#include <string>

#include "scene.h"

namespace khp {

// One owned device allocation (grows, never shrinks).
struct DevMem {
    void* p = nullptr;
    size_t bytes = 0;
    DevMem() = default;
    DevMem(const DevMem&) = delete;
    DevMem& operator=(const DevMem&) = delete;
    ~DevMem() {
        if (p) (void)hipFree(p);
    }
    hipError_t ensure(size_t n) {
        if (n <= bytes && p) return hipSuccess;
        if (p) (void)hipFree(p);
        p = nullptr;
        bytes = 0;
        hipError_t e = hipMalloc(&p, n ? n : 16);
        if (e == hipSuccess) bytes = n;
        return e;
    }
    void release() {
        if (p) (void)hipFree(p);
        p = nullptr;
        bytes = 0;
    }
    template <typename T>
    T* as() const { return (T*)p; }
};

// Per-object state of the flattened scene in HBM (object-id order): the same
// arrays HostScene holds on the host path.
struct DeviceObjects {
    DevMem rec;       // float4[4 * n_obj]: the 64-B intersection record
    DevMem aux;       // Aux[n_obj]
    DevMem bounds;    // float[6 * n_obj]
    DevMem centroid;  // float[3 * n_obj]
    DevMem tri_nrm;   // float[9 * n_tris]
    DevMem tri_frame; // float[9 * n_tris] hair frame (zeros unless fiberToTriangles)
    DevMem tri_uv;    // float[6 * n_tris] texcoords after the ctor's reordering (textured scenes)
    DevMem cone_h;    // float[n_cones] Cylinder::m_height (textured scenes)
    uint32_t n_obj = 0, n_tris = 0, n_cones = 0;
    void release() {
        rec.release();
        aux.release();
        bounds.release();
        centroid.release();
        tri_nrm.release();
        tri_frame.release();
        tri_uv.release();
        cone_h.release();
        n_obj = n_tris = n_cones = 0;
    }
};

// The BVH as the device build leaves it in HBM.
struct DeviceTree {
    DevMem nodes;  // BuildNode[n_nodes], DFS preorder (the host builder's layout)
    DevMem ids;    // uint32[n_obj], leaf-ordered object ids
    DevMem P;      // uint32[n_obj + 1], leaves starting before each position
    uint32_t n_nodes = 0, n_leaves = 0;
    void release() {
        nodes.release();
        ids.release();
        P.release();
        n_nodes = n_leaves = 0;
    }
};

struct DeviceLayout {
    uint32_t n_dnodes = 0, n_slots = 0;
    int32_t root_ref = 0, root_cnt = 0;
    float root_box[6] = {0, 0, 0, 0, 0, 0};
};

// CPU::Scene::flattenNode per-object state on the device (flatten.hip).
// device_ptrs: the scene's geometry arrays are device pointers (else host,
// copied).  Errors starting "EINVAL:" are input errors.
// textured: also write tri_uv / cone_h; models: HostScene::models (25 floats per model) or empty.
std::string device_flatten(const khp_scene* s, bool device_ptrs, uint32_t n_materials, bool textured,
                           const std::vector<float>& models, DeviceObjects& o,
                           hipStream_t st, double* kernel_ms);

// khp_gen_hairball + khp_fibers_to_cones on the device, into device arrays of
// n * (verts - 1) float4 each.
std::string device_gen_hairball(uint32_t n, uint32_t verts, const float center[3], float ball_r, float root_r,
                                uint32_t seed, float* d_base_r0, float* d_apex_r1, hipStream_t st);

// khp_gen_hairball followed by khp_fibers_to_triangles, on the device.
std::string device_gen_hairball_tris(uint32_t n, uint32_t verts, const float center[3], float ball_r, float root_r,
                                     uint32_t seed, uint32_t res, float* d_v, float* d_n, float* d_frame,
                                     hipStream_t st);

// BVH::addBaseDataStructure on the device from o.centroid / o.bounds: the host
// builder's tree (build_bvh), node for node.  Sets hs.depth / hs.max_leaf.
std::string device_build_bvh(HostScene& hs, const DeviceObjects& o, hipStream_t st, DeviceTree& t,
                             double* kernel_ms);

// make_device_layout on the device: interior records in pair order, leaf slots,
// and the slot-ordered primitive records gathered from o.rec / o.aux.
std::string device_layout(const DeviceObjects& o, DeviceTree& t, hipStream_t st, DevMem& dnodes, DevMem& prims,
                          DevMem& aux, DeviceLayout& out, double* kernel_ms);

// Copy the device tree into hs.nodes / hs.ids (introspection).
std::string download_tree(const DeviceTree& t, HostScene& hs, hipStream_t st);

}  // namespace khp
